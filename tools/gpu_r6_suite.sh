# round 6: the whole GPU suite + smoke (one call)
bash tools/gpu_steps.sh ${1:-r6_suite} \
  suite 1080 "env FEDMI_FAILOVER_REPORT=gpurun_out/${1:-r6_suite}/drills.jsonl python -u -m pytest tests -m gpu -q --timeout 420 --timeout-method thread -p no:cacheprovider --durations=25" \
  smoke 120 "python -c 'import __graft_entry__ as g; g.smoke()'"
