"""The product path on one GPU (coordinator + N GPU client processes over gRPC, peer or dist data plane):
  [DIAG_CLIENTS=n] [FEDMI_DEBUG_STATS=1] python tools/diag_system_topk.py <transport peer|dist> <compress Y|N>
      [extra client args...]
Prints the coordinator's round log and the tail of each client log; FEDMI_DEBUG_STATS=1 makes each client log
its LeNet stats rows after every phase of a round.  Used to localise the train-stats corruption of
tests/test_system_gpu.py (a graph-captured hipMemsetAsync replaying stale host bytes, fixed in the engine)."""
import sys
import tempfile
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "tests"))
from helpers import free_port, spawn_client, stop_proc, wait_heartbeat  # noqa: E402

from fedmi.control.coordinator import Coordinator, CoordinatorConfig  # noqa: E402

transport, compress = sys.argv[1], sys.argv[2] == "Y"
extra = tuple(sys.argv[3:])
tmp = Path(tempfile.mkdtemp(prefix="diag_sys_"))
addrs = [f"127.0.0.1:{free_port()}" for _ in range(int(__import__("os").environ.get("DIAG_CLIENTS", "2")))]
args = ("--agg", "collective", "--model", "lenet", "--n-train", "2560", "--n-test", "1000", "--transport", transport)
args += (("-c", "Y") if compress else ()) + extra
procs = [spawn_client(a, tmp, *args, log_path=tmp / f"client{i}.log", device="cuda:0") for i, a in enumerate(addrs)]
try:
    for a in addrs:
        wait_heartbeat(a, timeout=100)
    cfg = CoordinatorConfig(clients=addrs, rounds=3, agg="collective", root=str(tmp / "srv"), gzip=compress,
                            train_timeout_s=90, rpc_timeout_s=20, heartbeat_s=0.5)
    coord = Coordinator(cfg)
    coord.run()
    coord.close()
    print("RESULT round", coord.round, flush=True)
finally:
    for p in procs:
        stop_proc(p)
for i in range(len(addrs)):
    lines = (tmp / f"client{i}.log").read_text().splitlines()
    print(f"--- client{i} log tail ---")
    print("\n".join(lines[-int(__import__("os").environ.get("DIAG_TAIL", "25")):]))
