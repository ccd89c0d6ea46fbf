bash tools/gpu_r6_d.sh && bash tools/gpu_r6_c.sh
