"""Channels-last row reductions (zoo_ops.hip reduce_rows_kernel) at zoo BN shapes: the plain two-launch form
(row slabs + reduce_rows_finalize) against the one-launch form whose last-arriving workgroup sums the slabs.
Run under ``rocprofv3 --kernel-trace --stats`` for per-kernel times; prints CUDA-event ms per call.

    python tools/bench_rows.py [M:C ...]
"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

from fedmi import native  # noqa: E402

PER_LANE = [int(v) for v in sys.argv[1].split("=")[1].split(",")] if len(sys.argv) > 1 and sys.argv[1].startswith(
    "--per-lane=") else [0]
ARGS = sys.argv[2:] if PER_LANE != [0] else sys.argv[1:]
SHAPES = [tuple(int(v) for v in s.split(":")) for s in ARGS] or [
    (131072, 48), (131072, 96), (32768, 192), (8192, 384), (8192, 1024), (2048, 2432), (2048, 512)]
nat = native.require()
dev = torch.device("cuda", 0)
st = native.stream_handle(dev)
for pl in PER_LANE:
  if pl:
    nat.z_rows_tune(pl)
  for M, C in SHAPES:
      x = torch.randn(M, C, device=dev).to(torch.bfloat16)
      part = torch.empty(int(nat.z_reduce_rows_ws_floats(M, C)), device=dev)
      acc = torch.zeros(2 * C, device=dev)
      out = torch.empty(C, device=dev)
      ref = x.float().sum(0)
      res = {}
      for mode in ("two_launch", "last_arriver"):
          def call():
              if mode == "two_launch":
                  nat.z_reduce_rows(st, x.data_ptr(), 1, C, 0, 0, 0, 0, C, M, 0, part.data_ptr(), part.numel(),
                                    acc.data_ptr(), 0)
              else:
                  nat.z_reduce_rows(st, x.data_ptr(), 1, C, 0, 0, 0, 0, C, M, 0, part.data_ptr(), part.numel(),
                                    0, 0, out=out.data_ptr(), out_dt=0, scale=1.0)
          acc.zero_()
          call()
          torch.cuda.synchronize()
          got = acc[:C] if mode == "two_launch" else out
          err = float((got - ref).abs().max() / ref.abs().max())
          n = 50
          e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
          e0.record()
          for _ in range(n):
              call()
          e1.record()
          torch.cuda.synchronize()
          res[mode] = {"us": round(e0.elapsed_time(e1) / n * 1e3, 2), "rel_err": err}
      print(json.dumps({"per_lane": pl or 16, "M": M, "C": C, "MB": round(M * C * 2 / 2**20, 2), "slabs_ws_floats": part.numel(), **res}),
            flush=True)
