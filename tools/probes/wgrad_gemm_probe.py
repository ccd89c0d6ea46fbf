"""Probe: weight gradient of a 3x3 / stride-1 conv as im2col + library GEMM (bf16 in, fp32 out) vs conv2d_wgrad.

    python tools/probes/wgrad_gemm_probe.py

For each shape prints µs of: conv2d_wgrad (native split-K + reduce), im2col (torch pad + stack), the GEMM
(torch.mm with out_dtype=float32 -> hipBLASLt / rocBLAS), and the relative error of the GEMM result vs native.
"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from fedmi.ops import conv  # noqa: E402


def timed(fn, iters=50):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


def main():
    dev = torch.device("cuda:0")
    for N, H, C, O in [(128, 4, 512, 512), (128, 8, 256, 256), (128, 16, 128, 128), (128, 32, 64, 64)]:
        x = torch.randn(N, H, H, C, device=dev).bfloat16()
        dy = torch.randn(N, H, H, O, device=dev).bfloat16()
        shp = (x.shape, O, 3, 3, 1, 1, C)
        ws = torch.empty(max(conv.wgrad_ws_floats(*shp), 1), device=dev)
        dw = torch.empty(O, C, 3, 3, device=dev)
        cols = torch.empty(N * H * H, C, 9, dtype=torch.bfloat16, device=dev)

        def native():
            conv.conv2d_wgrad(x, dy, 3, 3, 1, 1, Cw=C, out=dw, ws=ws)

        def im2col():
            xp = F.pad(x, (0, 0, 1, 1, 1, 1))
            torch.stack([xp[:, r:r + H, s:s + H, :] for r in range(3) for s in range(3)], dim=-1,
                        out=cols.view(N, H, H, C, 9))

        res = {}

        def gemm():
            res["dw"] = torch.mm(dy.view(-1, O).t(), cols.view(-1, C * 9), out_dtype=torch.float32)

        t_nat = timed(native)
        t_col = timed(im2col)
        try:
            t_mm = timed(gemm)
            native()
            gemm()
            torch.cuda.synchronize()
            err = float((res["dw"].view(O, C, 3, 3) - dw).norm() / dw.norm())
        except Exception as e:  # noqa: BLE001
            t_mm, err = None, repr(e)[:200]
        print(json.dumps({"N": N, "H": H, "C": C, "O": O, "native_us": round(t_nat, 2), "im2col_us": round(t_col, 2),
                          "gemm_us": t_mm if t_mm is None else round(t_mm, 2), "rel_err": err,
                          "gemm_tflops": None if not t_mm else round(2 * O * C * 9 * N * H * H / t_mm / 1e6, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
