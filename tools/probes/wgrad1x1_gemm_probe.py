"""Probe: weight gradient of a 1x1 / stride-1 conv (NHWC bf16) -- a plain GEMM dW[O][C] = dY^T X over the pixels --
as the native split-K WGRAD (conv_igemm<WGRAD> + reduce) vs the library GEMM (torch.mm, bf16 in, fp32 out ->
hipBLASLt / rocBLAS), at the MobileNet pointwise shapes (batch 128).  Graph-replayed; prints µs, relative error vs
native, and whether two library runs are bit-identical.

    python tools/probes/wgrad1x1_gemm_probe.py
"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import torch  # noqa: E402

from fedmi.ops import conv  # noqa: E402
from wgrad_gemm_probe import timed  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    for N, H, C, O in [(128, 32, 32, 64), (128, 16, 64, 128), (128, 16, 128, 128), (128, 8, 128, 256),
                       (128, 8, 256, 256), (128, 4, 256, 512), (128, 4, 512, 512), (128, 2, 512, 1024),
                       (128, 2, 1024, 1024)]:
        x = torch.randn(N, H, H, C, device=dev).bfloat16()
        dy = torch.randn(N, H, H, O, device=dev).bfloat16()
        shp = (x.shape, O, 1, 1, 1, 0, C)
        ws = torch.empty(max(conv.wgrad_ws_floats(*shp), 1), device=dev)
        dw = torch.empty(O, C, 1, 1, device=dev)
        out = torch.empty(O, C, device=dev)

        def native():
            conv.conv2d_wgrad(x, dy, 1, 1, 1, 0, Cw=C, out=dw, ws=ws)

        def gemm():
            torch.mm(dy.view(-1, O).t(), x.view(-1, C), out_dtype=torch.float32, out=out)

        t_nat = timed(native)
        try:
            t_mm = timed(gemm)
            native()
            gemm()
            torch.cuda.synchronize()
            a = out.clone()
            gemm()
            torch.cuda.synchronize()
            err = float((out - dw.view(O, C)).norm() / dw.norm())
            bitstable = bool(torch.equal(a, out))
        except Exception as e:  # noqa: BLE001
            t_mm, err, bitstable = None, repr(e)[:200], None
        print(json.dumps({"N": N, "H": H, "C": C, "O": O, "native_us": round(t_nat, 2),
                          "gemm_us": t_mm if t_mm is None else round(t_mm, 2), "rel_err": err,
                          "gemm_bitstable": bitstable}), flush=True)


if __name__ == "__main__":
    main()
