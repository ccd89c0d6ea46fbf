#!/usr/bin/env python
"""-c Y kernel timings (csrc/kernels/compress.hip) at the LeNet and ResNet-18 state sizes.

For n = 62,006 (LeNet) and 11,173,962 (ResNet-18): device time of the
error-feedback delta + exact top-k (k = 1 % and 20 % of n, FEDMI_TOPK_RATIOS: the fused path ``topk_us``, and one
read+write pass over the state for scale ``rw_pass_us``), of the rank-ordered
scatter of 4 ranks' payloads, of int8 quantisation and of a 4-rank dequant
accumulate; plus payload bytes vs dense fp32.  One JSON line per size.
"""
from __future__ import annotations

import json
import os
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def _time(fn, iters):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main() -> int:
    from fedmi import native

    nat = native.require()
    dev = torch.device("cuda", 0)
    S = lambda: native.stream_handle(dev)   # noqa: E731
    out = []
    ratios = [float(v) for v in os.environ.get("FEDMI_TOPK_RATIOS", "0.01,0.2").split(",")]
    for (name, n), ratio in [(p, r) for p in (("lenet", 62006), ("resnet18", 11173962)) for r in ratios]:
        iters = 200 if n < 1e6 else 20
        k = max(1, int(round(n * ratio)))
        R = 4
        local = torch.randn(n, device=dev)
        glob = torch.randn(n, device=dev)
        resid = torch.zeros(n, device=dev)
        d = torch.empty(n, device=dev)
        idx = torch.empty(k, dtype=torch.int32, device=dev)
        val = torch.empty(k, device=dev)
        tstate = torch.zeros(nat.topk_state_bytes(), dtype=torch.uint8, device=dev)
        cidx = torch.empty(2 * n, dtype=torch.int32, device=dev)
        ckey = torch.empty(2 * n, dtype=torch.int32, device=dev)

        def topk_ef():
            nat.topk_ef(S(), local.data_ptr(), glob.data_ptr(), resid.data_ptr(), n, k, tstate.data_ptr(),
                        cidx.data_ptr(), ckey.data_ptr(), idx.data_ptr(), val.data_ptr())

        t_topk = _time(topk_ef, iters)
        # realistic rounds: a fresh update every call (the residual carries the unsent part forward)
        ups = [torch.randn(n, device=dev) * 0.01 for _ in range(4)]
        calls = [0]

        def topk_ef_fresh():
            local.copy_(glob).add_(ups[calls[0] % 4])
            calls[0] += 1
            topk_ef()

        resid.zero_()
        t_topk_fresh = _time(topk_ef_fresh, iters) - _time(lambda: local.copy_(glob).add_(ups[0]), iters)
        st_words = tstate.view(torch.int32).cpu()
        cand = int(st_words[2048 + 4])
        dense = torch.randn(n, device=dev)
        t_copy = _time(lambda: dense.mul_(1.0), iters)     # one read + write pass over the state
        idx_all = torch.stack([torch.randperm(n, device=dev)[:k].to(torch.int32) for _ in range(R)])
        val_all = torch.randn(R, k, device=dev)
        acc = torch.zeros(n, device=dev)
        t_scatter = _time(lambda: nat.scatter_add_ranked(S(), acc.data_ptr(), idx_all.data_ptr(), val_all.data_ptr(),
                                                          R, k, 1.0 / R, n), iters)
        nch = (n + 255) // 256
        q = torch.empty(n, dtype=torch.int8, device=dev)
        sc = torch.empty(nch, device=dev)
        t_q = _time(lambda: nat.quant_int8(S(), d.data_ptr(), n, q.data_ptr(), sc.data_ptr(), resid.data_ptr()), iters)
        q_all = q.repeat(R)
        s_all = sc.repeat(R)
        t_dq = _time(lambda: nat.dequant_accum(S(), q_all.data_ptr(), s_all.data_ptr(), R, n, acc.data_ptr(), 1.0 / R),
                     iters)
        rec = {"bench": "compress_kernels", "payload": name, "n": n, "k": k, "ratio": ratio,
               "topk_us": round(t_topk, 2), "topk_fresh_update_us": round(t_topk_fresh, 2), "candidates_last": cand,
               "rw_pass_us": round(t_copy, 2), "scatter_ranked_4rank_us": round(t_scatter, 2),
               "quant_int8_us": round(t_q, 2), "dequant_accum_4rank_us": round(t_dq, 2),
               "bytes_dense": 4 * n, "bytes_topk": 8 * k, "bytes_int8": n + 4 * nch,
               "ratio_topk": round(4 * n / (8 * k), 2), "ratio_int8": round(4 * n / (n + 4 * nch), 2)}
        print(json.dumps(rec), flush=True)
        out.append(rec)
    if len(sys.argv) > 1:
        Path(sys.argv[1]).write_text("".join(json.dumps(r) + "\n" for r in out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
