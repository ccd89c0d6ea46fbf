"""Probe: per-conv comparison of the deferred WGRAD reduction (the engine's own per-unit partial buffer, one
wgrad_reduce_multi launch after the backward) against an immediate reduction of the same operands at the moment the
WGRAD ran (large private workspace).  Prints, for every conv whose gradients differ, the two reduction descriptors
(split counts, kinds) and the size of the difference.

    python tools/probes/wred_defer_probe.py [model]
"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import torch  # noqa: E402

from fedmi.engine.base import TrainerConfig  # noqa: E402
from fedmi.engine.cnn_native import CNNNativeTrainer  # noqa: E402
from fedmi.engine.data import make_dataset  # noqa: E402
from fedmi.models import build_model  # noqa: E402
from fedmi.ops import conv  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "GoogLeNet"
    dev = torch.device("cuda:0")
    data = make_dataset("synthetic-cifar10", device=dev, n_train=256, n_test=64, seed=0)
    tr = CNNNativeTrainer(name, data, dev, TrainerConfig(batch_size=128, augment=False, use_graph=False),
                          init_state=build_model(name).state_dict())
    names = {p.grad.data_ptr(): k for k, p in tr.model.named_parameters() if p.grad is not None}
    big = torch.empty(64 << 20, device=dev)
    checks = []
    orig_c, orig_d = conv.conv2d_wgrad, conv.dwconv_wgrad

    def wrap_c(x, dy, R, S, stride, pad, Cw=None, out=None, deferred=None, ws=None, **kw):
        ref = torch.empty_like(out)
        orig_c(x, dy, R, S, stride, pad, Cw=Cw, out=ref, ws=big, deferred=(lst := []), **kw)
        conv.wgrad_reduce_multi(lst, dev)
        n0 = len(deferred) if deferred is not None else 0
        r = orig_c(x, dy, R, S, stride, pad, Cw=Cw, out=out, deferred=deferred, ws=ws, **kw)
        mine = deferred[n0] if deferred is not None and len(deferred) > n0 else None
        checks.append((out, ref, lst[0] if lst else None, mine, tuple(x.shape), tuple(dy.shape), ws.numel()))
        return r

    def wrap_d(x, dy, R, stride, pad, out=None, deferred=None, ws=None, **kw):
        ref = torch.empty_like(out)
        orig_d(x, dy, R, stride, pad, out=ref, ws=big, deferred=(lst := []), **kw)
        conv.wgrad_reduce_multi(lst, dev)
        n0 = len(deferred) if deferred is not None else 0
        r = orig_d(x, dy, R, stride, pad, out=out, deferred=deferred, ws=ws, **kw)
        mine = deferred[n0] if deferred is not None and len(deferred) > n0 else None
        checks.append((out, ref, lst[0] if lst else None, mine, tuple(x.shape), tuple(dy.shape), ws.numel()))
        return r

    conv.conv2d_wgrad, conv.dwconv_wgrad = wrap_c, wrap_d
    try:
        for start, nb in ((0, 128), (128, 80)):
            checks.clear()
            tr.grads_for_batch(start, nb)
            torch.cuda.synchronize()
            bad = 0
            for out, ref, it_ref, it_mine, xs, ys, cap in checks:
                if not torch.equal(out, ref):
                    bad += 1
                    d = (out - ref).abs()
                    print(json.dumps({"nb": nb, "param": names.get(out.data_ptr(), "?"), "x": xs, "dy": ys, "cap": cap,
                                      "ref_item": it_ref[2:] if it_ref else None,
                                      "deferred_item": it_mine[2:] if it_mine else None,
                                      "max_abs": float(d.max()), "ref_max": float(ref.abs().max()),
                                      "n_diff": int((d > 0).sum())}), flush=True)
            print(json.dumps({"nb": nb, "convs": len(checks), "differ": bad}), flush=True)
    finally:
        conv.conv2d_wgrad, conv.dwconv_wgrad = orig_c, orig_d


if __name__ == "__main__":
    main()
