"""Probe: one MobileNetV2 step's gradients (nb = 64, the gradient-tracking test's setup) with the small 1x1 WGRADs
on the library GEMM (conv.WGRAD_GEMM_PIXELS = 2048) vs the native kernels (= 0): which tensors differ, and is each
route bit-stable run to run.  Only the routed convs' weight gradients may differ.  (Round 6 ran it against a
since-reverted 512-pixel library threshold for halo-eligible shapes: profiles/r6_cnn/wgrad1x1_halo/small_shapes/.)

    python tools/probes/halo_lib_grad_diff.py [model]
"""
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
    name = sys.argv[1] if len(sys.argv) > 1 else "MobileNetV2"
    dev = torch.device("cuda:0")
    data = make_dataset("synthetic-cifar10", device=dev, n_train=128, n_test=64, seed=0)
    torch.manual_seed(0)
    init = build_model(name).state_dict()
    grads = {}
    for halo in (2048, 0, 0, 2048):
        conv.WGRAD_GEMM_PIXELS = halo
        tr = CNNNativeTrainer(name, data, dev, TrainerConfig(batch_size=64, augment=False, use_graph=False),
                              init_state=init)
        tr.grads_for_batch(0, 64)
        torch.cuda.synchronize()
        g = {k: p.grad.detach().float().clone() for k, p in tr.model.named_parameters()}
        if halo in grads:
            same = [k for k in g if not torch.equal(g[k], grads[halo][k])]
            print(f"halo={halo} rerun: {len(same)} tensors differ from the first run {same[:6]}", flush=True)
        else:
            grads[halo] = g
    a, b = grads[2048], grads[0]
    for k in a:
        if not torch.equal(a[k], b[k]):
            d = (a[k] - b[k]).abs().max().item()
            print(f"{k:40s} max|diff| {d:.3e}  max|g| {a[k].abs().max().item():.3e}", flush=True)


if __name__ == "__main__":
    main()
