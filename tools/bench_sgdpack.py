"""Time the CNN engine's step tail: fused SGD + weight images (conv.SgdPack) vs sgd_flat + pack launches.

    python tools/bench_sgdpack.py [--models ResNet18 MobileNet] [--iters 200] [--cold]

Prints one JSON line per model: microseconds per tail, both paths (HIP-graph replay of `iters` tails).
--cold: every tail follows a 1 GiB streaming pass that evicts the 256 MB last-level cache (as in a real
step, where the weights are cold after the forward / backward pass); the pass alone is timed and subtracted.
"""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from fedmi.engine.base import TrainerConfig  # noqa: E402
from fedmi.engine.cnn_native import CNNNativeTrainer  # noqa: E402
from fedmi.engine.data import make_dataset  # noqa: E402


def _time(fn, iters: int) -> float:
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
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


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", nargs="+", default=["ResNet18", "MobileNet"])
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--cold", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    flush = torch.zeros(1 << 28, device=dev) if a.cold else None   # 1 GiB

    def with_flush(fn):
        def run():
            flush.add_(1.0)
            fn()
        return run

    t_flush = _time(lambda: flush.add_(1.0), a.iters) if a.cold else 0.0
    data = make_dataset("synthetic-cifar10", device=dev, n_train=256, n_test=64, seed=0)
    for name in a.models:
        tr = CNNNativeTrainer(name, data, dev, TrainerConfig(batch_size=128, augment=False, use_graph=False,
                                                             lr=1e-6))
        fused = tr._sgdpack
        step = with_flush(tr._sgd) if a.cold else tr._sgd
        us_fused = _time(step, a.iters) - t_flush
        tr._sgdpack = None
        us_unfused = _time(step, a.iters) - t_flush
        tr._sgdpack = fused
        print(json.dumps({"model": name, "params": tr.fs.n_params, "convs": fused.n_convs,
                          "workgroups": fused.n_blocks, "tail_us_fused": round(us_fused, 2),
                          "tail_us_unfused": round(us_unfused, 2), "cold": a.cold,
                          "flush_us": round(t_flush, 2)}), flush=True)


if __name__ == "__main__":
    main()
