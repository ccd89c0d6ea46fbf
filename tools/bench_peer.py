#!/usr/bin/env python
"""Microbenchmark of the hipIpc peer all-reduce (csrc/comm/peer_comm.hip).

W processes on the visible GPUs (rank r on cuda:r % ngpu; on a one-GPU box all
ranks share cuda:0, which measures the kernels' barrier + copy cost, not xGMI).
Payloads: the LeNet flat state (62,006 fp32 = 248 KB) and the ResNet-18 flat
state (11.17 M fp32 = 44.7 MB).  Prints one JSON line per (world, algo, size).

  python tools/bench_peer.py --world 2 4 --iters 200
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
from pathlib import Path

import torch
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

SIZES = {"lenet": 62006, "resnet18": 11173962}


def _worker(rank, world, path, iters, q):
    import torch.distributed as dist

    from fedmi.parallel.peer import PeerAllReduce

    ngpu = torch.cuda.device_count()
    dev = torch.device("cuda", rank % ngpu)
    torch.cuda.set_device(dev)
    store = dist.FileStore(path, world)
    pc = PeerAllReduce(rank, world, 4 * max(SIZES.values()) + 4096, store, tag="bench", device=dev)
    pc.comm.set_timeout_ms(float(os.environ.get("FEDMI_BENCH_PEER_TIMEOUT_MS", "30000")))
    res = []
    for name, n in SIZES.items():
        x = torch.randn(n, device=dev)
        for algo in ("oneshot", "twoshot"):
            pc.algo = algo
            it = iters if n < 1_000_000 else max(10, iters // 10)
            for _ in range(5):
                pc.allreduce_mean_(x)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(it):
                pc.allreduce_mean_(x)
            e1.record()
            torch.cuda.synchronize()
            res.append((name, algo, n, e0.elapsed_time(e1) * 1e3 / it))
        # -c Y int8 + error feedback: the fused one-launch collective vs the unfused chain (delta, quantise, two
        # all-gathers, dequantise-accumulate), same data
        from fedmi.parallel.compress import Int8Compressor

        class _F:
            def __init__(self, t):
                self.t = t

            def float_state(self):
                return self.t

        for fused in (True, False):
            xs = x.clone()
            comp = Int8Compressor(_F(xs))
            comp.fused = fused
            it = iters if n < 1_000_000 else max(10, iters // 10)
            for _ in range(5):
                comp.aggregate(_F(xs), transport=pc)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(it):
                comp.aggregate(_F(xs), transport=pc)
            e1.record()
            torch.cuda.synchronize()
            res.append((name, "int8_fused" if fused else "int8_unfused", n, e0.elapsed_time(e1) * 1e3 / it))
    err = pc.error()
    pc.close()
    q.put((rank, res, err))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, nargs="+", default=[2, 4])
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--out", default=None)
    ap.add_argument("--no-gate", action="store_true",
                    help="ranks sharing a GPU skip the host gate before each collective (FEDMI_PEER_GATE=0): the "
                         "kernels' own barrier + copy cost, the round-2 measurement; a 2 s barrier timeout bounds "
                         "a peer whose kernel is not co-scheduled")
    a = ap.parse_args()
    if a.no_gate:
        os.environ["FEDMI_PEER_GATE"] = "0"
        os.environ["FEDMI_BENCH_PEER_TIMEOUT_MS"] = "2000"
    lines = []
    for world in a.world:
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        with tempfile.TemporaryDirectory() as td:
            path = os.path.join(td, "store")
            procs = [ctx.Process(target=_worker, args=(r, world, path, a.iters, q)) for r in range(world)]
            for p in procs:
                p.start()
            got = [q.get(timeout=600) for _ in procs]
            for p in procs:
                p.join(timeout=60)
        errs = [e for _, _, e in got]
        for i, (name, algo, n, _) in enumerate(got[0][1]):
            us = max(g[1][i][3] for g in got)
            rec = {"bench": "peer_allreduce", "world": world, "payload": name, "numel": n, "bytes": 4 * n,
                   "algo": algo, "us_per_call": round(us, 2), "alg_GBps": round(4 * n / us / 1e3, 2),
                   "gpus": torch.cuda.device_count(), "errors": errs, "host_gate": not a.no_gate}
            print(json.dumps(rec), flush=True)
            lines.append(rec)
    if a.out:
        Path(a.out).write_text("".join(json.dumps(r) + "\n" for r in lines))
    return 0


if __name__ == "__main__":
    sys.exit(main())
