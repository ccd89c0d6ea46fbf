"""Verify-and-select of the FedAvg data plane: hand-written hipIpc peer kernels vs RCCL.

Used by bench.py and by the product client (``GroupManager(transport="auto")``) at the first
data-plane generation.  The peer kernels (csrc/comm/peer_comm.hip) are checked against the
reference collective of the already-formed process group on random data -- every rank must
agree -- then each candidate is timed on a buffer the size of the model's flat state and the
fastest verified one is kept.  RCCL is a candidate only when the group is ``nccl`` (one rank
per GPU); ranks sharing a GPU (one-GPU rehearsals) verify against gloo and keep the peer
kernel.  The reference's data plane is a gRPC gather + CPU average (src/server.py:120-179).
"""
from __future__ import annotations

from typing import Dict, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


def timed_ms(fn, iters: int, device: torch.device, group=None) -> float:
    """ms per call (device time from events), MAX over the ranks of ``group``."""
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize(device)
    t = torch.tensor([e0.elapsed_time(e1) / iters], dtype=torch.float64)
    if dist.get_backend(group) == "nccl":
        t = t.to(device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def _all_true(flag: bool, device: torch.device, group=None) -> bool:
    on_gpu = dist.get_backend(group) == "nccl"
    t = torch.tensor([1.0 if flag else 0.0], device=device if on_gpu else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item() >= 1)


def verify_and_select(peer, numel: int, device: torch.device, group=None,
                      algos: Sequence[str] = ("oneshot", "twoshot"), iters: int = 20,
                      seed: int = 1234, compare_group: bool = True) -> Tuple[Optional[str], Dict]:
    """Returns (choice, info): choice is a peer algo name, or ``None`` for the process group's
    own all-reduce (RCCL).  Collective over ``group``; every rank returns the same choice.
    ``compare_group=False``: the peer kernel is only verified (an explicitly requested algo).
    Raises if no candidate verified and the group cannot carry FedAvg itself (gloo on GPUs
    sharing one device is a reference only, never the data plane of a GPU run)."""
    backend = dist.get_backend(group)
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    rccl = backend == "nccl"
    g = torch.Generator(device=device).manual_seed(seed + rank)
    probe = torch.randn(numel, generator=g, device=device)
    if rccl:
        ref = probe.clone()
        dist.all_reduce(ref, op=dist.ReduceOp.AVG, group=group)
    else:
        ref_h = probe.cpu()
        dist.all_reduce(ref_h, group=group)
        ref = (ref_h / world).to(device)
    info: Dict = {"verified_against": "rccl" if rccl else backend}
    times: Dict[str, float] = {}
    for algo in algos:
        peer.algo = algo
        got = probe.clone()
        peer.allreduce_mean_(got)
        good = bool(torch.allclose(got, ref, rtol=1e-5, atol=1e-6)) and peer.error() == 0
        ok = _all_true(good, device, group)
        info[f"{algo}_verified"] = ok
        if ok:
            buf = probe.clone()
            times[algo] = timed_ms(lambda: peer.allreduce_mean_(buf), iters, device, group)
    if rccl and compare_group:
        buf = probe.clone()
        times["rccl"] = timed_ms(lambda: dist.all_reduce(buf, op=dist.ReduceOp.AVG, group=group), iters,
                                 device, group)
    info["ms"] = {k: round(v, 5) for k, v in times.items()}
    peer_times = {a: t for a, t in times.items() if a != "rccl"}
    if not peer_times:
        if not rccl:
            raise RuntimeError(f"peer all-reduce failed verification against {backend}: {info}")
        info["chosen"] = "rccl"
        return None, info
    best = min(peer_times, key=peer_times.get)
    if "rccl" in times and times["rccl"] < peer_times[best]:
        info["chosen"] = "rccl"
        return None, info
    peer.algo = best
    info["chosen"] = best
    return best, info
