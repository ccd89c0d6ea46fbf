"""End-of-run FedAvg consistency guard.

After a synchronous FedAvg round every client must hold the SAME global model
(the reference gets this for free: one CPU average broadcast to everyone,
src/server.py:144-179).  fedmi's data plane averages in place on every client,
so a silently failed collective (a peer barrier that timed out and returned
early, a rank that skipped a round) would leave that client's model
un-averaged while the run still reports a throughput.

:func:`check_consistency` is the guard: every rank reports its transport error
flag and a blake2b digest of its flat model state (float + int entries); one
all-gather brings all of them to every rank.  The peer kernels and RCCL sum in
rank order / a fixed tree, so the digests are bit-identical on every rank when
the run was correct -- any difference is a real divergence, not rounding.
"""
from __future__ import annotations

import hashlib
from typing import Optional

import torch
import torch.distributed as dist


def model_digest(trainer) -> bytes:
    """16-byte blake2b of the bytes of the trainer's flat fp32 state and its integer buffers."""
    h = hashlib.blake2b(digest_size=16)
    for t in [trainer.float_state(), *trainer.int_state()]:      # BN counters are 0-dim int64 tensors
        h.update(t.detach().reshape(-1).contiguous().cpu().view(torch.uint8).numpy().tobytes())
    return h.digest()


def check_consistency(trainer, group=None, transport=None, device: Optional[torch.device] = None,
                      compressor=None) -> dict:
    """Collective over ``group``: every rank's (error word, model digest).

    Returns ``{"ok", "ranks", "transport_errors", "distinct_digests", "digest"}``; ``ok`` is
    identical on every rank.  ``transport`` is the peer transport (``error()`` != 0 after a
    barrier timeout); ``None`` for RCCL / gloo, whose failures raise instead.  ``compressor``
    (``-c Y`` top-k) contributes its sticky overflow flag as bit 30 of the error word: a select
    that produced more than k entries drops the excess identically on every rank, so the digests
    would still agree although the sparse update was wrong.
    """
    err = int(transport.error()) if transport is not None else 0
    over = getattr(compressor, "overflowed", None)
    if over is not None and over(clear=False):
        err |= 1 << 30
    dig = model_digest(trainer)
    words = [err] + [int.from_bytes(dig[i:i + 8], "little", signed=True) for i in (0, 8)]
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    if world == 1:
        rows = [words]
    else:
        on_gpu = dist.get_backend(group) == "nccl"
        mine = torch.tensor(words, dtype=torch.int64, device=device if on_gpu else "cpu")
        out = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(out, mine, group=group)
        rows = [o.cpu().tolist() for o in out]
    errors = [r[0] for r in rows]
    digests = {(r[1], r[2]) for r in rows}
    return {
        "ok": all(e == 0 for e in errors) and len(digests) == 1,
        "ranks": world,
        "transport_errors": errors,
        "distinct_digests": len(digests),
        "digest": dig.hex(),
    }
