#!/usr/bin/env python
"""fedmi headline benchmark (BASELINE.json): rounds/s + samples/s/client,
2-conv CNN (LeNet) FedAvg at 1/2/4/8 MI355X clients.

One process per GPU = one federated client (torchrun launches N ranks).
A *step* is one federated round with the reference's semantics
(SURVEY.md §6 / BASELINE.md "Round time"):

  1. local epoch: one pass over this client's strided 1/N shard of the 50,000
     training images at batch 128 with RandomCrop+HFlip augmentation, SGD
     (lr 0.1, momentum 0.9, wd 5e-4)   [fused HIP kernels, hipGraph replay]
  2. FedAvg of the full model across clients   [hand-written hipIpc peer all-reduce
     over xGMI (csrc/comm/peer_comm.hip) or RCCL -- ``--allreduce auto`` verifies
     both against each other at start-up and keeps the faster]
  3. every client evaluates the global model on the full 10,000-image test set
     (reference-literal: src/client.py:30 -> src/main.py:167-191).  At N>1 a
     second timed loop of the same length re-runs the round with the test set
     split over the clients (they all hold the same averaged model; per-round
     (loss, correct, count) summed over clients in one collective -- the same
     numbers, 1/N of the eval work) and reports it as
     ``rounds_per_sec_eval_split``; ``--eval-split`` makes that the headline
     ``value`` instead (labelled in ``config.eval_split``)
  4. the global model is persisted as Primary/optimizedModel.pth (rank 0) and
     every client checkpoint as checkpoint/<client>.pth ({'net','acc','epoch'}),
     by the native C++ writer (csrc/runtime/ckpt_writer.cpp: async device->pinned
     snapshot, torch.save-identical archive, no GIL); a round that finds the
     previous one still queued supersedes it (the files hold the newest model
     either way); the newest round is flushed to disk inside the timed region.

Total work per round is fixed (50k samples split over N clients) -> strong
scaling.  ``value`` is the whole-job training throughput (samples/s summed over
clients = 50,000 x rounds/s); rounds/s and samples/s/client are reported too.
Data: synthetic CIFAR-shaped uint8 images, random-init weights.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time
from pathlib import Path

import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

# Reference (CPU-measured, BASELINE.md / SURVEY.md §6) rounds/s at N clients.
BASELINE_ROUNDS_PER_S = {
    "lenet": {1: 0.373, 2: 0.428, 4: 0.436, 8: 0.426},
    "mobilenet": {2: 0.0137},
}
N_TRAIN, N_TEST, BATCH = 50000, 10000, 128


def _baseline_rounds(model: str, n: int):
    table = BASELINE_ROUNDS_PER_S.get(model.lower().replace("_", ""))
    if not table:
        return None
    if model.lower() == "lenet":
        return table[min(table, key=lambda k: abs(k - n))]
    return table.get(n)


def _breakdown(marks, phases, t0: float, t1: float, steps: int) -> dict:
    """Median per-round device ms of each phase (events between the phase boundaries), device busy
    per round (first -> last boundary), host ms spent issuing each phase, and the wall-clock round."""
    import statistics

    dev = {p: [] for p in phases}
    host = {p: [] for p in phases}
    span = []
    for row in marks:
        for i, p in enumerate(phases):
            dev[p].append(row[i][1].elapsed_time(row[i + 1][1]))
            host[p].append((row[i + 1][0] - row[i][0]) * 1e3)
        span.append(row[0][1].elapsed_time(row[-1][1]))
    gaps = [marks[i][0][1].elapsed_time(marks[i + 1][0][1]) - span[i] for i in range(len(marks) - 1)]
    med = lambda v: round(statistics.median(v), 4) if v else None  # noqa: E731
    mean = lambda v: round(sum(v) / len(v), 4) if v else None  # noqa: E731
    return {"device_ms": {p: med(v) for p, v in dev.items()}, "host_issue_ms": {p: med(v) for p, v in host.items()},
            "device_ms_mean": {p: mean(v) for p, v in dev.items()},
            "device_ms_max": {p: round(max(v), 4) for p, v in dev.items() if v},
            "host_issue_ms_mean": {p: mean(v) for p, v in host.items()},
            "device_round_span_ms": med(span), "device_round_span_ms_mean": mean(span),
            "device_idle_between_rounds_ms": med(gaps), "device_idle_between_rounds_ms_mean": mean(gaps),
            "device_idle_between_rounds_ms_max": round(max(gaps), 4) if gaps else None,
            "wall_ms_per_round": round((t1 - t0) / steps * 1e3, 4), "rounds": len(marks),
            "device_round_span_ms_each": [round(v, 3) for v in span],
            "device_train_ms_each": [round(v, 3) for v in dev[phases[0]]] if phases else []}


def make_transport(args, trainer, rank: int, world: int, rehearse: bool, device):
    """The FedAvg data plane at N>1.

    ``oneshot``/``twoshot``: hipIpc peer kernels.  ``rccl``: torch.distributed (RCCL).
    ``auto``: build the peer kernel, check it against the reference collective on random
    data (all ranks must agree), time both on the model's flat state and keep the faster.
    In the 1-GPU rehearsal RCCL cannot run (two ranks on one GPU), so the peer kernel
    is the GPU data plane and gloo the fallback.
    """
    from fedmi.parallel.peer import PeerAllReduce

    x = trainer.float_state()
    want = args.allreduce
    if want == "rccl":
        return None, {"chosen": "rccl" if not rehearse else "gloo"}
    algos = ["oneshot", "twoshot"] if want == "auto" else [want]
    cap = max(4 * x.numel(), 16 * (int(x.numel() * args.topk_ratio) + 64), x.numel() + 4 * (x.numel() // 256 + 64))
    store = dist.distributed_c10d._get_default_store()
    ok = torch.ones(1, device=device if not rehearse else "cpu")
    peer = None
    try:
        peer = PeerAllReduce(rank, world, cap, store, tag="bench", algo=algos[0], device=device)
    except Exception as e:  # pragma: no cover - depends on the node's IPC/peer support
        print(f"[bench] rank {rank}: peer transport unavailable: {e!r}", file=sys.stderr)
        ok.zero_()
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if ok.item() < 1:
        if peer is not None:
            peer.close()
        if want != "auto":
            raise RuntimeError("--allreduce peer transport failed on some rank")
        return None, {"chosen": "rccl", "reason": "peer transport unavailable"}
    from fedmi.parallel.select import verify_and_select

    try:
        choice, info = verify_and_select(peer, x.numel(), device, algos=algos, compare_group=want == "auto")
    except RuntimeError:
        peer.close()
        raise
    if choice is None:
        peer.close()
        if want != "auto":
            raise RuntimeError(f"peer all-reduce ({want}) failed verification: {info}")
        return None, info
    return peer, info


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20, help="timed federated rounds")
    ap.add_argument("--warmup", type=int, default=3, help="untimed rounds")
    ap.add_argument("--model", default="lenet",
                    help="lenet (headline) | resnet18 | mobilenet | ... (native HIP engines on GPU)")
    ap.add_argument("--noniid", type=int, default=0,
                    help="non-IID label shards per client (BASELINE config 3: ResNet-18, 2 shards); 0 = strided IID")
    ap.add_argument("--compress", default="none", choices=["none", "Y", "topk", "int8"],
                    help="-c Y data-plane compression of the FedAvg update (Y = the product default, int8 + error "
                         "feedback)")
    ap.add_argument("--topk-ratio", type=float, default=0.2)
    ap.add_argument("--compress-warmup", type=int, default=0, help="dense FedAvg rounds before compression starts")
    ap.add_argument("--seed", type=int, default=17, help="model-init / augmentation seed (same on every rank)")
    ap.add_argument("--allreduce", default="auto", choices=["auto", "rccl", "oneshot", "twoshot"],
                    help="FedAvg transport at N>1: hipIpc peer kernels (oneshot/twoshot), RCCL, or auto = verify "
                         "the peer kernel against RCCL and time both, keep the faster")
    ap.add_argument("--no-eval", action="store_true", help="skip per-round eval (NOT the headline config)")
    ap.add_argument("--eval-full", action="store_true",
                    help="(the default) every client evaluates the whole test set, as the reference does")
    ap.add_argument("--eval-split", action="store_true",
                    help="headline loop with the 10k test set split over the clients and the accumulators summed "
                         "(same numbers, 1/N of the eval work); labelled in config.eval_split")
    ap.add_argument("--no-split-compare", action="store_true",
                    help="N>1: skip the second timed loop that measures the split-eval round")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of hipGraph replay")
    ap.add_argument("--ckpt-dir", default=None)
    # 2 slots: the writer takes 0.22 ms per LeNet round (profiles/r6_lenet/ckpt_write_probe.jsonl), so 2 keep it off
    # the critical path at every N; with 4 the host ran 4 rounds ahead and timed rounds 2-4 after a 3-round warmup
    # trained ~0.9 ms slower (16 slots: every round; 1-2 slots or a 10-round warmup: none) -- 107.8 vs 109.2
    # rounds/s (profiles/r6_lenet/slots.md)
    ap.add_argument("--ckpt-slots", type=int, default=2, help="pinned snapshot slots of the checkpoint writer")
    ap.add_argument("--ckpt-coalesce", action="store_true",
                    help="a writer that falls behind by --ckpt-slots rounds supersedes queued rounds (files "
                         "still end at the newest round) instead of stalling the round loop")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--trace", action="store_true",
                    help="print every rank's per-round train/test stats to stderr (synchronising: not for timing)")
    ap.add_argument("--peer-timeout-ms", type=float, default=30000.0,
                    help="wall-clock limit of a peer-collective barrier (a lost peer fails the run, never hangs it)")
    ap.add_argument("--breakdown", action="store_true",
                    help="per-round device time of each phase (train / allreduce / eval / checkpoint) from events "
                         "recorded between the phases, and the host-side gaps")
    ap.add_argument("--project-world", type=int, default=0,
                    help="PROJECTION (1 GPU, labelled as such): one client runs rank 0's share of an N-client "
                         "round -- its strided 1/N training shard, a 1/N test shard, the same checkpoint writer -- "
                         "with NO collective; the per-client critical path of the N-GPU run minus the all-reduce")
    ap.add_argument("--inject-fault", default="none", choices=["none", "skip-allreduce"],
                    help="testing the end-of-run guard: the last rank skips the first timed round's FedAvg")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}; launch N>1 with torch.distributed.run",
              file=sys.stderr)
        return 2
    if args.project_world and world != 1:
        print("[bench] --project-world is a single-process projection", file=sys.stderr)
        return 2
    shard_world = args.project_world or world        # the client count whose per-client work this run does
    if not torch.cuda.is_available():
        print("[bench] no GPU visible", file=sys.stderr)
        return 2
    # FEDMI_BENCH_REHEARSE=1: rehearse the N-rank code path on ONE GPU (every rank on cuda:0,
    # gloo collectives) -- the multi-GPU run itself uses one GPU per rank and RCCL over xGMI
    rehearse = os.environ.get("FEDMI_BENCH_REHEARSE", "0") == "1"
    device = torch.device("cuda", 0 if rehearse else local_rank)
    torch.cuda.set_device(device)
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=device)

    from fedmi.ckpt import OPTIMIZED_MODEL, RoundCheckpointWriter, client_ckpt_path, mount_dir
    from fedmi.engine import build_trainer
    from fedmi.engine.base import TrainerConfig
    from fedmi.engine.data import make_dataset, strided_schedule
    from fedmi.parallel.fedavg import EvalHistory, FedAvg, broadcast_state_, eval_shard
    from fedmi.parallel.compress import make_compressor
    from fedmi.utils.trace import phase

    data = make_dataset("synthetic-cifar10", device=device, n_train=N_TRAIN, n_test=N_TEST, seed=0)
    cfg = TrainerConfig(seed=args.seed, use_graph=not args.no_graph)
    trainer = build_trainer(args.model, data, device, cfg)
    broadcast_state_(trainer, 0)                     # one shared init (reference quirk A7 fixed)
    if args.noniid > 0:     # McMahan-style label shards: each client trains only its own shard
        from fedmi.engine.data import contiguous_schedule, label_shard_indices

        shards = label_shard_indices(data.train.y.cpu().numpy(), world, args.noniid, seed=0)
        trainer.set_train_data(data.train.subset(shards[rank]))
        trainer.set_schedule(*contiguous_schedule(len(shards[rank]), BATCH))
    else:
        trainer.set_schedule(*strided_schedule(N_TRAIN, BATCH, rank, shard_world))
    transport, select = None, {}
    if world > 1:
        transport, select = make_transport(args, trainer, rank, world, rehearse, device)
        if transport is not None:
            transport.comm.set_timeout_ms(float(args.peer_timeout_ms))
            transport.timeout_ms = float(args.peer_timeout_ms)
        elif args.inject_fault != "none":
            # a rank skipping an RCCL collective hangs its peers inside RCCL: the guard test needs the
            # peer transport, whose barriers time out
            print("[bench] --inject-fault needs the peer transport", file=sys.stderr)
            return 2
    agg = FedAvg(compressor=make_compressor(args.compress, args.topk_ratio, trainer, args.compress_warmup),
                 transport=transport)
    split_eval = shard_world > 1 and args.eval_split
    if split_eval:
        trainer.set_test_data(eval_shard(data.test, rank, shard_world))
    # N>1 with full per-client eval: a second timed loop measures the split-eval round (reported, not headline)
    compare_split = shard_world > 1 and not split_eval and not args.no_split_compare and not args.no_eval
    hist = EvalHistory(trainer, args.warmup + args.steps + (args.steps + 1 if compare_split else 0))
    if args.trace:
        ys = trainer.train_set.y.long().cpu()
        print(f"[trace] rank {rank} start: {len(ys)} train samples, labels {torch.bincount(ys, minlength=10).tolist()}, "
              f"|w| {float(trainer.float_state().norm()):.4f}, sched {len(getattr(trainer, '_starts', []))} batches",
              file=sys.stderr, flush=True)

    root = Path(args.ckpt_dir or tempfile.mkdtemp(prefix="fedmi_bench_"))
    prim = mount_dir(root, primary=True) if rank == 0 else None
    cpath = client_ckpt_path(root, f"client{rank}")
    # native C++ writer (fedmi/ckpt, csrc/runtime/ckpt_writer.cpp); every round is written, in order
    writer = RoundCheckpointWriter(slots=args.ckpt_slots, coalesce=args.ckpt_coalesce)
    PHASES = ("train", "allreduce", "eval", "checkpoint")
    marks = []          # --breakdown: per round, (host perf_counter, cuda event) at each phase boundary
    fault_round = args.warmup if args.inject_fault == "skip-allreduce" and rank == world - 1 else -1

    def stamp(row):
        if args.breakdown:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            row.append((time.perf_counter(), e))

    def one_round(r: int) -> None:
        row = []
        stamp(row)
        with phase("local-train"):
            trainer.train_epoch()
        stamp(row)
        with phase("allreduce"):
            if r != fault_round:
                agg.average(trainer)
        stamp(row)
        if not args.no_eval:
            with phase("eval"):
                trainer.evaluate()
                hist.record()
        stamp(row)
        # global model -> Primary/optimizedModel.pth (rank 0) + this client's checkpoint, one snapshot
        with phase("checkpoint"):
            writer.submit([prim / OPTIMIZED_MODEL, cpath] if prim is not None else cpath, trainer.state_dict(),
                          acc=1, epoch=r + 1)
        stamp(row)
        if args.breakdown and r >= args.warmup:
            marks.append(row)
        if args.trace:
            ts, fs = trainer.train_stats(), trainer.float_state()
            ev = trainer.eval_stats() if not args.no_eval else None
            print(f"[trace] rank {rank} round {r + 1}: train loss {ts.loss:.4f} acc {ts.acc:.2f} ({ts.count})"
                  + (f" | eval acc {ev.acc:.2f} ({ev.count})" if ev else "")
                  + f" | finite {bool(torch.isfinite(fs).all())} |w| {float(fs.norm()):.4f}", file=sys.stderr, flush=True)

    def barrier():
        if world > 1:
            if rehearse:
                dist.barrier()
            else:
                dist.barrier(device_ids=[local_rank])
        torch.cuda.synchronize(device)

    for r in range(args.warmup):
        one_round(r)
    writer.flush()
    barrier()
    t0 = time.perf_counter()
    for r in range(args.warmup, args.warmup + args.steps):
        one_round(r)
    tl = [time.perf_counter()]
    writer.flush()
    tl.append(time.perf_counter())
    rounds_eval = hist.reduce() if not args.no_eval and split_eval else None
    tl.append(time.perf_counter())
    barrier()
    t1 = time.perf_counter()
    tail = {"loop_ms": round((tl[0] - t0) * 1e3, 3), "flush_ms": round((tl[1] - tl[0]) * 1e3, 3),
            "eval_reduce_ms": round((tl[2] - tl[1]) * 1e3, 3), "barrier_ms": round((t1 - tl[2]) * 1e3, 3)}
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    T = float(elapsed.item())
    full_eval_stats = trainer.eval_stats() if not args.no_eval and not split_eval else None
    T_split = None
    if compare_split:
        # the same rounds with the test set split over the clients (after the headline's timed region)
        trainer.set_test_data(eval_shard(data.test, rank, shard_world))
        one_round(args.warmup + args.steps)              # untimed: the eval graph re-captures for the shard
        writer.flush()
        barrier()
        t2 = time.perf_counter()
        for r in range(args.warmup + args.steps + 1, args.warmup + 2 * args.steps + 1):
            one_round(r)
        writer.flush()
        hist.reduce()
        barrier()
        el2 = torch.tensor([time.perf_counter() - t2], dtype=torch.float64, device=device)
        if world > 1:
            dist.all_reduce(el2, op=dist.ReduceOp.MAX)
        T_split = float(el2.item())

    # end-of-run guard (outside the timed region): no peer barrier timed out on any rank and every
    # client holds the bit-identical global model -- else the throughput above is not a FedAvg run
    from fedmi.parallel.consistency import check_consistency

    consistency = check_consistency(trainer, transport=transport, device=device, compressor=agg.compressor)
    breakdown = dict(_breakdown(marks, PHASES, t0, t1, args.steps), tail=tail) if args.breakdown else None

    tr_stats = trainer.train_stats()
    if args.no_eval:
        ev_stats = None
    elif rounds_eval is not None:
        ev_stats = rounds_eval[-1]
    else:
        ev_stats = full_eval_stats
    rounds_per_s = args.steps / T
    value = rounds_per_s * N_TRAIN / (args.project_world or 1)
    base_r = _baseline_rounds(args.model, world)
    metric = ("rounds/sec + samples/sec/client, 2-conv CNN FedAvg at 1/2/4/8 MI355X clients"
              if args.model.lower() == "lenet" else f"rounds/sec + samples/sec/client, {args.model} FedAvg")
    if args.project_world:
        metric = f"PROJECTION (1 GPU, no collective) of the per-client round at N={args.project_world}: " + metric
    out = {
        "metric": metric,
        "value": round(value, 3),
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(T / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": round(rounds_per_s / base_r, 3) if base_r else None,
        "dtype": "bf16",
        "data": "synthetic (CIFAR-shaped uint8 50k/10k, class-structured), random-init weights",
        "config": {"model": args.model, "global_batch": BATCH * world, "seq_len": None,
                   "parallelism": f"fedavg-dp{world}" if not args.project_world
                   else f"projection-of-fedavg-dp{args.project_world} (rank 0's share, no collective)",
                   "per_client_batch": BATCH,
                   "local_epochs_per_round": 1, "eval_per_round": not args.no_eval,
                   "eval_split": "full-per-client" if not split_eval else f"1/{shard_world}-per-client",
                   "data_split": f"noniid-{args.noniid}-shards" if args.noniid else "strided-iid",
                   "aggregation": agg.label() + (" [1-GPU rehearsal]" if rehearse and world > 1 else ""),
                   "hip_graph": not args.no_graph},
        "rounds_per_sec": round(rounds_per_s, 4),
        **({"rounds_per_sec_eval_split": round(args.steps / T_split, 4),
            "value_eval_split": round(args.steps / T_split * N_TRAIN / (args.project_world or 1), 3)}
           if T_split else {}),
        "samples_per_sec_per_client": round(value / world, 3),
        # what actually carried FedAvg, and among how many ranks
        "data_plane": {"aggregation": agg.label(), "world": agg.world(),
                       "collective_world": (transport.world if transport is not None
                                            else (dist.get_world_size() if dist.is_initialized() else 1)),
                       "backend": ("peer-hipipc" if transport is not None
                                   else (dist.get_backend() if dist.is_initialized() else "none"))},
        "baseline_rounds_per_sec": base_r,
        "last_round": {"train_loss": round(tr_stats.loss, 4), "train_acc": round(tr_stats.acc, 3),
                       **({"test_loss": round(ev_stats.loss, 4), "test_acc": round(ev_stats.acc, 3)}
                          if ev_stats else {})},
        "allreduce_ms_last": round(agg.timer.last_ms, 4),
        "checkpoint": {"writer": writer.backend, "files_written": writer.written,
                       "rounds_coalesced": writer.coalesced},
        **({"transport_select": select} if select else {}),
        "consistency": consistency,
        **({"native_backend": {"aten_fallbacks": sum(trainer.mode.fallbacks.values()),
                               "fallback_ops": dict(trainer.mode.fallbacks),
                               "native_ops": sum(trainer.mode.native_ops.values())}}
           if getattr(trainer, "mode", None) is not None and hasattr(trainer.mode, "fallbacks") else {}),
        **({"breakdown": breakdown} if breakdown else {}),
        **({"compression": {"kind": args.compress, "bytes_per_round_per_client":
                            agg.compressor.bytes_sent // max(1, agg.compressor.rounds),
                            "dense_bytes_per_round_per_client": agg.compressor.dense_bytes // max(1, agg.compressor.rounds)}}
           if agg.compressor is not None and agg.compressor.rounds else {}),
    }
    writer.close()
    if transport is not None:
        transport.close()          # store barrier first: no rank unmaps memory a peer's kernel may still read
    rc = 0
    if not consistency["ok"]:
        # no throughput line: a run whose clients diverged did not measure FedAvg
        print(f"[bench] rank {rank}: CONSISTENCY CHECK FAILED {json.dumps(consistency)}", file=sys.stderr, flush=True)
        out["value"] = None
        rc = 3
    if rank == 0:
        line = json.dumps(out)
        if rc == 0:
            print(line, flush=True)
        if args.json_out:
            Path(args.json_out).write_text(line + "\n")
    if world > 1:
        dist.destroy_process_group()
    return rc


if __name__ == "__main__":
    sys.exit(main())
