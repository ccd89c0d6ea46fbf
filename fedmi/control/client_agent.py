"""Client agent: the ``federated.Trainer`` servicer run by every client.

Reference: src/client.py:15-35 (+ the import-time trainer in src/main.py).

  StartTrain(rank, world) -> one local epoch on this client's shard, then
      * ``agg="grpc"`` (reference semantics): reply = base64(checkpoint of the
        LOCAL model); the coordinator averages and sends it back (SendModel);
      * ``agg="collective"`` (fedmi default): FedAvg happens right here as an
        RCCL all-reduce among the clients (rank/world from the request, the
        data-plane generation + rendezvous store from gRPC metadata); every
        client evaluates the global model; only rank 0 uploads the (already
        averaged) checkpoint so the coordinator can persist/replicate it.
        Checkpoints are written by a background writer; rank 0's upload is
        pipelined (the reply carries the newest checkpoint serialised so far,
        usually the previous round's) unless the coordinator asks for this
        round's (``x-fedmi-sync-ckpt: 1``, e.g. on the final round).
        A new membership generation starts with a resync from rank 0.
        Round lease (``x-fedmi-lease: K``, fedmi extension): one StartTrain runs K
        consecutive synchronous rounds (round numbers x-fedmi-round .. +K-1, one
        data-plane generation), each fenced, averaged, evaluated and checkpointed
        exactly like a single round; per-round stats return in the trailing
        metadata, so the gRPC round trip is paid once per K rounds instead of once
        per round (control plane off the critical path).  A collective
        that fails inside a lease rolls this client back to the last committed
        round (the previous lease round) and ends the call with ABORTED.
  SendModel(b64 checkpoint) -> install it (resync / grpc-mode broadcast), persist,
      evaluate.
  HeartBeat() -> status 1.

Fixes vs the reference: one lock serialises RPCs that touch the model
(quirk: concurrent StartTrain/SendModel raced on one global net), requests
from a coordinator with an older *term* are rejected (split-brain fencing),
checkpoints are never ``module.``-prefixed, the checkpoint dir is created.
"""
from __future__ import annotations

import json
import os
import threading
import time
from pathlib import Path
from typing import Optional

import grpc
import torch

from .. import ckpt as ck
from ..engine.base import LocalTrainer
from ..engine.data import contiguous_schedule, strided_schedule
from ..parallel.fedavg import FedAvg
from ..parallel.group import GroupManager, Membership
from ..utils.metrics import MetricsLog, Timer, log
from ..utils.trace import phase
from ..wire import proto as P

META_TERM = "x-fedmi-term"
META_ROUND = "x-fedmi-round"
META_GEN = "x-fedmi-gen"
META_STORE = "x-fedmi-store"
META_SYNC = "x-fedmi-sync-ckpt"        # "1": the reply must carry THIS round's checkpoint
META_UPLOAD = "x-fedmi-upload"         # "0": leave the checkpoint out of the StartTrain reply (fetched later)
META_FETCH = "x-fedmi-fetch"           # on SendModel: "1" = return the newest checkpoint instead of installing
META_HAVE = "x-fedmi-have-epoch"       # on a fetch: the coordinator already holds this epoch (reply empty unless newer)
META_LEASE = "x-fedmi-lease"           # on StartTrain: "K" = run K consecutive synchronous rounds in this call


def metadata_dict(context) -> dict:
    try:
        return {k: v for k, v in (context.invocation_metadata() or ())}
    except Exception:
        return {}


class ClientAgent(P.TrainerServicer):
    def __init__(self, trainer: LocalTrainer, address: str, *, root: str | Path = ".", agg: str = "collective",
                 group: Optional[GroupManager] = None, fedavg: Optional[FedAvg] = None, batch_size: int = 128,
                 local_shard: bool = False, resume: bool = False, metrics: Optional[MetricsLog] = None,
                 verbose: bool = True, writer: Optional[ck.AsyncCheckpointWriter] = None):
        if agg not in ("collective", "grpc"):
            raise ValueError(f"agg must be 'collective' or 'grpc', not {agg!r}")
        self.trainer = trainer
        self.address = address
        self.agg = agg
        self.group = group
        self.fedavg = fedavg or FedAvg()
        self.batch = batch_size
        self.local_shard = local_shard          # non-IID: the client owns its data, rank does not pick batches
        self.metrics = metrics or MetricsLog()
        self.verbose = verbose
        self.writer = writer or ck.AsyncCheckpointWriter()
        self.lock = threading.RLock()
        self.max_term = 0
        self.round = 0
        self._busy_gen: Optional[int] = None    # generation of the round holding the lock
        self._ready_lock = threading.Lock()
        self._ready: Optional[tuple] = None     # (epoch, bytes) newest serialised global checkpoint
        self._sent_epoch = -1
        self._ready_branch = 0                  # bumped when SendModel installs a model (rollback / resync):
                                                # checkpoints serialised on the abandoned branch are dropped
        self.ckpt_path = ck.client_ckpt_path(root, address.replace("/", "_"))
        # fault injection (tests / drills): stall this many seconds right before the FedAvg
        # collective, so a kill lands while the other clients wait inside it
        self.fault_stall_avg_s = float(os.environ.get("FEDMI_FAULT_STALL_AVG_S", "0") or 0)
        self.fault_stall_from = int(os.environ.get("FEDMI_FAULT_STALL_FROM_ROUND", "0") or 0)
        self._round_start = None                # (float, [int]) device copies of the round's starting global model
        self._debug_stats = os.environ.get("FEDMI_DEBUG_STATS", "0") == "1"
        self._select_logged = False
        self._overflow_logged = False
        self._newest_term = 0                   # highest term any StartTrain carried (read without the lock)
        if self._debug_stats:
            from ..parallel import compress as _comp
            _comp.PROBE = self._probe
        if resume and self.ckpt_path.exists():
            c = ck.load(self.ckpt_path)
            trainer.load_state_dict(c["net"])
            self.round = int(c.get("epoch", 0))
            self._log(f"resumed from {self.ckpt_path} (epoch {self.round})")
        else:
            # reference bootstrap: persist the initial model (src/main.py:231-239)
            ck.save(self.ckpt_path, ck.make_checkpoint(trainer.state_dict(), acc=1, epoch=self.round))

    def _log(self, msg: str) -> None:
        if self.verbose:
            log(f"client {self.address}", msg)

    def _probe(self, tag: str) -> None:
        """FEDMI_DEBUG_STATS=1: synchronise and log the trainer's stats rows after each phase (diagnostics
        for a stats word that changed outside the training kernels)."""
        st = getattr(self.trainer, "stats", None)
        if not self._debug_stats or st is None:
            return
        torch.cuda.synchronize(st.device)
        log(f"client {self.address}", f"probe {tag}: stats {st.cpu().view(-1).tolist()}")   # even with --quiet

    # ---- helpers ------------------------------------------------------------------
    def _fence(self, meta: dict, context) -> None:
        term = int(meta.get(META_TERM, "0") or 0)
        if term and term < self.max_term:
            context.abort(grpc.StatusCode.FAILED_PRECONDITION,
                          f"stale coordinator term {term} < {self.max_term}")
        self.max_term = max(self.max_term, term)

    def _schedule(self, rank: int, world: int):
        n = len(self.trainer.train_set)
        if self.local_shard:
            return contiguous_schedule(n, self.batch)
        return strided_schedule(n, self.batch, rank, world)

    def _persist_async(self, acc, epoch: int, keep: bool) -> None:
        """Checkpoint off the RPC thread (pinned snapshot + writer thread); with ``keep`` the
        serialised bytes are also kept for the coordinator's upload."""
        def _keep(_path, data, _epoch=epoch, _branch=self._ready_branch):
            with self._ready_lock:
                if _branch != self._ready_branch:
                    return                      # serialised before a rollback: not the committed history
                if self._ready is None or _epoch >= self._ready[0]:
                    self._ready = (_epoch, data)

        self.writer.submit(self.ckpt_path, self.trainer.state_dict(), acc=acc, epoch=epoch,
                           on_done=_keep if keep else None)

    def _snapshot_round_start(self) -> None:
        """Device copy of the model this round starts from (the last committed global model): one
        D2D copy of the flat state, the rollback target if the round's collective fails."""
        fs, ints = self.trainer.float_state(), self.trainer.int_state()
        if self._round_start is None or self._round_start[0].shape != fs.shape or len(self._round_start[1]) != len(ints):
            self._round_start = (torch.empty_like(fs), [torch.empty_like(b) for b in ints])
        self._round_start[0].copy_(fs, non_blocking=True)
        for d, b in zip(self._round_start[1], ints):
            d.copy_(b, non_blocking=True)

    def _restore_round_start(self) -> Optional[float]:
        if self._round_start is None:
            return None
        self.trainer.float_state().copy_(self._round_start[0])
        for b, src in zip(self.trainer.int_state(), self._round_start[1]):
            b.copy_(src)
        self.trainer.after_aggregate()
        comp = getattr(self.fedavg, "compressor", None)
        if comp is not None:
            comp.reset(self.trainer)
        return ck.state_digest(self.trainer.state_dict())

    def _reset_ready(self, epoch: int, data: bytes) -> None:
        """A model installed by the coordinator (rollback, rejoin resync) is the committed history from now
        on: the ready buffer holds it, uploads restart after its epoch, and writer callbacks of checkpoints
        serialised before it (a branch the coordinator discarded, possibly labelled with HIGHER epochs) are
        ignored -- otherwise the fetcher would install the abandoned model and the re-run rounds up to that
        epoch would never be uploaded."""
        with self._ready_lock:
            self._ready_branch += 1
            self._ready = (epoch, data)
            self._sent_epoch = epoch

    def _take_ready(self) -> tuple:
        """(epoch, b64) of the newest serialised checkpoint not uploaded yet, or (-1, '')."""
        with self._ready_lock:
            if self._ready is None or self._ready[0] <= self._sent_epoch:
                return -1, ""
            self._sent_epoch = self._ready[0]
            return self._ready[0], ck.to_b64(self._ready[1])

    # ---- RPCs ---------------------------------------------------------------------
    def StartTrain(self, request, context):
        t_enter = time.time()
        meta = metadata_dict(context)
        gen = int(meta.get(META_GEN, "0") or 0)
        term = int(meta.get(META_TERM, "0") or 0)
        if term > self._newest_term:
            self._newest_term = term            # seen before the lock: a running lease stops at its next round
        busy = self._busy_gen
        if self.group is not None and busy is not None and gen > busy:
            # a newer membership while an older round is still blocked in its collective
            self._log(f"generation {gen} supersedes running generation {busy}: interrupting it")
            self.group.interrupt()
        with self.lock:
            self._busy_gen = gen
            try:
                return self._start_train(request, context, meta, gen, t_enter)
            finally:
                self._busy_gen = None

    def _start_train(self, request, context, meta: dict, gen: int, t_enter: float = 0.0):
        term = int(meta.get(META_TERM, "0") or 0)
        first_of_term = term > self.max_term and self.max_term > 0
        self._fence(meta, context)
        rank, world = int(request.rank), int(request.world)
        if world <= 0 or not 0 <= rank < world:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"bad rank/world {rank}/{world}")
        rnd = int(meta.get(META_ROUND, self.round + 1) or self.round + 1)
        if self.agg == "collective" and first_of_term and rnd <= self.round:
            # a newly promoted coordinator resumes from its replica, which can trail the rounds this client
            # committed under the previous term (a lease keeps running until the new term reaches it): report
            # the committed round instead of re-running it; the coordinator pulls rank 0's model of that round
            # and continues after it (once per term, so a coordinator that cannot reach that model rolls back)
            self._lease_trailer(context, [], -1)
            context.abort(grpc.StatusCode.FAILED_PRECONDITION,
                          f"round {rnd} of term {term}: this client already committed round {self.round}")
        lease = max(1, int(meta.get(META_LEASE, "1") or 1)) if self.agg == "collective" else 1
        t = Timer()
        rec0 = {"role": "client", "address": self.address, "rank": rank, "world": world, "agg": self.agg,
                "generation": gen}
        if self.agg == "collective":
            host, _, port = (meta.get(META_STORE) or "127.0.0.1:0").rpartition(":")
            changed = False
            if self.group is not None:
                with phase("group"):
                    try:
                        changed = self.group.ensure(Membership(gen, rank, world, host, int(port)))
                    except Exception as e:      # rendezvous failed (a member never showed up)
                        context.abort(grpc.StatusCode.ABORTED, f"data-plane group failed: {e}"[:500])
                self.fedavg.transport = self.group.transport
                self.fedavg.abort = self.group.abort_event
                self._probe("group")
            elif world > 1:
                context.abort(grpc.StatusCode.FAILED_PRECONDITION, "collective aggregation needs a GroupManager")
            if changed and self.group is not None and self.group.select_info and not self._select_logged:
                rec0["transport_select"] = self.group.select_info      # the auto data-plane decision, once
                self._select_logged = True
            if changed and world > 1:
                # new member set: everyone starts this generation from rank 0's model (one anchor
                # for the -c Y compressors; undoes any partially applied aborted round)
                self.fedavg.resync(self.trainer, 0)
                rec0["resync"] = True
                self._probe("resync")
            elif changed and self.fedavg.compressor is not None:
                self.fedavg.compressor.reset(self.trainer)
            rec0["group_ms"] = t.ms()
        lease_stats = []
        ck_epoch, message = -1, ""
        for i in range(lease):
            r = rnd + i
            if i > 0 and term and term < max(self.max_term, self._newest_term):
                # a newer coordinator reached this client mid-lease: stop at the committed round
                self._lease_trailer(context, lease_stats, -1)
                context.abort(grpc.StatusCode.FAILED_PRECONDITION,
                              f"lease of term {term} superseded by term {self._newest_term} after round {self.round}")
            rec = dict(rec0, round=r, lease=lease, lease_index=i) if i == 0 else dict(
                {k: v for k, v in rec0.items() if k not in ("group_ms", "resync", "transport_select")},
                round=r, lease=lease, lease_index=i)
            last = i == lease - 1
            tr, ck_epoch, message = self._one_round(rank, world, r, meta, gen, context, rec, lease_stats,
                                                    t_enter if i == 0 else time.time(), last)
            lease_stats.append((r, round(tr.loss, 6), round(rec.get("test_acc", -1.0), 4), round(time.time(), 6)))
        self._lease_trailer(context, lease_stats, ck_epoch)
        return P.TrainReply(message=message)

    def _lease_trailer(self, context, lease_stats, ck_epoch: int) -> None:
        last = lease_stats[-1] if lease_stats else (self.round, -1.0, -1.0, time.time())
        try:
            context.set_trailing_metadata((("x-fedmi-client-round", str(self.round)),
                                           ("x-fedmi-ckpt-epoch", str(ck_epoch)),
                                           ("x-fedmi-train-loss", f"{last[1]:.6f}"),
                                           ("x-fedmi-test-acc", f"{last[2]:.4f}"),
                                           ("x-fedmi-lease-stats", json.dumps(lease_stats, separators=(",", ":")))))
        except Exception:
            pass

    def _one_round(self, rank: int, world: int, rnd: int, meta: dict, gen: int, context, rec: dict, lease_stats,
                   t_enter: float, last: bool):
        """One synchronous round (local epoch, FedAvg, eval, checkpoint) of a StartTrain lease."""
        t = Timer()
        if self.agg == "collective" and world > 1:
            self._snapshot_round_start()
        t1 = Timer()
        with phase("local-train"):
            self.trainer.set_schedule(*self._schedule(rank, world))
            self._probe("pre-train")
            self.trainer.train_epoch()
            self._probe("train")
            tr = self.trainer.train_stats()
        rec.update(tr.as_dict("train"))
        rec["train_ms"] = t1.ms()
        if self.agg == "collective":
            if self.fault_stall_avg_s > 0 and world > 1 and rnd >= self.fault_stall_from:
                self.trainer.synchronize()
                time.sleep(self.fault_stall_avg_s)
            t2 = Timer()
            with phase("allreduce"):
                try:
                    self.fedavg.average(self.trainer)
                    self._probe("average")
                    tp = self.fedavg.transport
                    err = "peer collective timed out (a client was lost)" if tp is not None and tp.error() else ""
                    err = err or self._lost_peer()
                except Exception as e:          # gloo / RCCL error: a peer was lost mid-collective
                    err = f"collective failed: {e}"
            if err:
                self._void_round(rnd, gen, err, context, lease_stats)
            rec["allreduce_ms"] = t2.ms()
            t3 = Timer()
            with phase("eval"):
                self.trainer.evaluate()
                ev = self.trainer.eval_stats()
            self._probe("eval")
            # a stream-ordered collective (RCCL) the watchdog aborted surfaces only here, after the eval's sync
            err = self._lost_peer() if world > 1 else ""
            if err:
                self._void_round(rnd, gen, err, context, lease_stats)
            rec["eval_ms"] = t3.ms()
            rec.update(ev.as_dict("test"))
            self.round = rnd
            self._check_compressor(rnd)
            t4 = Timer()
            with phase("checkpoint"):
                self._persist_async(ev.acc, rnd, keep=(rank == 0))
                sync = last and meta.get(META_SYNC) == "1"
                if rank == 0 and sync:
                    self.writer.flush()
                upload = last and rank == 0 and (sync or meta.get(META_UPLOAD) != "0")
                ck_epoch, message = self._take_ready() if upload else (-1, "")
            rec["ckpt_ms"] = t4.ms()
            self._probe("ckpt")
        else:
            # reference parameter-server path: the reply IS this round's local model
            self.round = rnd
            t4 = Timer()
            data = ck.to_bytes(ck.make_checkpoint(self.trainer.state_dict(), acc=tr.acc, epoch=rnd))
            self.writer.submit_bytes(self.ckpt_path, data)
            ck_epoch, message = rnd, ck.to_b64(data)
            rec["ckpt_ms"] = t4.ms()
        rec["round_ms"] = t.ms()
        rec["t_enter"], rec["t_exit"] = t_enter, time.time()
        self.metrics.write(**rec)
        self._log(f"round {rnd} rank {rank}/{world}: train loss {tr.loss:.4f} acc {tr.acc:.2f}%"
                  + (f" | test acc {rec['test_acc']:.2f}%" if "test_acc" in rec else ""))
        return tr, ck_epoch, message

    def _lost_peer(self) -> str:
        """The coordinator reported a lost client for this generation (abort watchdog)."""
        g = self.group
        if g is not None and g.abort_event.is_set():
            return "collective aborted: the coordinator reported a lost client"
        return ""

    def _void_round(self, rnd: int, gen: int, err: str, context, lease_stats) -> None:
        """The round is void: back to the global model it started from (identical on every survivor; a peer
        collective may have written the mean into part of the model before failing), then ABORTED."""
        digest = self._restore_round_start()
        self.metrics.write(role="client", address=self.address, event="round_aborted", round=rnd,
                           generation=gen, error=err[:200], restored_sum=digest)
        # the lease's earlier rounds are committed: report how far this client got
        self._lease_trailer(context, lease_stats, -1)
        # ABORTED (not UNAVAILABLE): this client is alive, only the round is void
        context.abort(grpc.StatusCode.ABORTED, err[:500])

    def _check_compressor(self, rnd: int) -> None:
        """-c Y top-k: log the kernel's sticky overflow flag once (it is a kernel bug, never a data condition);
        checked every 64 rounds (the read synchronises)."""
        comp = getattr(self.fedavg, "compressor", None)
        over = getattr(comp, "overflowed", None)
        if over is None or self._overflow_logged or rnd % 64:
            return
        if over(clear=False):
            self._overflow_logged = True
            self._log("WARNING: top-k select overflowed (entries beyond k were dropped on every rank)")
            self.metrics.write(role="client", address=self.address, event="topk_overflow", round=rnd)

    def SendModel(self, request, context):
        meta = metadata_dict(context)
        if meta.get(META_FETCH) == "1":
            return self._fetch(meta, context)
        with self.lock:
            self._fence(meta, context)
            data = ck.from_b64(request.model)
            c = ck.from_bytes(data)
            self.trainer.load_state_dict(c["net"])
            comp = getattr(self.fedavg, "compressor", None)
            if comp is not None:
                comp.reset(self.trainer)
            self.writer.submit_bytes(self.ckpt_path, data)
            epoch = int(c.get("epoch", 0) or 0)
            self._reset_ready(epoch, data)
            self.round = max(self.round, epoch)
            self.trainer.evaluate()
            ev = self.trainer.eval_stats()
            self.metrics.write(role="client", address=self.address, event="send_model", round=self.round,
                               epoch=int(c.get("epoch", 0) or 0), state_sum=ck.state_digest(c["net"]),
                               **ev.as_dict("test"))
            self._log(f"installed model (epoch {self.round}): test loss {ev.loss:.4f} acc {ev.acc:.2f}%")
            return P.SendModelReply(reply="success")

    def _fetch(self, meta: dict, context):
        """The coordinator pulls the newest serialised global checkpoint off the round's critical path
        (fedmi extension over the reference's SendModel: the reply string carries the base64 model).
        Takes only the ready-buffer lock, so it never waits for a running StartTrain."""
        term = int(meta.get(META_TERM, "0") or 0)
        if term and term < self.max_term:
            context.abort(grpc.StatusCode.FAILED_PRECONDITION, f"stale coordinator term {term} < {self.max_term}")
        have = int(meta.get(META_HAVE, "-1") or -1)
        with self._ready_lock:
            ready = self._ready
        if ready is None:
            epoch, b64 = -1, ""
        elif ready[0] <= have:
            epoch, b64 = ready[0], ""           # nothing newer than what the coordinator holds
        else:
            epoch, b64 = ready[0], ck.to_b64(ready[1])
        try:
            context.set_trailing_metadata((("x-fedmi-ckpt-epoch", str(epoch)),))
        except Exception:
            pass
        return P.SendModelReply(reply=b64)

    def HeartBeat(self, request, context):
        return P.HeartBeatResponse(status=1)

    def close(self) -> None:
        self.writer.close()
        self.metrics.close()


def serve_client(agent: ClientAgent, address: str, gzip: bool = False, max_workers: int = 10):
    """Start the client's gRPC server (reference src/client.py:38-52); returns the server."""
    server = P.make_server(max_workers=max_workers, gzip=gzip)
    P.add_TrainerServicer_to_server(agent, server)
    port = server.add_insecure_port(address)
    if port == 0:
        raise RuntimeError(f"could not bind {address}")
    server.start()
    return server, port


def wait_forever(server, stop: Optional[threading.Event] = None) -> None:
    try:
        while stop is None or not stop.is_set():
            time.sleep(0.5)
    finally:
        server.stop(grace=1.0)
