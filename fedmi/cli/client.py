"""Client process: ``python -m fedmi.cli.client -a host:port ...``.

Reference-compatible flags (src/client.py:55-71 + the flags of the imported
src/main.py:20-28): ``-a/--address`` (listen address AND checkpoint name),
``-c/--compressFlag Y``, ``-r/--resume``, ``--lr``.  One client = one GPU:
``--device cuda:N`` (default: LOCAL_RANK / first GPU, CPU if none).
"""
from __future__ import annotations

import argparse
import os
import signal
import sys
import threading

import torch

from ..control.client_agent import ClientAgent, serve_client
from ..engine import build_trainer
from ..engine.base import TrainerConfig
from ..engine.data import label_shard_indices, make_dataset
from ..parallel.compress import make_compressor
from ..parallel.fedavg import FedAvg
from ..parallel.group import GroupManager
from ..utils.metrics import MetricsLog, log


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description="fedmi federated client (one GPU)")
    ap.add_argument("-c", "--compressFlag", help="'Y': gzip gRPC + compressed FedAvg updates (int8 + error feedback)")
    ap.add_argument("-a", "--address", default="temp", help="listen address host:port (also the checkpoint name)")
    ap.add_argument("-r", "--resume", action="store_true", help="resume from checkpoint/<address>.pth")
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--model", default="lenet")
    ap.add_argument("--device", default="auto")
    ap.add_argument("--agg", default="collective", choices=["collective", "grpc"])
    ap.add_argument("--backend", default="auto", help="dist data-plane backend: nccl (RCCL) | gloo | auto")
    ap.add_argument("--transport", default="auto", choices=["auto", "peer", "dist"],
                    help="FedAvg data plane: peer = hipIpc peer kernels among the node's GPU clients (also "
                         "several clients on one GPU); dist = torch.distributed (--backend); auto (GPU) = verify the "
                         "peer kernels against the process group's all-reduce at the first multi-client generation, "
                         "time both, keep the faster (CPU: dist)")
    ap.add_argument("--collective-timeout", type=float, default=20.0,
                    help="seconds before a collective with a lost peer fails (peer barrier / RCCL abort)")
    ap.add_argument("--data", default="synthetic-cifar10",
                    help="synthetic-cifar10 | synthetic-mnist | cifar10-bin:<dir>")
    ap.add_argument("--n-train", type=int, default=None)
    ap.add_argument("--n-test", type=int, default=None)
    ap.add_argument("--batch-size", type=int, default=128)
    ap.add_argument("--seed", type=int, default=0, help="model-init / augmentation seed (same on all clients)")
    ap.add_argument("--data-seed", type=int, default=0)
    ap.add_argument("--noniid", type=int, default=0, help="label shards per client (0 = reference strided IID)")
    ap.add_argument("--client-index", type=int, default=0)
    ap.add_argument("--num-clients", type=int, default=1)
    ap.add_argument("--compress", default=None, choices=["none", "topk", "int8"],
                    help="update compression (default with -c Y: int8 + error feedback, see "
                         "fedmi.parallel.compress.DEFAULT_Y)")
    ap.add_argument("--topk-ratio", type=float, default=0.2)
    ap.add_argument("--compress-warmup", type=int, default=0, help="dense FedAvg rounds before -c Y compression starts")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--root", default=".")
    ap.add_argument("--metrics", default=None)
    ap.add_argument("--quiet", action="store_true")
    return ap


def pick_device(spec: str) -> torch.device:
    if spec != "auto":
        return torch.device(spec)
    if torch.cuda.is_available():
        return torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    return torch.device("cpu")


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    gzip = a.compressFlag == "Y"
    dev = pick_device(a.device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "3")   # surface peer loss as an error, no teardown
        os.environ.setdefault("TORCH_NCCL_BLOCKING_WAIT", "1")          # collectives honour the PG timeout
    log(f"client {a.address}", f"Client is running on {a.address} ({dev}); Compression {a.compressFlag} enabled")
    data = make_dataset(a.data, device=dev, n_train=a.n_train, n_test=a.n_test, seed=a.data_seed)
    cfg = TrainerConfig(lr=a.lr, batch_size=a.batch_size, seed=a.seed, use_graph=not a.no_graph)
    trainer = build_trainer(a.model, data, dev, cfg)
    if a.noniid > 0:
        shards = label_shard_indices(data.train.y.cpu().numpy(), a.num_clients, a.noniid, seed=a.data_seed)
        trainer.set_train_data(data.train.subset(shards[a.client_index]))
    backend = a.backend if a.backend != "auto" else ("nccl" if dev.type == "cuda" else "gloo")
    transport = a.transport if a.transport != "auto" else ("auto" if dev.type == "cuda" else "dist")
    comp_kind = a.compress if a.compress is not None else ("Y" if gzip else "none")
    fedavg = FedAvg(compressor=make_compressor(comp_kind, a.topk_ratio, trainer, a.compress_warmup))
    n = trainer.float_state().numel()
    cap = max(4 * n, 16 * (int(n * a.topk_ratio) + 64), n + 4 * (n // 256 + 64))
    group = GroupManager(backend, dev, timeout_s=a.collective_timeout, transport=transport, peer_capacity=cap,
                         peer_timeout_ms=1000.0 * a.collective_timeout, model_numel=n)
    agent = ClientAgent(trainer, a.address, root=a.root, agg=a.agg, group=group,
                        fedavg=fedavg, batch_size=a.batch_size, local_shard=a.noniid > 0, resume=a.resume,
                        metrics=MetricsLog(a.metrics, background=True), verbose=not a.quiet)
    server, port = serve_client(agent, a.address, gzip=gzip)
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    signal.signal(signal.SIGINT, lambda *_: stop.set())
    while not stop.is_set():
        stop.wait(0.5)
    server.stop(grace=1.0)
    agent.close()
    if agent.group is not None:
        agent.group.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
