"""Shared test helpers (ports, subprocess clients, small CPU trainers)."""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def small_trainer(model="mlp", n_train=512, n_test=256, seed=0, lr=0.05):
    from fedmi.engine import build_trainer
    from fedmi.engine.base import TrainerConfig
    from fedmi.engine.data import make_dataset

    spec = "synthetic-mnist" if model == "mlp" else "synthetic-cifar10"
    data = make_dataset(spec, device="cpu", n_train=n_train, n_test=n_test, seed=0)
    return build_trainer(model, data, torch.device("cpu"), TrainerConfig(lr=lr, seed=seed, eval_batch_size=256))


def spawn_client(address: str, root: Path, *extra: str, log_path: Path | None = None,
                 device: str = "cpu", env_extra: dict | None = None) -> subprocess.Popen:
    env = dict(os.environ)
    env.update(env_extra or {})
    env["PYTHONPATH"] = str(ROOT) + os.pathsep + env.get("PYTHONPATH", "")
    env["OMP_NUM_THREADS"] = "1"
    cmd = [sys.executable, "-m", "fedmi.cli.client", "-a", address, "--device", device, "--root", str(root),
           "--quiet", *extra]
    out = open(log_path, "w") if log_path else subprocess.DEVNULL
    return subprocess.Popen(cmd, env=env, cwd=str(root), stdout=out, stderr=subprocess.STDOUT,
                            start_new_session=True)


def wait_heartbeat(address: str, timeout: float = 60.0) -> None:
    from fedmi.wire import proto as P

    stub = P.TrainerStub(P.make_channel(address))
    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            if stub.HeartBeat(P.Request(), timeout=1.0).status == 1:
                return
        except Exception:
            time.sleep(0.2)
    raise TimeoutError(f"client {address} did not come up")


def stop_proc(p: subprocess.Popen) -> None:
    if p.poll() is None:
        try:
            os.killpg(p.pid, 15)
        except ProcessLookupError:
            return
        try:
            p.wait(timeout=10)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, 9)
            p.wait(timeout=10)


def spawn_server(root: Path, *args: str, log_path: Path | None = None) -> subprocess.Popen:
    """``python server.py ...`` (the reference-compatible coordinator entry point) in its own session."""
    env = dict(os.environ)
    env["PYTHONPATH"] = str(ROOT) + os.pathsep + env.get("PYTHONPATH", "")
    env["OMP_NUM_THREADS"] = "1"
    out = open(log_path, "w") if log_path else subprocess.DEVNULL
    return subprocess.Popen([sys.executable, str(ROOT / "server.py"), *args], env=env, cwd=str(root), stdout=out,
                            stderr=subprocess.STDOUT, start_new_session=True)


def kill9(p: subprocess.Popen) -> float:
    """SIGKILL the process group; returns the kill time (time.time())."""
    t = time.time()
    try:
        os.killpg(p.pid, 9)
    except ProcessLookupError:
        pass
    p.wait(timeout=10)
    return t


def read_jsonl(path: Path) -> list:
    import json

    if not Path(path).exists():
        return []
    out = []
    for line in Path(path).read_text().splitlines():
        try:
            out.append(json.loads(line))
        except ValueError:          # a line being written
            pass
    return out


def wait_for(pred, timeout: float = 60.0, step: float = 0.05):
    t0 = time.time()
    while time.time() - t0 < timeout:
        v = pred()
        if v:
            return v
        time.sleep(step)
    raise TimeoutError("condition not reached")


def seed_band(native, fp32, floor: float, k: float = 2.0, lower_only: bool = False):
    """Multi-seed parity gate: a chaotic few-epoch trajectory is not an oracle for ONE seed
    (any rounding change moves it), but the MEAN over seeds must agree with the fp32 engine's mean within
    ``k`` x the fp32 engine's own seed-to-seed standard deviation (never tighter than ``floor``).  Returns
    (gap, tolerance, details) and asserts.  ``lower_only``: only a native mean BELOW fp32's by more than the
    tolerance fails (a gate on "learns no worse than fp32" where fp32 itself stays at chance in some seeds)."""
    import statistics

    assert len(native) == len(fp32) >= 3, (native, fp32)
    mn, mf = statistics.fmean(native), statistics.fmean(fp32)
    sd = statistics.stdev(fp32)
    tol = max(floor, k * sd)
    info = {"native": [round(v, 4) for v in native], "fp32": [round(v, 4) for v in fp32],
            "mean_native": round(mn, 4), "mean_fp32": round(mf, 4), "fp32_sd": round(sd, 4), "tol": round(tol, 4)}
    assert (mn >= mf - tol) if lower_only else (abs(mn - mf) <= tol), info
    return abs(mn - mf), tol, info
