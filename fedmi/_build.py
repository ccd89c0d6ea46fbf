"""Build the fedmi native extension (HIP kernels + C++ runtime + bindings) for gfx950.

The extension is compiled IN-TREE with ``hipcc --offload-arch=gfx950`` so the
``.so`` travels with the repository snapshot to the GPU box.  No torch headers
are needed: device memory is passed as raw pointers from torch tensors.

Usage:  python -m fedmi._build [--force] [-j N]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build" / "native"
PKG = ROOT / "fedmi"
ARCH = os.environ.get("FEDMI_OFFLOAD_ARCH", "gfx950")

SOURCES = [
    CSRC / "kernels" / "lenet_kernels.hip",
    CSRC / "kernels" / "flat_ops.hip",
    CSRC / "kernels" / "compress.hip",
    CSRC / "kernels" / "conv_igemm.hip",
    CSRC / "kernels" / "cnn_ops.hip",
    CSRC / "kernels" / "dwconv.hip",
    CSRC / "kernels" / "zoo_ops.hip",
    CSRC / "comm" / "peer_comm.hip",
    CSRC / "runtime" / "lenet_engine.cpp",
    CSRC / "runtime" / "ckpt_writer.cpp",
    CSRC / "runtime" / "crc32_fast.cpp",
    CSRC / "bindings.cpp",
    CSRC / "bindings_cnn.cpp",
    CSRC / "bindings_comm.cpp",
    CSRC / "bindings_zoo.cpp",
    CSRC / "bindings_io.cpp",
]
HEADERS = sorted(CSRC.rglob("*.h"))


# build variants: the module name carries the variant (csrc/bindings.cpp FEDMI_MODULE); an A/B build adds
# its -D switch here for one experiment and is removed with the losing code
VARIANTS = {"": [], "stamps": ["-DFEDMI_STAMPS", "-DFEDMI_MODULE=_fedmi_native_stamps"]}


def ext_path(variant: str = "") -> Path:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    name = "_fedmi_native" + (f"_{variant}" if variant else "")
    return PKG / f"{name}{suffix}"


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build fedmi native code)")


def _stamp(variant: str = "") -> str:
    h = hashlib.sha256()
    h.update(ARCH.encode())
    h.update(variant.encode())
    for p in SOURCES + HEADERS + [Path(__file__)]:
        h.update(p.name.encode())
        h.update(p.read_bytes())
    return h.hexdigest()


def _compile(src: Path, variant: str = "") -> Path:
    import pybind11

    bdir = BUILD.with_name(BUILD.name + (f"_{variant}" if variant else ""))
    bdir.mkdir(parents=True, exist_ok=True)
    obj = bdir / (src.stem + ".o")
    cmd = [
        _hipcc(), "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", *VARIANTS[variant],
        "-Wno-unused-result", "-I", str(CSRC),
        "-I", pybind11.get_include(), "-I", sysconfig.get_paths()["include"],
        "-c", str(src), "-o", str(obj),
    ]
    if src.suffix == ".cpp":
        cmd[1:1] = ["-fvisibility=hidden"]
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"compile failed: {src.name}\n{' '.join(cmd)}\n{proc.stdout}\n{proc.stderr}")
    return obj


def build(force: bool = False, jobs: int = 4, verbose: bool = True, variant: str = "") -> Path:
    out = ext_path(variant)
    bdir = BUILD.with_name(BUILD.name + (f"_{variant}" if variant else ""))
    stamp_file = bdir / "stamp"
    stamp = _stamp(variant)
    if not force and out.exists() and stamp_file.exists() and stamp_file.read_text() == stamp:
        if verbose:
            print(f"[fedmi build] up to date: {out.name}")
        return out
    bdir.mkdir(parents=True, exist_ok=True)
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda src: _compile(src, variant), SOURCES))
    tmp = out.with_suffix(".tmp.so")
    cmd = [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-lz", "-o", str(tmp)]
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"link failed\n{' '.join(cmd)}\n{proc.stdout}\n{proc.stderr}")
    os.replace(tmp, out)
    stamp_file.write_text(stamp)
    if verbose:
        print(f"[fedmi build] built {out} ({out.stat().st_size // 1024} KiB, arch={ARCH})")
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--stamps", action="store_true", help="also build the per-phase timestamp diagnostic variant")
    ap.add_argument("--variant", default="", choices=[v for v in VARIANTS if v], help="also build this variant")
    a = ap.parse_args(argv)
    build(force=a.force, jobs=a.jobs)
    if a.stamps:
        build(force=a.force, jobs=a.jobs, variant="stamps")
    if a.variant:
        build(force=a.force, jobs=a.jobs, variant=a.variant)
    return 0


if __name__ == "__main__":
    sys.exit(main())
