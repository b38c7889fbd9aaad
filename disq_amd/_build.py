"""Locate (and, on request, build) the in-tree native libraries under disq_amd/_build/."""
from __future__ import annotations

import os
import subprocess

_PKG = os.path.dirname(os.path.abspath(__file__))
BUILD_DIR = os.path.join(_PKG, "_build")
CSRC = os.path.join(_PKG, "csrc")
GPU_LIB = os.path.join(BUILD_DIR, "libdisq_gpu.so")
SYNTH_LIB = os.path.join(BUILD_DIR, "libdisq_synth.so")


def build(jobs: int = 8) -> None:
    """Compile every native library for gfx950 (hipcc cross-compiles without a GPU)."""
    env = dict(os.environ)
    env.setdefault("ARCH", "gfx950")
    subprocess.run(["make", "-s", f"-j{jobs}", "-C", CSRC], check=True, env=env)


def _need(path: str) -> str:
    if not os.path.exists(path):
        raise RuntimeError(
            f"{os.path.basename(path)} is not built; run __graft_entry__.build() or "
            f"`make -C {CSRC}` first")
    return path


def gpu_lib_path() -> str:
    # DQ_GPU_LIB: an alternative build of the same library (A/B of compile-time kernel variants in
    # one GPU session; tools/gpu_variant_ab.sh); never set by the product path
    alt = os.environ.get("DQ_GPU_LIB")
    return _need(alt if alt else GPU_LIB)


def synth_lib_path() -> str:
    if not os.path.exists(SYNTH_LIB):
        subprocess.run(["make", "-s", "-C", CSRC, os.path.join("..", "_build", "libdisq_synth.so")],
                       check=True)
    return _need(SYNTH_LIB)
