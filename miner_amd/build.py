"""Build libminer_hip.so (the HIP/CDNA4 scoring kernels + C ABI) in-tree for gfx950.

    python -m miner_amd.build            # -> miner_amd/libminer_hip.so

hipcc cross-compiles for gfx950 without a GPU, so this runs in the build container; the .so then
travels with the repo snapshot to the GPU box (it is git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "miner_score.hip")      # the fused scoring kernel
SOURCES = [SRC, os.path.join(HERE, "csrc", "miner_metrics.hip"), os.path.join(HERE, "csrc", "fastformer.hip"),
           os.path.join(HERE, "csrc", "corpus.hip"), os.path.join(HERE, "csrc", "news.hip")]
HEADERS = [os.path.join(ROOT, "include", h) for h in ("miner_score.h", "miner_metrics.h", "miner_fastformer.h", "miner_corpus.h", "miner_news.h")] + [os.path.join(HERE, "csrc", "cdna4_common.h")]
LIB = os.path.join(HERE, "libminer_hip.so")
ARCH = os.environ.get("MINER_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc"), shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libminer_hip.so)")


DEBUG_LIB = os.path.join(HERE, "libminer_hip_dbg.so")


def build_library(force: bool = False, verbose: bool = False, debug: bool = False) -> str:
    """Compile csrc/*.hip -> miner_amd/libminer_hip.so (skipped when up to date).

    ``debug`` builds the diagnostic variant libminer_hip_dbg.so instead (-DMINER_NEWS_DEBUG:
    every DMA / store address of the news kernel is range-checked and violations are printed;
    load it with MINER_HIP_LIB=miner_amd/libminer_hip_dbg.so)."""
    lib = DEBUG_LIB if debug else LIB
    deps = SOURCES + HEADERS
    if not force and os.path.exists(lib) and all(os.path.getmtime(lib) >= os.path.getmtime(p) for p in deps):
        return lib
    tmp = lib + f".tmp{os.getpid()}"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wno-pass-failed", *(["-DMINER_NEWS_DEBUG"] if debug else []),
           "-I", os.path.join(ROOT, "include"), *SOURCES, "-o", tmp]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"hipcc failed ({res.returncode}):\n{res.stderr[-4000:]}")
    os.replace(tmp, lib)
    return lib


if __name__ == "__main__":
    print(build_library(force="--force" in sys.argv, verbose=True, debug="--debug" in sys.argv))
