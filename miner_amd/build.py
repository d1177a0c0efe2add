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
           os.path.join(HERE, "csrc", "corpus.hip"), os.path.join(HERE, "csrc", "news.hip"),
           os.path.join(HERE, "csrc", "miner_auc.hip"), os.path.join(HERE, "csrc", "wide.hip"),
           os.path.join(HERE, "csrc", "news_x2.hip")]
HEADERS = [os.path.join(ROOT, "include", h) for h in ("miner_score.h", "miner_metrics.h", "miner_fastformer.h", "miner_corpus.h", "miner_news.h", "miner_wide.h")] + [os.path.join(HERE, "csrc", "cdna4_common.h")]
LIB = os.path.join(HERE, "libminer_hip.so")
ARCH = os.environ.get("MINER_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc"), shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libminer_hip.so)")


DEBUG_LIB = os.path.join(HERE, "libminer_hip_dbg.so")


# per-file flags, each from an interleaved A/B on the box: hipcc's SLP vectorizer packs scalar fp32
# work of these kernels into v_pk_* ops on operands in non-adjacent registers, and the v_mov pairs
# it adds to gather them cost more VALU issue than the packing saves (profiles/r05_*_noslp_ab.txt);
# news_x2.hip under the max-ILP machine scheduler: -0.54 % on the headline kernel, bit-identical
# (profiles/r05_sched_strategy_ab.txt; the same strategy costs FastFormer +2.8 %)
FILE_FLAGS = {"fastformer.hip": ["-fno-slp-vectorize"],
              "news_x2.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]}


def _flags(debug: bool) -> list:
    return [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wno-pass-failed",
            *(["-DMINER_NEWS_DEBUG"] if debug else []), "-I", os.path.join(ROOT, "include")]


def _stamp(debug: bool) -> str:
    """Build configuration an object / the library was made with: the target, the flags and the
    hipcc version. Objects and the library are reused only when it matches."""
    try:
        ver = subprocess.run([hipcc(), "--version"], capture_output=True, text=True, timeout=60).stdout.strip()
    except (OSError, subprocess.SubprocessError, RuntimeError):
        ver = "unknown"
    return "\n".join([" ".join(_flags(debug)), repr(sorted(FILE_FLAGS.items())), ver])


def _objdir(debug: bool) -> str:
    import hashlib
    tag = hashlib.sha1(_stamp(debug).encode()).hexdigest()[:12]
    return os.path.join(ROOT, "build", ("obj_dbg_" if debug else "obj_") + ARCH + "_" + tag)


def build_library(force: bool = False, verbose: bool = False, debug: bool = False, jobs: int = None) -> str:
    """Compile csrc/*.hip -> miner_amd/libminer_hip.so (skipped when up to date).

    Each translation unit is compiled to its own object in parallel (non-rdc HIP: every object
    carries and registers its own gfx950 code object), then linked; an object is rebuilt when its
    source or any shared header is newer.

    ``debug`` builds the diagnostic variant libminer_hip_dbg.so instead (-DMINER_NEWS_DEBUG:
    every DMA / store address of the news kernel is range-checked and violations are printed;
    load it with MINER_HIP_LIB=miner_amd/libminer_hip_dbg.so)."""
    from concurrent.futures import ThreadPoolExecutor
    lib = DEBUG_LIB if debug else LIB
    deps = SOURCES + HEADERS
    od = _objdir(debug)
    stamp_file = lib + ".buildcfg"
    stamp_ok = os.path.exists(stamp_file) and open(stamp_file).read() == os.path.basename(od)
    if not force and stamp_ok and os.path.exists(lib) and \
            all(os.path.getmtime(lib) >= os.path.getmtime(p) for p in deps):
        return lib
    os.makedirs(od, exist_ok=True)
    hdr_t = max(os.path.getmtime(h) for h in HEADERS)
    flags = _flags(debug)

    def compile_one(src):
        obj = os.path.join(od, os.path.basename(src)[:-4] + ".o")
        if not force and os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), hdr_t):
            return obj
        tmp = obj + f".tmp{os.getpid()}"
        cmd = [hipcc(), *flags, *FILE_FLAGS.get(os.path.basename(src), []), "-c", src, "-o", tmp]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"hipcc failed on {os.path.basename(src)} ({res.returncode}):\n{res.stderr[-4000:]}")
        os.replace(tmp, obj)
        return obj

    jobs = jobs or min(len(SOURCES), max(1, (os.cpu_count() or 4) // 2))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    tmp = lib + f".tmp{os.getpid()}"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"link failed ({res.returncode}):\n{res.stderr[-4000:]}")
    os.replace(tmp, lib)
    with open(stamp_file, "w") as f:
        f.write(os.path.basename(od))
    return lib


ASAN_DRIVER = os.path.join(ROOT, "tests", "native", "abi_errors.cpp")


def build_asan_driver(force: bool = False, verbose: bool = False) -> str:
    """Every csrc/*.hip with AddressSanitizer on its HOST code (``-Xarch_host -fsanitize=address``;
    the gfx950 device code is built as usual and never runs), linked with
    tests/native/abi_errors.cpp into build/asan/abi_errors: a CPU program that drives the
    argument-error paths of every C-ABI entry point (SURVEY §5 sanitizer builds; run by
    tests/test_asan_abi.py). GPU-side sanitizers are not available on this pool."""
    from concurrent.futures import ThreadPoolExecutor
    od = os.path.join(ROOT, "build", "asan")
    exe = os.path.join(od, "abi_errors")
    deps = SOURCES + HEADERS + [ASAN_DRIVER]
    if not force and os.path.exists(exe) and all(os.path.getmtime(exe) >= os.path.getmtime(p) for p in deps):
        return exe
    os.makedirs(od, exist_ok=True)
    flags = [f"--offload-arch={ARCH}", "-O1", "-g", "-Xarch_host", "-fsanitize=address", "-fno-omit-frame-pointer",
             "-std=c++17", "-Wno-pass-failed", "-I", os.path.join(ROOT, "include")]

    def compile_one(src):
        obj = os.path.join(od, os.path.splitext(os.path.basename(src))[0] + ".o")
        if not force and os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(p) for p in [src] + HEADERS):
            return obj
        lang = ["-x", "hip"] if src.endswith(".hip") else ["-x", "c++"]
        cmd = [hipcc(), *flags, *lang, "-c", src, "-o", obj + ".tmp"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"asan build failed on {os.path.basename(src)}:\n{res.stderr[-4000:]}")
        os.replace(obj + ".tmp", obj)
        return obj

    with ThreadPoolExecutor(min(len(SOURCES) + 1, max(1, (os.cpu_count() or 4) // 2))) as ex:
        objs = list(ex.map(compile_one, SOURCES + [ASAN_DRIVER]))
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-fsanitize=address", *objs, "-o", exe + ".tmp"]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"asan link failed:\n{res.stderr[-4000:]}")
    os.replace(exe + ".tmp", exe)
    return exe


if __name__ == "__main__":
    if "--asan" in sys.argv:
        print(build_asan_driver(force="--force" in sys.argv, verbose=True))
    else:
        print(build_library(force="--force" in sys.argv, verbose=True, debug="--debug" in sys.argv))
