"""Ablation timing of the fp32 news scoring kernel: which phase the time goes to.

    python tools/news_ablate.py --build          # CPU: miner_amd/libminer_hip_abl.so (experiment bits on)
    python tools/news_ablate.py [--B 262144]     # GPU: one process, variants interleaved

Each variant sets MINER_NEWS_ABL (news.hip news_score32: 1 no wave priority, 2 no row DMAs, 4 no
compute, 8 no GELU, 16 candidate product as VALU adds, 32 history product skipped; "x6" variants:
the bf16x6 form, MINER_NEWS_F32X6=1); the timing
variants produce wrong scores by design. Prints the median ms per launch and per 131k impressions.
"""
import argparse
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "miner_amd", "libminer_hip_abl.so")
VARIANTS = [("full", 0), ("no prio", 1), ("no row DMA", 2), ("no compute", 4), ("no GELU", 8),
            ("no cand MFMA", 16), ("no hist MFMA", 32), ("DMA only on 8 waves", 64),
            ("no DMA, no compute", 6), ("no DMA, no hist", 34), ("no DMA, no cand", 18),
            ("no DMA, no MFMA", 50), ("x6 full", "x6:0"), ("x6 no compute", "x6:4"), ("x6 no DMA", "x6:2"),
            ("x6 no cand", "x6:16"), ("x6 no hist", "x6:32"), ("x6 no GELU", "x6:8")]
if os.environ.get("ABLATE_SET") == "s7":         # S7 placement: second pair (4096), mui waves (128)
    VARIANTS = [("full", 0), ("S7 at pair 1", 4096), ("S7 on waves 0-3", 128), ("S7 pair 1, waves 0-3", 4224),
                ("no S7 prio", 1), ("S7 pair 1, no prio", 4097)]


def build():
    sys.path.insert(0, ROOT)
    from miner_amd.build import hipcc, SOURCES, ARCH
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wno-pass-failed",
           "-DMINER_NEWS_ABL_MASK=0x7fffffff", "-I", os.path.join(ROOT, "include"), *SOURCES, "-o", LIB]
    subprocess.run(cmd, check=True)
    print("built", LIB)


def run(B, reps):
    os.environ["MINER_HIP_LIB"] = LIB
    sys.path.insert(0, ROOT)
    import torch
    from miner_amd import news, ops, synthetic
    dev = "cuda:0"
    n_news, L, C, d, K, Dc = 104000, 50, 40, 768, 32, 200
    g = torch.Generator(device=dev).manual_seed(36)
    table = torch.randn((n_news, d), generator=g, device=dev) / d ** 0.5
    lens = torch.randint(0, L + 1, (B,), generator=g, device=dev)
    mask = torch.arange(L, device=dev)[None, :] >= (L - lens)[:, None]
    hid = torch.randint(1, n_news, (B, L), generator=g, device=dev, dtype=torch.int32)
    hid[~mask] = 0
    cid = torch.randint(1, n_news, (B, C), generator=g, device=dev, dtype=torch.int32)
    W1, Q, W2 = synthetic.init_weights(36, d, Dc, K, device=dev)
    nt = news.precompute(table, ops.pack_weights(W1, Q, W2, dtype=torch.float32))
    times = {v: [] for v, _ in VARIANTS}
    for rep in range(reps + 1):
        for name, bits in VARIANTS:
            if isinstance(bits, str):
                os.environ["MINER_NEWS_F32X6"] = "1"
                bits = int(bits.split(":")[1])
            else:
                os.environ.pop("MINER_NEWS_F32X6", None)
            os.environ["MINER_NEWS_ABL"] = str(bits)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            news.score(nt, hid, mask, cid, validate=False)
            b.record()
            torch.cuda.synchronize()
            if rep:
                times[name].append(a.elapsed_time(b))
    base = statistics.median(times["full"])
    for name, _ in VARIANTS:
        m = statistics.median(times[name])
        print(f"{name:22s} {m:8.3f} ms  per 131k {m * 131072 / B:7.3f}  ({m / base:5.3f} of full)", flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--B", type=int, default=262144)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    if a.build:
        build()
    else:
        run(a.B, a.reps)
