"""A/B of the news scoring kernels across commits (news.hip of each commit built alone).

    python tools/bisect_news.py --build C1 C2 ...            # CPU: tools/bisect/libnews_<C>.so
    python tools/bisect_news.py --build wt:NAME[:FLAG,FLAG]  # the working tree's news.hip with -D flags
    python tools/bisect_news.py [--dtype fp32|bf16] [--B N] [--d 256 --n-news 65238] C1 C2 ...   # GPU

Every version runs the same inputs (config 3: L=50, K=32, d=768, C=40, 104k-row table) through its
own precompute and scoring entry points in one process, reps interleaved; prints the median ms per
scoring launch and the largest score difference against the first commit.
"""
import argparse
import ctypes
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "bisect")


def build(commits):
    sys.path.insert(0, ROOT)
    from miner_amd.build import hipcc
    for c in commits:
        if c.startswith("wt:"):
            parts = c.split(":")
            name, flags = parts[1], (["-D" + f for f in parts[2].split(",")] if len(parts) > 2 and parts[2] else [])
            os.makedirs(OUT, exist_ok=True)
            lib = os.path.join(OUT, f"libnews_{name}.so")
            subprocess.run([hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wno-pass-failed",
                            *flags, "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "miner_amd", "csrc", "news.hip"),
                            "-o", lib], check=True)
            print("built", lib, flush=True)
            continue
        src = os.path.join("/tmp", "bisect_news", c)
        for sub in ("miner_amd/csrc", "include"):
            os.makedirs(os.path.join(src, sub), exist_ok=True)
        files = subprocess.run(["git", "-C", ROOT, "ls-tree", "--name-only", c, "include/"], capture_output=True,
                               text=True, check=True).stdout.split()
        for f in files + ["miner_amd/csrc/news.hip", "miner_amd/csrc/cdna4_common.h"]:
            r = subprocess.run(["git", "-C", ROOT, "show", f"{c}:{f}"], capture_output=True)
            if r.returncode == 0:
                with open(os.path.join(src, f), "wb") as fh:
                    fh.write(r.stdout)
        os.makedirs(OUT, exist_ok=True)
        lib = os.path.join(OUT, f"libnews_{c}.so")
        subprocess.run([hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wno-pass-failed",
                        "-I", os.path.join(src, "include"), os.path.join(src, "miner_amd", "csrc", "news.hip"),
                        "-o", lib], check=True)
        print("built", lib, flush=True)


def run(commits, dtype, B, reps, d=768, n_news=104000):
    import torch
    sys.path.insert(0, ROOT)
    from miner_amd import ops, synthetic
    P, I = ctypes.c_void_p, ctypes.c_int
    dev = "cuda:0"
    L, C, K, Dc = 50, 40, 32, 200
    dt = torch.float32 if dtype == "fp32" else torch.bfloat16
    code = 0 if dtype == "fp32" else 1
    g = torch.Generator(device=dev).manual_seed(36)
    table = (torch.randn((n_news, d), generator=g, device=dev) / d ** 0.5).to(dt)
    lens = torch.randint(0, L + 1, (B,), generator=g, device=dev)
    mask = torch.arange(L, device=dev)[None, :] >= (L - lens)[:, None]
    hid = torch.randint(1, n_news, (B, L), generator=g, device=dev, dtype=torch.int32)
    hid[~mask] = 0
    cid = torch.randint(1, n_news, (B, C), generator=g, device=dev, dtype=torch.int32)
    W1, Q, W2 = synthetic.init_weights(36, d, Dc, K, device=dev)
    pw = ops.pack_weights(W1, Q, W2, dtype=dt)          # the packed layout is the same in every commit
    m8 = mask.contiguous().view(torch.uint8)
    st = torch.cuda.current_stream().cuda_stream
    runs = {}
    for c in commits:
        h = ctypes.CDLL(os.path.join(OUT, f"libnews_{c.split(':')[1] if c.startswith('wt:') else c}.so"))
        h.miner_news_precompute.argtypes = [P, I, P, I, P, I, I, I, P, P]
        h.miner_score_news.argtypes = [P, I, I, P, P, P, I, P, P, P, P, P, I, I, I, I, I, P, P]
        logits = torch.empty((n_news, K), device=dev)
        proj = torch.empty_like(table)
        assert h.miner_news_precompute(st, code, table.data_ptr(), n_news, pw.buf.data_ptr(), d, Dc, K,
                                       logits.data_ptr(), proj.data_ptr()) == 0
        runs[c] = (h, logits, proj, torch.empty((B, C), device=dev))

    def launch(c):
        h, logits, proj, out = runs[c]
        rc = h.miner_score_news(st, code, 0, table.data_ptr(), logits.data_ptr(), proj.data_ptr(), n_news,
                                hid.data_ptr(), m8.data_ptr(), None, cid.data_ptr(), None, B, L, C, d, K,
                                out.data_ptr(), None)
        assert rc == 0, rc

    for c in commits:
        launch(c)
    torch.cuda.synchronize()
    times = {c: [] for c in commits}
    for _ in range(reps):
        for c in commits:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            launch(c)
            b.record()
            torch.cuda.synchronize()
            times[c].append(a.elapsed_time(b))
    ref = runs[commits[0]][3]
    for c in commits:
        diff = float((runs[c][3] - ref).abs().max())
        print(f"{dtype} B={B} {c}: {statistics.median(times[c]):.3f} ms (min {min(times[c]):.3f}, "
              f"per 131k {statistics.median(times[c]) * 131072 / B:.3f}), max |score - {commits[0]}| {diff:.2e}",
              flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--B", type=int, default=1000000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--n-news", type=int, default=104000)
    ap.add_argument("commits", nargs="+")
    a = ap.parse_args()
    if a.build:
        build(a.commits)
    else:
        run(a.commits, a.dtype, a.B, a.reps, a.d, a.n_news)
