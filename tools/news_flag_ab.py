"""bf16 news-path kernel builds A/B (news.hip alone with extra -D / compiler flags), interleaved in one
process on the same precomputed table (the main library's miner_news_precompute): median ms per
launch of miner_score_news and the max score difference against the first build.

    python tools/news_flag_ab.py --build NAME [FLAGS...]                 # CPU: tools/bisect/libnews_NAME.so
    python tools/news_flag_ab.py [--cfg 3|2] [--B N] NAME1 NAME2 ...     # GPU (config 3: d 768, 104k news;
                                                                         #      config 2: d 256, 65,238 news)
    python tools/news_flag_ab.py --pre NAME1 NAME2 ...                   # GPU: the fp32 precompute, config 3
"""
import argparse
import ctypes
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "bisect")
sys.path.insert(0, ROOT)


def build(name, *flags):
    from miner_amd.build import hipcc
    os.makedirs(OUT, exist_ok=True)
    lib = os.path.join(OUT, f"libnews_{name}.so")
    subprocess.run([hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wno-pass-failed",
                    *flags, "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "miner_amd", "csrc", "news.hip"),
                    "-o", lib], check=True)
    print("built", lib, flush=True)


def run_pre(names, reps=9):
    """fp32 per-news precompute (miner_news_precompute) of the config-3 table, 104,000 x 768: median ms
    per call and max |logits / proj difference| against the first build."""
    import torch
    from miner_amd import ops, synthetic
    P, I = ctypes.c_void_p, ctypes.c_int
    dev = "cuda:0"
    d, n_news, Dc, K = 768, 104000, 200, 32
    g = torch.Generator(device=dev).manual_seed(36)
    table = torch.randn((n_news, d), generator=g, device=dev) / d ** 0.5
    W1, Q, W2 = synthetic.init_weights(36, d, Dc, K, device=dev)
    pw = ops.pack_weights(W1, Q, W2, dtype=torch.float32)
    st = torch.cuda.current_stream().cuda_stream
    libs, lg, pj = {}, {}, {}
    for n in names:
        h = ctypes.CDLL(os.path.join(OUT, f"libnews_{n}.so"))
        h.miner_news_precompute.argtypes = [P, I, P, I, P, I, I, I, P, P]
        libs[n] = h
        lg[n] = torch.empty((n_news, K), device=dev)
        pj[n] = torch.empty((n_news, d), device=dev)

    def launch(n):
        rc = libs[n].miner_news_precompute(st, 0, table.data_ptr(), n_news, pw.buf.data_ptr(), d, Dc, K,
                                           lg[n].data_ptr(), pj[n].data_ptr())
        assert rc == 0, rc

    times = {n: [] for n in names}
    for n in names:
        launch(n)
    torch.cuda.synchronize()
    for _ in range(reps):
        for n in names:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            launch(n)
            b.record()
            torch.cuda.synchronize()
            times[n].append(a.elapsed_time(b))
    for n in names:
        dl = float((lg[n] - lg[names[0]]).abs().max() / lg[names[0]].abs().max())
        dp = float((pj[n] - pj[names[0]]).abs().max() / pj[names[0]].abs().max())
        print(f"{n}: precompute {statistics.median(times[n]):.3f} ms, max |diff vs {names[0]}| / max: logits {dl:.2e}, "
              f"proj {dp:.2e}", flush=True)


def run(names, cfg=3, B=None, reps=9):
    import torch
    from miner_amd import news, ops, synthetic
    P, I = ctypes.c_void_p, ctypes.c_int
    dev = "cuda:0"
    d, n_news = (768, 104000) if cfg == 3 else (256, 65238)
    B = B or (1_000_000 if cfg == 3 else 50_000)
    L, C, K, Dc = 50, 40, 32, 200
    g = torch.Generator(device=dev).manual_seed(36)
    table = (torch.randn((n_news, d), generator=g, device=dev) / d ** 0.5).to(torch.bfloat16)
    lens = torch.randint(0, L + 1, (B,), generator=g, device=dev)
    mask = (torch.arange(L, device=dev)[None, :] >= (L - lens)[:, None])
    hid = torch.randint(1, n_news, (B, L), generator=g, device=dev, dtype=torch.int32)
    hid[~mask] = 0
    cid = torch.randint(1, n_news, (B, C), generator=g, device=dev, dtype=torch.int32)
    W1, Q, W2 = synthetic.init_weights(36, d, Dc, K, device=dev)
    nt = news.precompute(table, ops.pack_weights(W1, Q, W2, dtype=torch.bfloat16))
    m8 = mask.contiguous().view(torch.uint8)
    st = torch.cuda.current_stream().cuda_stream
    libs = {}
    for n in names:
        h = ctypes.CDLL(os.path.join(OUT, f"libnews_{n}.so"))
        h.miner_score_news.argtypes = [P, I, I, P, P, P, I, P, P, P, P, P, I, I, I, I, I, P, P]
        libs[n] = h
    out = {n: torch.empty((B, C), device=dev) for n in names}

    def launch(n):
        rc = libs[n].miner_score_news(st, 1, 0, nt.table.data_ptr(), nt.logits.data_ptr(), nt.proj.data_ptr(), n_news,
                                      hid.data_ptr(), m8.data_ptr(), None, cid.data_ptr(), None, B, L, C, d, K,
                                      out[n].data_ptr(), None)
        assert rc == 0, rc

    times = {n: [] for n in names}
    for n in names:
        launch(n)
    torch.cuda.synchronize()
    for _ in range(reps):
        for n in names:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            launch(n)
            b.record()
            torch.cuda.synchronize()
            times[n].append(a.elapsed_time(b))
    for n in names:
        ms = statistics.median(times[n])
        print(f"config {cfg} {n}: {ms:.3f} ms per {B} impressions ({B * C / ms / 1e6:.2f} G pairs/s), "
              f"max |score - {names[0]}| {float((out[n] - out[names[0]]).abs().max()):.2e}", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--build":
        build(*sys.argv[2:])
    else:
        ap = argparse.ArgumentParser()
        ap.add_argument("--cfg", type=int, default=3)
        ap.add_argument("--B", type=int, default=None)
        ap.add_argument("--pre", action="store_true", help="time the fp32 precompute instead of the scoring kernel")
        ap.add_argument("names", nargs="+")
        a = ap.parse_args()
        if a.pre:
            run_pre(a.names)
        else:
            run(a.names, a.cfg, a.B)
