"""Per-wave stage cycles of the fp32 news scoring kernel (diagnostic build with -DMINER_STAMPS).

    python tools/news_stages.py --build                 # -> miner_amd/libminer_hip_stamps.so (CPU ok)
    python tools/news_stages.py [--batch 32768]         # on the GPU; MINER_NEWS_F32X6=1 for the bf16x6 form

Lane 0 of each wave sums s_memtime deltas between the stage marks of news_score32 (the stamps cost
a few instructions each and make every mark wait for outstanding LDS reads: read the SHARES).
Reported as shader cycles per impression per workgroup (one workgroup per CU).
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
STAGES = ["vm_wait (row DMAs)", "barrier", "item start / softmax / aux", "DMA issue",
          "history product", "gelu + split", "candidate product", "pass end + loop"]
STAGESX2 = ["vm_wait (row DMAs)", "barrier", "item/S7/softmax/aux+LDS rd", "DMA issue",
            "history product", "scale + gelu + split", "candidate product", "pass end + loop"]
STAGES16 = ["slot wait + barrier", "item start rest / aux", "softmax phases", "DMA issue", "history product",
            "gelu + frag", "cand product + pass end", "S7"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--batch", type=int, default=32768)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16", "x2"])
    ap.add_argument("--d", type=int, default=768, help="embedding dim (256 with --n-news 65238: config 2)")
    ap.add_argument("--n-news", type=int, default=104000)
    ap.add_argument("--lib", default=None, help="a stamps library built with extra flags (default: the stamps build)")
    ap.add_argument("--flags", default="", help="--build: extra -D flags, comma separated (with --lib as the output)")
    args = ap.parse_args()
    import stage_profile
    if args.build:
        extra = ["-D" + f for f in args.flags.split(",") if f]
        stage_profile.build(extra, out=args.lib or stage_profile.STAMP_LIB)
        return
    os.environ["MINER_HIP_LIB"] = args.lib or stage_profile.STAMP_LIB
    import torch
    from miner_amd import _lib, news, ops, synthetic
    x2 = args.dtype == "x2"
    if x2:
        args.dtype = "fp32"
    fn = _lib.lib().miner_news_x2_debug_stage_cycles if x2 else _lib.lib().miner_news_debug_stage_cycles
    fn.argtypes = [ctypes.c_void_p]
    fn.restype = ctypes.c_int
    dev = "cuda:0"
    B, n_news, L, C, d, K, Dc = args.batch, args.n_news, 50, 40, args.d, 32, 200
    g = torch.Generator(device=dev).manual_seed(36)
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    table = (torch.randn((n_news, d), generator=g, device=dev) / d ** 0.5).to(dt)
    lens = torch.randint(0, L + 1, (B,), generator=g, device=dev)
    mask = torch.arange(L, device=dev)[None, :] >= (L - lens)[:, None]
    hid = torch.randint(1, n_news, (B, L), generator=g, device=dev, dtype=torch.int32)
    hid[~mask] = 0
    cid = torch.randint(1, n_news, (B, C), generator=g, device=dev, dtype=torch.int32)
    W1, Q, W2 = synthetic.init_weights(36, d, Dc, K, device=dev)
    nt = news.precompute(table, ops.pack_weights(W1, Q, W2, dtype=dt), x2=x2)
    news.score(nt, hid, mask, cid, validate=False, x2=x2)
    out = (ctypes.c_ulonglong * 65)()
    fn(out)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 3
    a.record()
    for _ in range(reps):
        news.score(nt, hid, mask, cid, validate=False, x2=x2)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    assert fn(out) == 0
    n = out[64]
    kind = "fp32 news_score_x2 (fp16 pairs)" if x2 else "bf16 news_score" if args.dtype == "bf16" else \
        f"fp32 news_score32 ({'bf16x6' if os.environ.get('MINER_NEWS_F32X6') else 'fp32 MFMA'})"
    print(f"{kind} B={B} d={d}: "
          f"{ms:.3f} ms/launch ({ms / B * 131072:.2f} ms per 131k), cycles per impression per workgroup:")
    print(f"  {'stage':28s}" + "".join(f"  wave{w}" for w in range(8)))
    names = STAGES16 if args.dtype == "bf16" else STAGES
    if x2:
        names = STAGESX2
    elif args.dtype == "fp32" and not os.environ.get("MINER_NEWS_F32X6"):
        names = STAGES[:4] + ["S7", "in-wave softmax", "products (history + candidate)", STAGES[7]]
    for i, name in enumerate(names):
        print(f"  {name:28s}" + "".join(f" {out[8 * w + i] / n:6.0f}" for w in range(8)))
    print(f"  {'total':28s}" + "".join(f" {sum(out[8 * w + i] for i in range(8)) / n:6.0f}" for w in range(8)))


if __name__ == "__main__":
    main()
