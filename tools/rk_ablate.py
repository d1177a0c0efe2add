"""Config-5 ranker (rk_fused<fp16>) stage ablation: corpus.hip built with -DMINER_RK_ABL=<bits>
(1 no DMAs, 2 no MFMAs, 4 no epilogue / top-k, 8 no per-chunk barrier; results wrong, time only),
every build timed interleaved in one process on the same inputs (2048 users x 200k news, K=64, d=768).

    python tools/rk_ablate.py --build 0 1 2 4 5 6 7 8     # CPU: tools/bisect/librk_abl<bits>.so
    python tools/rk_ablate.py 0 1 2 4 5 6 7 8 16s          # GPU; a trailing "s": the split form
                                                           # (miner_rank_topk_ws, MINER_RK_SPLIT=1);
                                                           # "g": the 64-byte 4-stage geometry;
                                                           # "<bits>n" builds without SLP vectorizing
"""
import ctypes
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "bisect")
sys.path.insert(0, ROOT)


def build(variants, extra=()):
    """variant "<bits>" or "<bits>w<W>" (-DMINER_RK_DMAW=W: the next chunk's DMAs within the first W
    MFMA pairs of a chunk)"""
    from miner_amd.build import hipcc
    os.makedirs(OUT, exist_ok=True)
    for v in variants:
        lib = os.path.join(OUT, f"librk_abl{v}.so")
        v = str(v)
        noslp = ["-fno-slp-vectorize"] if "n" in v else []    # "<bits>n": without the SLP vectorizer
        # "<bits>i" / "<bits>m": the max-ILP / max-memory-clause machine scheduler
        sched = [f for c, f in (("i", "max-ilp"), ("m", "max-memory-clause")) if c in v]
        noslp += ["-mllvm", f"-amdgpu-sched-strategy={sched[0]}"] if sched else []
        bits, _, w = v.rstrip("nim").partition("w")
        wdef = [f"-DMINER_RK_DMAW={w}", *noslp] if w else noslp
        subprocess.run([hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wno-pass-failed",
                        f"-DMINER_RK_ABL={bits}", *wdef, *extra, "-I", os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "miner_amd", "csrc", "corpus.hip"), "-o", lib], check=True)
        print("built", lib, flush=True)


def run(variants, U=2048, N=200000, reps=3):
    import torch
    P, I = ctypes.c_void_p, ctypes.c_int
    dev = "cuda:0"
    K, d, topk = 64, 768, 100
    g = torch.Generator(device=dev).manual_seed(5)
    table = (torch.randn((N, d), generator=g, device=dev) / d ** 0.5).half()
    mui = (torch.randn((U, K, d), generator=g, device=dev) / 4).half()
    proj = (torch.randn((U, K, d), generator=g, device=dev) / 4).half()
    ts = torch.empty(U, topk, device=dev)
    ti = torch.empty(U, topk, device=dev, dtype=torch.int32)
    st = torch.cuda.current_stream().cuda_stream
    ws = torch.empty(U * 8 * topk * 8, dtype=torch.uint8, device=dev)
    os.environ["MINER_RK_SPLIT"] = "1"
    libs = {}
    for v in variants:
        h = ctypes.CDLL(os.path.join(OUT, f"librk_abl{v.rstrip('sg')}.so"))
        h.miner_rank_topk_ws.argtypes = [P, I, I, P, P, P, I, I, I, I, I, P, P, P, ctypes.c_size_t]
        libs[v] = h

    def launch(v):
        os.environ["MINER_RK_GEO"] = "1" if "g" in v else "0"
        rc = libs[v].miner_rank_topk_ws(st, 2, 0, mui.data_ptr(), proj.data_ptr(), table.data_ptr(), U, N, d, K, topk,
                                        ts.data_ptr(), ti.data_ptr(), ws.data_ptr() if v.endswith("s") else None,
                                        ws.numel() if v.endswith("s") else 0)
        assert rc == 0, rc

    times = {v: [] for v in variants}
    first = {}
    for v in variants:
        launch(v)
        torch.cuda.synchronize()
        first[v] = (ts.clone(), ti.clone())
    torch.cuda.synchronize()
    for _ in range(reps):
        for v in variants:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            launch(v)
            b.record()
            torch.cuda.synchronize()
            times[v].append(a.elapsed_time(b))
    fl = U * N * 4 * K * d
    for v in variants:
        t = statistics.median(times[v])
        same = bool(torch.equal(first[v][0], first[variants[0]][0]) and torch.equal(first[v][1], first[variants[0]][1]))
        print(f"ABL={v:>3s}: {t:8.2f} ms  ({fl / t / 1e9 / 2500:.3f} of fp16 peak)  all {[round(x, 1) for x in times[v]]}"
              f"  top-k identical to {variants[0]}: {same}", flush=True)


if __name__ == "__main__":
    args = sys.argv[1:]
    if args and args[0] == "--build":
        build(args[1:])
    else:
        run(args)
