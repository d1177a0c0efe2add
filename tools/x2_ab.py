"""Interleaved A/B of news_score_x2 builds (news_x2.hip of a commit or of the working tree with
extra flags, each built alone): the same precomputed tables and impressions (config 3 shape, the
bench's synthetic ids), median ms per launch and max |score difference| against the first build.

    python tools/x2_ab.py --build NAME [REV|-] [FLAGS...]   # CPU: tools/bisect/libx2_NAME.so
    python tools/x2_ab.py NAME1 NAME2 ... [--B N]          # GPU (X2AB_LOSS=1: with the disagreement;
                                                          # NAME@loss: that entry alone with it)
"""
import ctypes
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "bisect")
sys.path.insert(0, ROOT)


def build(name, rev="-", *flags):
    from miner_amd.build import hipcc
    src = os.path.join(ROOT, "miner_amd", "csrc", "news_x2.hip")
    inc = os.path.join(ROOT, "include")
    if rev != "-":
        d = os.path.join("/tmp", "x2_ab", rev)
        for sub in ("miner_amd/csrc", "include"):
            os.makedirs(os.path.join(d, sub), exist_ok=True)
        for f in ["miner_amd/csrc/news_x2.hip", "miner_amd/csrc/cdna4_common.h", "include/miner_news.h",
                  "include/miner_score.h"]:
            with open(os.path.join(d, f), "wb") as fh:
                fh.write(subprocess.run(["git", "-C", ROOT, "show", f"{rev}:{f}"], capture_output=True, check=True).stdout)
        src, inc = os.path.join(d, "miner_amd", "csrc", "news_x2.hip"), os.path.join(d, "include")
    os.makedirs(OUT, exist_ok=True)
    lib = os.path.join(OUT, f"libx2_{name}.so")
    subprocess.run([hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wno-pass-failed",
                    *flags, "-I", inc, src, "-o", lib], check=True)
    print("built", lib, flush=True)


def run(names, B=1_000_000, reps=5, d=768, n_news=104000):
    import torch
    from miner_amd import news, ops, synthetic
    P, I = ctypes.c_void_p, ctypes.c_int
    dev = "cuda:0"
    L, C, K, Dc = 50, 40, 32, 200
    table = synthetic.news_table(3, n_news, d, device=dev)
    beh = synthetic.behaviors(3, 0, B, L=L, n_news=n_news, C=C, device=dev)
    W1, Q, W2 = synthetic.init_weights(3, d, Dc, K, device=dev)
    nt = news.precompute(table, ops.pack_weights(W1, Q, W2, dtype=torch.float32), x2=True)
    mask = beh.his_mask.contiguous().view(torch.uint8)
    st = torch.cuda.current_stream().cuda_stream
    libs = {}
    for n in names:
        h = ctypes.CDLL(os.path.join(OUT, f"libx2_{n.split('@')[0]}.so"))
        h.miner_score_news_x2.argtypes = [P, I, P, P, P, P, P, I, P, P, P, P, P, I, I, I, I, I, P, P, P]
        libs[n] = h
    out = {n: torch.empty(B * C, device=dev) for n in names}
    loss_all = os.environ.get("X2AB_LOSS") == "1"      # with the eval loss's disagreement output
    lossn = {n: loss_all or n.endswith("@loss") for n in names}
    dis = {n: torch.empty(B, device=dev) for n in names}

    def launch(n):
        loss = lossn[n]
        px = nt.x2
        rc = libs[n].miner_score_news_x2(st, 0, px.table2.data_ptr(), px.table_unit.data_ptr(), nt.logits.data_ptr(),
                                         px.proj2.data_ptr(), px.proj_unit.data_ptr(), n_news, beh.his_ids.data_ptr(),
                                         mask.data_ptr(), None, beh.cand_ids.data_ptr(), None, B, L, C, d, K,
                                         out[n].data_ptr(), None, dis[n].data_ptr() if loss else None)
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
        diff = float((out[n] - out[names[0]]).abs().max())
        if lossn[n] and lossn[names[0]]:
            diff = max(diff, float((dis[n] - dis[names[0]]).abs().max()))
        t = statistics.median(times[n])
        print(f"{n}: {t:.3f} ms per {B} impressions ({B * C / t / 1e3:.1f} M pairs/s), all "
              f"{[round(x, 2) for x in times[n]]}, max |diff vs {names[0]}| {diff:.2e}", flush=True)


if __name__ == "__main__":
    a = sys.argv[1:]
    if a and a[0] == "--build":
        build(*a[1:])
    else:
        B, d, nn = 1_000_000, 768, 104000
        for flag in ("--B", "--d", "--n-news"):
            if flag in a:
                i = a.index(flag)
                v = int(a[i + 1])
                a = a[:i] + a[i + 2:]
                if flag == "--B":
                    B = v
                elif flag == "--d":
                    d = v
                else:
                    nn = v
        run(a, B, d=d, n_news=nn)
