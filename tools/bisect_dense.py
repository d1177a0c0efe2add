"""Bisect the fused dense-row kernel (miner_fused<bf16>, config 3) across commits.

    python tools/bisect_dense.py --build C1 C2 ...   # CPU: miner_score.hip of each commit -> tools/bisect/libscore_<C>.so
    python tools/bisect_dense.py C1 C2 ...           # GPU: interleaved timing of every build on one batch

Each build compiles only that commit's miner_score.hip (+ its cdna4_common.h and include/ headers),
so the same inputs run through every version in one process; each version packs its own weights.
Prints the median ms per launch of 32,768 impressions (L=50, K=32, d=768, Dc=200, C=40).
"""
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
        src = os.path.join("/tmp", "bisect_src", c)
        os.makedirs(os.path.join(src, "miner_amd", "csrc"), exist_ok=True)
        os.makedirs(os.path.join(src, "include"), exist_ok=True)
        files = subprocess.run(["git", "-C", ROOT, "ls-tree", "--name-only", c, "include/"], capture_output=True,
                               text=True, check=True).stdout.split()
        for f in files + ["miner_amd/csrc/miner_score.hip", "miner_amd/csrc/cdna4_common.h"]:
            r = subprocess.run(["git", "-C", ROOT, "show", f"{c}:{f}"], capture_output=True)
            if r.returncode != 0:              # cdna4_common.h appeared after the first versions
                continue
            data = r.stdout
            with open(os.path.join(src, f), "wb") as fh:
                fh.write(data)
        os.makedirs(OUT, exist_ok=True)
        lib = os.path.join(OUT, f"libscore_{c}.so")
        subprocess.run([hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wno-pass-failed",
                        "-I", os.path.join(src, "include"), os.path.join(src, "miner_amd", "csrc", "miner_score.hip"),
                        "-o", lib], check=True)
        print("built", lib)


def run(commits, reps=7):
    import torch
    sys.path.insert(0, ROOT)
    from miner_amd import synthetic
    P, I = ctypes.c_void_p, ctypes.c_int
    dev = "cuda:0"
    B, L, d, C, K, Dc = 32768, 50, 768, 40, 32, 200
    imp = synthetic.impressions(36, 0, B, L=L, d=d, C=C, device=dev, dtype=torch.bfloat16)
    W1, Q, W2 = [w.to(torch.bfloat16).contiguous() for w in synthetic.init_weights(36, d, Dc, K, device=dev)]
    mask = imp.his_mask.contiguous().view(torch.uint8)
    st = torch.cuda.current_stream().cuda_stream
    libs = {}
    for c in commits:
        h = ctypes.CDLL(os.path.join(OUT, f"libscore_{c}.so"))
        h.miner_packed_weights_bytes.restype = ctypes.c_size_t
        h.miner_packed_weights_bytes.argtypes = [I, I, I, I]
        h.miner_pack_weights.argtypes = [P, I, P, P, P, I, I, I, P]
        h.miner_score.argtypes = [P, I, I, P, P, P, P, P, P, I, I, I, I, I, I, P, P]
        buf = torch.empty(h.miner_packed_weights_bytes(1, d, Dc, K), dtype=torch.uint8, device=dev)
        assert h.miner_pack_weights(st, 1, W1.data_ptr(), Q.data_ptr(), W2.data_ptr(), d, Dc, K, buf.data_ptr()) == 0
        libs[c] = (h, buf)
    out = {c: torch.empty((B, C), device=dev) for c in commits}

    def launch(c):
        h, buf = libs[c]
        rc = h.miner_score(st, 1, 0, imp.history.data_ptr(), mask.data_ptr(), None, imp.candidates.data_ptr(), None,
                           buf.data_ptr(), B, L, C, d, Dc, K, out[c].data_ptr(), None)
        assert rc == 0, rc

    times = {c: [] for c in commits}
    for c in commits:
        launch(c)
    torch.cuda.synchronize()
    for _ in range(reps):
        for c in commits:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            launch(c)
            b.record()
            torch.cuda.synchronize()
            times[c].append(a.elapsed_time(b))
    ref = out[commits[0]]
    for c in commits:
        diff = float((out[c] - ref).abs().max())
        print(f"{c}: {statistics.median(times[c]):.3f} ms per launch (min {min(times[c]):.3f}), "
              f"max |score - {commits[0]}| {diff:.2e}", flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "--build":
        build(sys.argv[2:])
    else:
        run(sys.argv[1:])
