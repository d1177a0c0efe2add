"""Dense-row kernel builds A/B (miner_score.hip alone with extra -D flags), interleaved on the
bench's dense_rows_kernel fp32 inputs (L=50, K=32, d=768, Dc=200, C=40): median ms per launch and
the max score difference against the first build.

    python tools/dense_flag_ab.py --build NAME [FLAGS...]     # CPU: tools/bisect/libdense_NAME.so
    python tools/dense_flag_ab.py [--dtype fp32|bf16] [--B N] NAME1 NAME2 ...   # GPU
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
    lib = os.path.join(OUT, f"libdense_{name}.so")
    subprocess.run([hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wno-pass-failed",
                    *flags, "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "miner_amd", "csrc", "miner_score.hip"),
                    "-o", lib], check=True)
    print("built", lib, flush=True)


def run(names, dtype="fp32", B=8192, reps=9):
    import torch
    from miner_amd import synthetic
    P, I = ctypes.c_void_p, ctypes.c_int
    dev = "cuda:0"
    L, d, C, K, Dc = 50, 768, 40, 32, 200
    dt = 0 if dtype == "fp32" else 1
    tdt = torch.float32 if dt == 0 else torch.bfloat16
    imp = synthetic.impressions(36, 0, B, L=L, d=d, C=C, device=dev, dtype=tdt)
    W1, Q, W2 = [w.to(tdt).contiguous() for w in synthetic.init_weights(36, d, Dc, K, device=dev)]
    mask = imp.his_mask.contiguous().view(torch.uint8)
    st = torch.cuda.current_stream().cuda_stream
    libs = {}
    for n in names:
        h = ctypes.CDLL(os.path.join(OUT, f"libdense_{n}.so"))
        h.miner_packed_weights_bytes.restype = ctypes.c_size_t
        h.miner_packed_weights_bytes.argtypes = [I, I, I, I]
        h.miner_pack_weights.argtypes = [P, I, P, P, P, I, I, I, P]
        h.miner_score.argtypes = [P, I, I, P, P, P, P, P, P, I, I, I, I, I, I, P, P]
        buf = torch.empty(h.miner_packed_weights_bytes(dt, d, Dc, K), dtype=torch.uint8, device=dev)
        assert h.miner_pack_weights(st, dt, W1.data_ptr(), Q.data_ptr(), W2.data_ptr(), d, Dc, K, buf.data_ptr()) == 0
        libs[n] = (h, buf)
    out = {n: torch.empty((B, C), device=dev) for n in names}

    def launch(n):
        h, buf = libs[n]
        rc = h.miner_score(st, dt, 0, imp.history.data_ptr(), mask.data_ptr(), None, imp.candidates.data_ptr(), None,
                           buf.data_ptr(), B, L, C, d, Dc, K, out[n].data_ptr(), None)
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
    ref = out[names[0]]
    for n in names:
        ms = statistics.median(times[n])
        print(f"{n}: {ms:.3f} ms per {B} impressions ({B * C / ms / 1e3:.1f} M pairs/s), "
              f"max |score - {names[0]}| {float((out[n] - ref).abs().max()):.2e}", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--build":
        build(*sys.argv[2:])
    else:
        ap = argparse.ArgumentParser()
        ap.add_argument("--dtype", default="fp32")
        ap.add_argument("--B", type=int, default=8192)
        ap.add_argument("names", nargs="+")
        a = ap.parse_args()
        run(a.names, a.dtype, a.B)
