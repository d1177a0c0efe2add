"""A/B of whole-library builds on the dense fp32 path (Miner.score on [B, L, d] rows, config-3 shape):
each build is a separate libminer_hip with extra -D flags, timed in its own process.

    python tools/dense_ab.py --build NAME [FLAGS...]    # CPU: tools/bisect/libminer_NAME.so
    python tools/dense_ab.py NAME1 NAME2 ...             # GPU: median ms per 8,192-impression launch
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "bisect")
sys.path.insert(0, ROOT)


def build(name, *flags):
    from miner_amd.build import hipcc, SOURCES, ARCH
    os.makedirs(OUT, exist_ok=True)
    lib = os.path.join(OUT, f"libminer_{name}.so")
    subprocess.run([hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wno-pass-failed",
                    "-I", os.path.join(ROOT, "include"), *flags, *SOURCES, "-o", lib], check=True)
    print("built", lib)


def time_one():
    import statistics
    import torch
    from miner_amd import ops, synthetic
    dev = "cuda:0"
    n, L, C, d, Dc, K = 8192, 50, 40, 768, 200, 32
    W1, Q, W2 = synthetic.init_weights(36, d, Dc, K, device=dev)
    imp = synthetic.impressions(36, 0, n, L=L, d=d, C=C, device=dev, dtype=torch.float32)
    pw = ops.pack_weights(W1, Q, W2, dtype=torch.float32)
    s0 = ops.score(imp.history, imp.his_mask, imp.candidates, pw)
    torch.cuda.synchronize()
    ts = []
    for _ in range(7):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(5):
            ops.score(imp.history, imp.his_mask, imp.candidates, pw)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / 5)
    torch.save(s0.cpu(), os.path.join(OUT, f"scores_{os.environ['DENSE_AB_NAME']}.pt"))
    print(f"{os.environ['DENSE_AB_NAME']}: {statistics.median(ts):.3f} ms per {n} impressions "
          f"({n * C / statistics.median(ts) / 1e3:.1f} M pairs/s)", flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "--build":
        build(sys.argv[2], *sys.argv[3:])
    elif sys.argv[1] == "--one":
        time_one()
    else:
        import torch
        first = None
        for name in sys.argv[1:]:
            env = dict(os.environ, MINER_HIP_LIB=os.path.join(OUT, f"libminer_{name}.so"), DENSE_AB_NAME=name)
            subprocess.run([sys.executable, __file__, "--one"], env=env, check=True)
            s = torch.load(os.path.join(OUT, f"scores_{name}.pt"))
            if first is None:
                first = s
            print(f"  max |score - {sys.argv[1]}| {float((s - first).abs().max()):.3e}", flush=True)
