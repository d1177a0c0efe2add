"""Per-stage cycle breakdown of the fused kernel (diagnostic build with -DMINER_STAMPS).

    python tools/stage_profile.py [--build] [--batch 8192] [--dtype bf16|f32]

Thread 0 of each workgroup sums s_memtime deltas between the barriers that delimit the stages;
reported as shader cycles per impression per workgroup (one workgroup per CU). Read the SHARES:
the stamps themselves cost a few instructions per stage.
"""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
STAMP_LIB = os.path.join(ROOT, "miner_amd", "libminer_hip_stamps.so")
STAGES = ["S0 wait history DMA", "S1 rest (S-partials+barrier)", "S2 Q·Pᵀ", "S3 softmax", "S4 A·E", "S5 W2+gelu",
          "S6 products", "S6 reduce", "S7 score", "loop tail", "S1 loop (wave 0)", "S1 tanh (wave 0)"]
FF_STAGES = ["E load + LN0", "G12 q,k", "qfs partial", "q softmax", "pq + qks partial", "k softmax", "pk + wv store",
             "G3 transform", "G4 + LN1", "G5 + gelu", "G6 + LN2", "pooler GEMM", "pooler rest", "scores"]



def build(extra=(), out=STAMP_LIB):
    from miner_amd.build import hipcc, SOURCES, ARCH
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-DMINER_STAMPS", "-DMINER_NEWS_ABL_MASK=0x7fffffff",
           "-Wno-pass-failed", "-I", os.path.join(ROOT, "include"), *extra, *SOURCES, "-o", out]
    subprocess.run(cmd, check=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--variant", default=None, help="build: -D flags, comma separated; run: library suffix")
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--L", type=int, default=50)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--C", type=int, default=40)
    ap.add_argument("--kernel", default="miner", choices=["miner", "fastformer"])
    ap.add_argument("--cflag", action="append", default=[], help="build: extra compiler flag (repeatable), "
                    "e.g. -fno-slp-vectorize as miner_amd/build.py FILE_FLAGS gives fastformer.hip")
    args = ap.parse_args()
    lib = STAMP_LIB if not args.variant else STAMP_LIB.replace(".so", "_" + args.variant.replace(",", "_").replace("=", "") + ".so")
    if args.build:
        build([*(["-D" + x for x in args.variant.split(",")] if args.variant else ()), *args.cflag], lib)
        return
    os.environ["MINER_HIP_LIB"] = lib
    if args.kernel == "fastformer":
        return fastformer(args)
    import torch
    from miner_amd import _lib, ops, synthetic
    h = _lib.lib()
    fn = h.miner_debug_stage_cycles
    fn.argtypes = [ctypes.c_void_p]
    fn.restype = ctypes.c_int
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    imp = synthetic.impressions(36, 0, args.batch, L=args.L, d=args.d, C=args.C, device="cuda", dtype=dt)
    W1, Q, W2 = synthetic.init_weights(36, args.d, 200, 32, device="cuda")
    pw = ops.pack_weights(W1, Q, W2, dtype=dt)
    for _ in range(2):
        ops.score(imp.history, imp.his_mask, imp.candidates, pw)
    torch.cuda.synchronize()
    out = (ctypes.c_ulonglong * 16)()
    fn(out)  # reset
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 3
    ev0.record()
    for _ in range(reps):
        ops.score(imp.history, imp.his_mask, imp.candidates, pw)
    ev1.record()
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / reps
    names = STAGES
    assert fn(out) == 0
    n = out[12]
    tot = sum(out[i] for i in range(len(names)))
    print(f"{args.dtype} L={args.L} d={args.d} C={args.C} batch={args.batch}: {ms:.3f} ms/launch, "
          f"{n} impression-passes, {tot / n:.0f} cycles per impression per workgroup")
    for i, name in enumerate(names):
        print(f"  {name:22s} {out[i] / n:10.0f} cycles  {100.0 * out[i] / tot:5.1f}%")


def fastformer(args):
    import torch
    from miner_amd import _lib, synthetic
    from miner_amd import fastformer as ff
    h = _lib.lib()
    fn = h.miner_ff_debug_stage_cycles
    fn.argtypes = [ctypes.c_void_p]
    fn.restype = ctypes.c_int
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    n_news = 65238
    table = synthetic.news_table(1, n_news, 256, device="cuda", dtype=dt)
    beh = synthetic.behaviors(1, 0, args.batch, L=args.L, n_news=n_news, C=args.C, device="cuda")
    packed = ff.pack(synthetic.fastformer_params(0).to("cuda"), dt)
    run = lambda: ff.score_gather(table, beh.his_ids, beh.his_mask, beh.cand_ids, packed,
                                  cand_offsets=beh.cand_offsets, validate=False)
    for _ in range(2):
        run()
    torch.cuda.synchronize()
    out = (ctypes.c_ulonglong * 17)()
    fn(out)  # reset
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 3
    ev0.record()
    for _ in range(reps):
        run()
    ev1.record()
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / reps
    assert fn(out) == 0
    n = out[16]
    tot = sum(out[i] for i in range(len(FF_STAGES)))
    print(f"fastformer {args.dtype} L={args.L} C={args.C} batch={args.batch}: {ms:.3f} ms/launch, "
          f"{n} impression-passes, {tot / n:.0f} cycles per impression per workgroup")
    for i, name in enumerate(FF_STAGES):
        print(f"  {name:22s} {out[i] / n:10.0f} cycles  {100.0 * out[i] / tot:5.1f}%")


if __name__ == "__main__":
    main()
