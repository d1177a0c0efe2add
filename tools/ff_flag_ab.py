"""FastFormer kernel builds A/B (fastformer.hip alone with extra -D flags), interleaved on the bench's
config-4 inputs (50k impressions of news ids, bf16): median ms per launch, max |score diff|.

    python tools/ff_flag_ab.py --build NAME [FLAGS...]     # CPU: tools/bisect/libff_NAME.so
    python tools/ff_flag_ab.py NAME1 NAME2 ...             # GPU
"""
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
    lib = os.path.join(OUT, f"libff_{name}.so")
    subprocess.run([hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wno-pass-failed",
                    *flags, "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "miner_amd", "csrc", "fastformer.hip"),
                    "-o", lib], check=True)
    print("built", lib, flush=True)


def run(names, B=50000, reps=7):
    import torch
    from miner_amd import synthetic
    P, I = ctypes.c_void_p, ctypes.c_int
    dev = "cuda:0"
    n_news = 65238
    table = synthetic.news_table(1, n_news, 256, device=dev, dtype=torch.bfloat16)
    beh = synthetic.behaviors(1, 0, B, L=50, n_news=n_news, C=40, device=dev)
    params = synthetic.fastformer_params(0).to(dev)
    mask = beh.his_mask.contiguous().view(torch.uint8)
    st = torch.cuda.current_stream().cuda_stream
    libs, packs = {}, {}
    for n in names:
        h = ctypes.CDLL(os.path.join(OUT, f"libff_{n}.so"))
        h.miner_fastformer_packed_bytes.restype = ctypes.c_size_t
        h.miner_fastformer_packed_bytes.argtypes = [I]
        h.miner_fastformer_pack.argtypes = [P, I, P, P]
        h.miner_fastformer_score_gather.argtypes = [P, I, P, I, P, P, P, P, P, I, I, I, P, P]
        buf = torch.empty(h.miner_fastformer_packed_bytes(1), dtype=torch.uint8, device=dev)
        assert h.miner_fastformer_pack(st, 1, params.data_ptr(), buf.data_ptr()) == 0
        libs[n], packs[n] = h, buf
    out = {n: torch.empty(int(beh.cand_ids.numel()), device=dev) for n in names}

    def launch(n):
        rc = libs[n].miner_fastformer_score_gather(st, 1, table.data_ptr(), n_news, beh.his_ids.data_ptr(),
                                                   mask.data_ptr(), beh.cand_ids.data_ptr(), beh.cand_offsets.data_ptr(),
                                                   packs[n].data_ptr(), B, 50, 40, out[n].data_ptr(), None)
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
    # the fp32 parity mode of the first build (exact fp32 arithmetic) as the accuracy yardstick
    h0 = libs[names[0]]
    t32 = table.float()
    buf32 = torch.empty(h0.miner_fastformer_packed_bytes(0), dtype=torch.uint8, device=dev)
    assert h0.miner_fastformer_pack(st, 0, params.data_ptr(), buf32.data_ptr()) == 0
    ref = torch.empty_like(out[names[0]])
    assert h0.miner_fastformer_score_gather(st, 0, t32.data_ptr(), n_news, beh.his_ids.data_ptr(), mask.data_ptr(),
                                            beh.cand_ids.data_ptr(), beh.cand_offsets.data_ptr(), buf32.data_ptr(),
                                            B, 50, 40, ref.data_ptr(), None) == 0
    torch.cuda.synchronize()
    scale = float(ref.abs().max())
    for n in names:
        err = (out[n] - ref).abs()
        print(f"{n}: {statistics.median(times[n]):.3f} ms per {B} impressions, max |diff vs {names[0]}| "
              f"{float((out[n] - out[names[0]]).abs().max()):.2e}, vs fp32: max {float(err.max()):.2e} "
              f"mean {float(err.mean()):.2e} (max |ref| {scale:.2e})", flush=True)


if __name__ == "__main__":
    a = sys.argv[1:]
    if a and a[0] == "--build":
        build(*a[1:])
    else:
        run(a)
