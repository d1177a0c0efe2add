"""fp32 per-news precompute of the config-3 table (104,000 x 768, Dc 200, K 32), its two forms timed
interleaved in one process: MINER_DTYPE_F32 (the W1 / W2 products on fp16 pairs) and
MINER_DTYPE_F32_MFMA (every product on the fp32 MFMA). Prints the median HIP-event ms per launch of
each and the max relative difference of their outputs. Usage: python tools/pre_ab.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from miner_amd import _lib, ops, synthetic  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = "cuda:0"
    n, d, Dc, K = 104000, 768, 200, 32
    g = torch.Generator().manual_seed(5)
    table = (torch.randn((n, d), generator=g) / d ** 0.5).to(dev)
    W1, Q, W2 = synthetic.init_weights(5, d, Dc, K, device=dev)
    pw = ops.pack_weights(W1, Q, W2, dtype=torch.float32)
    lib = _lib.lib()
    st = torch.cuda.current_stream().cuda_stream
    outs = {}
    for code in (_lib.DTYPE_F32, _lib.DTYPE_F32_MFMA):
        outs[code] = (torch.empty((n, K), device=dev), torch.empty((n, d), device=dev))
    times = {c: [] for c in outs}

    def run(code):
        lg, pj = outs[code]
        rc = lib.miner_news_precompute(st, code, table.data_ptr(), n, pw.buf.data_ptr(), d, Dc, K,
                                       lg.data_ptr(), pj.data_ptr())
        assert rc == 0, rc

    for code in outs:
        for _ in range(3):
            run(code)
    torch.cuda.synchronize()
    for _ in range(reps):
        for code in outs:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            run(code)
            b.record()
            torch.cuda.synchronize()
            times[code].append(a.elapsed_time(b))
    med = {c: sorted(v)[len(v) // 2] for c, v in times.items()}
    print(f"pairs (F32) {med[_lib.DTYPE_F32]:.4f} ms, fp32 MFMA (F32_MFMA) {med[_lib.DTYPE_F32_MFMA]:.4f} ms per launch")
    for i, name in enumerate(("logits", "proj")):
        x, y = outs[_lib.DTYPE_F32][i], outs[_lib.DTYPE_F32_MFMA][i]
        print(f"{name}: max |pairs - mfma| / max |mfma| = {float((x - y).abs().max() / y.abs().max()):.3e}")


if __name__ == "__main__":
    main()
