"""Time the FastFormer kernel on the config-4 shape (50k impressions, L=50, C=40) — GPU only.

    python tools/ff_time.py [--dtype bf16|fp32] [--iters N] [--B 50000]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from miner_amd import fastformer as ff  # noqa: E402
from miner_amd import synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--B", type=int, default=50000)
    ap.add_argument("--L", type=int, default=50)
    ap.add_argument("--C", type=int, default=40)
    ap.add_argument("--dense", action="store_true", help="dense [B, L, H] rows (bench.py config4_subline), not ids")
    a = ap.parse_args()
    dt = {"bf16": torch.bfloat16, "fp32": torch.float32}[a.dtype]
    dev = "cuda:0"
    n_news = 65238
    table = synthetic.news_table(1, n_news, 256, device=dev, dtype=dt)
    beh = synthetic.behaviors(1, 0, a.B, L=a.L, n_news=n_news, C=a.C, device=dev)
    packed = ff.pack(synthetic.fastformer_params(0).to(dev), dt)
    offs = beh.cand_offsets
    run = lambda: ff.score_gather(table, beh.his_ids, beh.his_mask, beh.cand_ids, packed, cand_offsets=offs,
                                  validate=False)
    if a.dense:                    # the bench's config-4 sub-line inputs (bench.py config4_subline)
        g = torch.Generator().manual_seed(1000)
        lens = torch.randint(0, a.L + 1, (a.B,), generator=g)
        mask = (torch.arange(a.L)[None, :] >= (a.L - lens)[:, None]).to(dev)
        hist = (torch.randn(a.B, a.L, 256, generator=g) * 0.0625).to(dev, dt)
        cand = (torch.randn(a.B, a.C, 256, generator=g) * 0.0625).to(dev, dt)
        run = lambda: ff.score(hist, mask, cand, packed)
    for _ in range(2):
        run()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(a.iters):
        run()
    en.record()
    torch.cuda.synchronize()
    ms = st.elapsed_time(en) / a.iters
    pairs = int(offs[-1])
    flops = a.B * (13 * 2 * 64 * 256 * 256)   # MFMA work incl. the pad to 64 rows
    print(json.dumps({"dtype": a.dtype, "B": a.B, "ms": round(ms, 4), "pairs_per_s": pairs / ms * 1e3,
                      "imps_per_s": a.B / ms * 1e3, "mfma_tflops_padded": flops / ms / 1e9,
                      "cycles_per_imp_per_cu": ms * 1e-3 * 2.4e9 * 256 / a.B}))


if __name__ == "__main__":
    main()
