"""Generate tests/golden/corpus_*.npz by running the REFERENCE's own Miner (src/model/model.py:13-138)
with the whole news table as every user's candidate set — what BASELINE config 5's full-corpus
ranking computes — at config-5 history / interest shapes (L=200, K=64, Dc=200) and a small d.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_corpus_golden.py

A stub news encoder (embedding-table lookup, as in make_golden.py) stands in for the RoBERTa
encoder. Recorded: news table, history ids / mask, the module weights (poly_attn.linear.weight,
poly_attn.context_codes, target_aware_attn.linear.weight), mui [U,K,d] and the scores [U,N] of
every user against every news row. Data only: no reference code is stored.
"""
from __future__ import annotations

import os
import sys

import numpy as np

REF = os.environ.get("MINER_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


def main():
    if not os.path.isdir(os.path.join(REF, "src")):
        print(f"reference not found at {REF}: skipping")
        return 0
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import torch
    import torch.nn as nn
    from src.model.model import Miner                      # noqa: E402  (reference)

    class StubNewsEncoder(nn.Module):
        def __init__(self, table):
            super().__init__()
            self.embed_dim = table.shape[1]
            self.register_buffer("table", table)

        def forward(self, title_encoding, title_attn_mask, sapo_encoding=None, sapo_attn_mask=None):
            return self.table[title_encoding[:, 0]]

    def run_case(name, *, U, L, K, Dc, d, N, score_type, seed, hist_len):
        rng = np.random.default_rng(seed)
        table = (rng.standard_normal((N, d)) / np.sqrt(d)).astype(np.float32)   # row 0 = the pad news
        his_ids = np.zeros((U, L), np.int64)
        for u in range(U):
            n = int(hist_len[u])
            his_ids[u, L - n:] = rng.integers(1, N, size=n)                     # left-padded (reader.py:369)
        his_mask = his_ids != 0
        torch.manual_seed(seed)
        model = Miner(StubNewsEncoder(torch.from_numpy(table)), False, K, Dc, score_type, 0.2).eval()
        t = lambda x: torch.from_numpy(np.ascontiguousarray(x))
        cand = np.tile(np.arange(N), (U, 1))                                    # every news is a candidate
        with torch.no_grad():
            title, his = t(cand)[..., None], t(his_ids)[..., None]
            ones = lambda x: torch.ones_like(x, dtype=torch.bool)
            mui, scores = model(title=title, title_mask=ones(title), his_title=his, his_title_mask=ones(his),
                                his_mask=t(his_mask), sapo=title, sapo_mask=ones(title), his_sapo=his,
                                his_sapo_mask=ones(his))
        arrs = dict(U=U, L=L, K=K, Dc=Dc, d=d, N=N, score_type=score_type, table=table, his_ids=his_ids,
                    his_mask=his_mask, W1=model.poly_attn.linear.weight.detach().numpy(),
                    Q=model.poly_attn.context_codes.detach().numpy(), mui=mui.numpy(), scores=scores.numpy())
        if score_type == "weighted":
            arrs["W2"] = model.target_aware_attn.linear.weight.detach().numpy()
        path = os.path.join(OUT, f"corpus_{name}.npz")
        np.savez_compressed(path, **arrs)
        print(f"{name}: U={U} L={L} K={K} d={d} N={N} {score_type} -> {os.path.getsize(path) / 1e6:.2f} MB, "
              f"score rms {float(scores.pow(2).mean().sqrt()):.4f}")

    # config-5 shapes with d = 128: a full history, a short one, an all-padded one, a ragged one
    run_case("c5_weighted", U=5, L=200, K=64, Dc=200, d=128, N=700, score_type="weighted", seed=51,
             hist_len=[200, 37, 0, 150, 1])
    run_case("c5_max", U=3, L=200, K=64, Dc=200, d=128, N=600, score_type="max", seed=52, hist_len=[200, 90, 3])
    run_case("k32_mean", U=3, L=77, K=32, Dc=200, d=64, N=333, score_type="mean", seed=53, hist_len=[77, 10, 40])
    return 0


if __name__ == "__main__":
    sys.exit(main())
