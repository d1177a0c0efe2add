"""Generate tests/golden/fastformer_*.npz by running the REFERENCE's own FastFormer model
(src/model/model.py:223-327 FastFormer, :329-545 AttentionPooling / FastSelfAttention /
FastAttention / FastformerLayer / FastformerEncoder; HF Bert* blocks) on CPU, eval mode.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_fastformer_golden.py

A stub news encoder (embedding-table lookup, as in make_golden.py) stands in for the RoBERTa
encoder. Recorded per case: news table, history / candidate ids, his_mask, every parameter of the
user encoder (state_dict arrays), the user vectors (the encoder's pooled output) and the matching
scores. Data only: no reference code is stored.
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
    from src.model.model import FastFormer                 # noqa: E402  (reference)

    class StubNewsEncoder(nn.Module):
        def __init__(self, table):
            super().__init__()
            self.embed_dim = table.shape[1]
            self.register_buffer("table", table)

        def forward(self, title_encoding, title_attn_mask, sapo_encoding=None, sapo_attn_mask=None):
            return self.table[title_encoding[:, 0]]

    def run_case(name, *, B, L, C, seed, hist_len=None, scale=1.0):
        torch.manual_seed(seed)
        rng = np.random.default_rng(seed)
        d = 256   # FastFormer's hidden size is fixed (model.py:251)
        n_news = 1 + B * (L + C)
        table = torch.from_numpy((rng.standard_normal((n_news, d)) * scale).astype(np.float32))
        enc = StubNewsEncoder(table)
        model = FastFormer(news_encoder=enc, score_type="weighted", dropout=0.2).eval()
        # the reference initialises biases to 0 and LayerNorm to (1, 0) (model.py:536-545): randomise
        # them so the fixtures exercise every parameter
        with torch.no_grad():
            for pname, prm in model.fast_attn.named_parameters():
                if pname.endswith("bias"):
                    prm.copy_(torch.randn_like(prm) * 0.05)
                elif "LayerNorm.weight" in pname:
                    prm.copy_(1.0 + torch.randn_like(prm) * 0.1)
        his_ids = rng.integers(1, n_news, (B, L))
        cand_ids = rng.integers(1, n_news, (B, C))
        lens = rng.integers(0, L + 1, B) if hist_len is None else np.full(B, hist_len)
        his_mask = np.arange(L)[None, :] >= (L - lens)[:, None]
        his_ids = np.where(his_mask, his_ids, 0)
        t = lambda x: torch.from_numpy(np.ascontiguousarray(x))
        with torch.no_grad():
            title, his = t(cand_ids)[..., None], t(his_ids)[..., None]
            ones = lambda x: torch.ones_like(x, dtype=torch.bool)
            scores = model(title=title, title_mask=ones(title), his_title=his, his_title_mask=ones(his),
                           his_mask=t(his_mask), sapo=title, sapo_mask=ones(title), his_sapo=his,
                           his_sapo_mask=ones(his))
            user = model.fast_attn(input_embs=table[t(his_ids)], attention_mask=t(his_mask))
        arrs = dict(B=B, L=L, C=C, table=table.numpy(), his_ids=his_ids, cand_ids=cand_ids, his_mask=his_mask,
                    user=user.numpy(), scores=scores.numpy())
        for k, v in model.fast_attn.state_dict().items():
            arrs["p." + k] = v.numpy()
        path = os.path.join(OUT, f"fastformer_{name}.npz")
        np.savez_compressed(path, **arrs)
        print(f"{name}: B={B} L={L} C={C} -> {os.path.getsize(path) / 1e6:.2f} MB, "
              f"score rms {float(scores.pow(2).mean().sqrt()):.4f}")

    run_case("cfg4_slice", B=6, L=50, C=40, seed=4, scale=0.0625)
    run_case("edge_short", B=4, L=20, C=7, seed=5, scale=1.0)        # L <= 32, embeddings ~ N(0,1)
    run_case("edge_empty", B=3, L=50, C=5, seed=6, hist_len=0)        # all-padded histories
    run_case("edge_full", B=3, L=64, C=70, seed=7, hist_len=64)       # L = 64, C > 64
    return 0


if __name__ == "__main__":
    sys.exit(main())
