"""ORACLE — test infrastructure only.

Full-corpus ranking (BASELINE config 5) restated on the CPU: the reference's user encoder and
click score (src/model/model.py:159-185 PolyAttention, :200-216 TargetAwareAttention, :127-136
aggregation) with the candidate set of every user = the whole news table, through the same
functions as oracle/miner_oracle.py (pinned to the reference by tests/golden/*.npz), and the
top-k with the kernel's documented tie order (score descending, then news id ascending). Pinned
directly by tests/golden/corpus_ref.npz (the reference Miner scoring a whole table):
tests/test_corpus_oracle.py.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from oracle import miner_oracle as orc


def encode(E, mask, W1, Q, W2=None, bias=None):
    """-> (mui [U,K,d], proj [U,K,d] = gelu(mui·W2ᵀ) or None) in fp32 (model.py:159-185, :212)."""
    mui = orc.poly_attention_torch(E, mask, W1, Q, bias)
    proj = F.gelu(F.linear(mui, W2)) if W2 is not None else None
    return mui, proj


def corpus_scores(mui, proj, news, score_type="weighted", chunk=4096):
    """[U,N] click scores of every user against every news row (model.py:127-136, 213-214)."""
    out = []
    for lo in range(0, news.shape[0], chunk):
        cand = news[lo:lo + chunk].unsqueeze(0).expand(mui.shape[0], -1, -1)
        M = torch.matmul(cand, mui.permute(0, 2, 1))
        if score_type == "max":
            s = M.max(dim=2)[0]
        elif score_type == "mean":
            s = M.mean(dim=2)
        elif score_type == "weighted":
            w = F.softmax(torch.matmul(cand, proj.permute(0, 2, 1)), dim=2)
            s = torch.mul(w, M).sum(dim=2)
        else:
            raise ValueError("Invalid method of aggregating matching score")
        out.append(s)
    return torch.cat(out, 1)


def topk(scores, k):
    """(scores [U,k], ids [U,k]) best first, ties by lower id; past N: (-inf, -1)."""
    s = np.asarray(scores, np.float64)
    U, N = s.shape
    ts = np.full((U, k), -np.inf)
    ti = np.full((U, k), -1, np.int64)
    ids = np.arange(N)
    for u in range(U):
        order = np.lexsort((ids, -s[u]))[:k]
        ts[u, :len(order)] = s[u, order]
        ti[u, :len(order)] = order
    return ts, ti
