"""ORACLE — test infrastructure only.

CPU restatement of the reference's FastFormer user encoder and its click predictor
(src/model/model.py:223-327 FastFormer.forward, :329-545 AttentionPooling, FastSelfAttention,
FastAttention, FastformerLayer, FastformerEncoder; the HF BertSelfOutput / BertIntermediate /
BertOutput blocks they use), same ATen ops in the same order, eval mode (dropout off), written
over a flat parameter dict named like the reference's ``fast_attn.state_dict()``. Pinned by
tests/golden/fastformer_*.npz (made by importing the reference's FastFormer):
tests/test_fastformer_oracle.py.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

HEADS, HEAD_DIM, HIDDEN, EPS = 16, 16, 256, 1e-12   # model.py:245-266 config


def _lin(x, p, name):
    return F.linear(x, p[name + ".weight"], p.get(name + ".bias"))


def _self_attention(p, pre, x, ext):
    """FastSelfAttention.forward (model.py:409-459)."""
    B, L, _ = x.shape
    mq = _lin(x, p, pre + "query")
    mk = _lin(x, p, pre + "key")
    qfs = _lin(mq, p, pre + "query_att").transpose(1, 2) / HEAD_DIM ** 0.5
    qfs = qfs + ext
    qw = torch.softmax(qfs, dim=-1).unsqueeze(2)
    ql = mq.view(B, L, HEADS, HEAD_DIM).permute(0, 2, 1, 3)
    pq = torch.matmul(qw, ql).transpose(1, 2).view(-1, 1, HEADS * HEAD_DIM)
    mqk = mk * pq.repeat(1, L, 1)
    qks = (_lin(mqk, p, pre + "key_att") / HEAD_DIM ** 0.5).transpose(1, 2)
    qks = qks + ext
    kw = torch.softmax(qks, dim=-1).unsqueeze(2)
    kl = mqk.view(B, L, HEADS, HEAD_DIM).permute(0, 2, 1, 3)
    pk = torch.matmul(kw, kl)
    wv = (pk * ql).transpose(1, 2)
    wv = wv.reshape(wv.size()[:-2] + (HEADS * HEAD_DIM,))
    return _lin(wv, p, pre + "transform") + mq


def _ln(x, p, name):
    return F.layer_norm(x, (HIDDEN,), p[name + ".weight"], p[name + ".bias"], EPS)


def user_vectors(p: dict, embs: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """FastformerEncoder.forward (model.py:511-545) + AttentionPooling (:347-367): [B,L,256] -> [B,256]."""
    B, L, _ = embs.shape
    ext = (1.0 - mask.unsqueeze(1).to(embs.dtype)) * -10000.0
    x = embs + p["position_embeddings.weight"][:L].unsqueeze(0)
    x = _ln(x, p, "LayerNorm")
    for i in range(2):
        pre = f"encoders.{i}."
        so = _self_attention(p, pre + "attention.self.", x, ext)
        a = _ln(_lin(so, p, pre + "attention.output.dense") + x, p, pre + "attention.output.LayerNorm")
        h = F.gelu(_lin(a, p, pre + "intermediate.dense"))
        x = _ln(_lin(h, p, pre + "output.dense") + a, p, pre + "output.LayerNorm")
    e = torch.tanh(_lin(x, p, "poolers.0.att_fc1"))
    alpha = torch.exp(_lin(e, p, "poolers.0.att_fc2"))
    alpha = alpha * mask.unsqueeze(2)
    alpha = alpha / (torch.sum(alpha, dim=1, keepdim=True) + 1e-8)
    return torch.bmm(x.permute(0, 2, 1), alpha).reshape(B, -1)


def scores(p: dict, embs: torch.Tensor, mask: torch.Tensor, cand: torch.Tensor) -> torch.Tensor:
    """FastFormer.forward tail (model.py:321-322): candidate_repr · user -> [B, C]."""
    u = user_vectors(p, embs, mask)
    return torch.matmul(cand, u.unsqueeze(-1)).squeeze(-1)
