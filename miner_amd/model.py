"""Drop-in mirror of the reference's src/model/model.py scoring modules, backed by libminer_hip.so.

Same class names, constructor signatures, parameter names (so reference state_dicts load as-is)
and forward contracts as the reference:

* ``Miner``                 src/model/model.py:13-138
* ``PolyAttention``         src/model/model.py:141-185
* ``TargetAwareAttention``  src/model/model.py:188-216

plus ``Miner.score(...)``, the entry point after the news encoder (the reference has no such
method: ``forward`` = news encoder + ``score``). All arithmetic of the scoring path runs in the
fused HIP kernel; calling these modules with CPU tensors raises (no CPU fallback).

``precision`` selects the kernel mode: ``"fp32"`` (default; parity with the reference to 1e-5) or
``"bf16"`` (bf16 operands, fp32 accumulation; the throughput mode). Since round 4 the fp32 mode runs
its two large products (S1 ``W1·Eᵀ`` and S5 ``W2·muiᵀ``) as bf16x6: every fp32 operand cut exactly
into three bf16 terms, the six leading partial products on the bf16 matrix cores (error against
float64 within 1.5x the fp32 MFMA's, tests/test_gpu_parity.py); ``MINER_DENSE_FP32=mfma32`` selects
the exact fp32 fma chains of ``v_mfma_f32_32x32x2_f32`` for every product.
"""
from __future__ import annotations

from typing import Union

import torch
import torch.nn as nn
from torch import Tensor

from . import ops

_PREC = {"fp32": torch.float32, "bf16": torch.bfloat16}


def pairwise_cosine_similarity(x: Tensor, y: Tensor, zero_diagonal: bool = False) -> Tensor:
    """src/utils.py:9-29 — host-side helper for the (off-by-default) category bias."""
    xn = torch.linalg.norm(x, dim=2, keepdim=True)
    yn = torch.linalg.norm(y, dim=2, keepdim=True)
    dist = torch.matmul(torch.div(x, xn), torch.div(y, yn).permute(0, 2, 1))
    if zero_diagonal:
        assert x.shape[1] == y.shape[1]
        mask = torch.eye(x.shape[1], device=dist.device, dtype=torch.bool).expand_as(dist)
        dist = dist.masked_fill(mask, 0)
    return dist


class _PackCache:
    """miner_pack_weights() output per (dtype, device), re-packed when a parameter changes
    (tracked through the parameters' version counters and storage pointers)."""

    def __init__(self):
        self._c = {}

    def get(self, dtype: torch.dtype, w_poly: Tensor = None, context_codes: Tensor = None, w_target: Tensor = None):
        """Packed weights for (W1, Q[, W2]), or W2 alone when w_poly is None (TargetAwareAttention)."""
        params = [t for t in (w_poly, context_codes, w_target) if t is not None]
        key = (dtype, params[0].device)
        stamp = tuple((t._version, t.data_ptr()) for t in params)
        hit = self._c.get(key)
        if hit is not None and hit[0] == stamp:
            return hit[1]
        with torch.no_grad():
            if w_poly is None:
                packed = ops.pack_target_weights(w_target.detach(), dtype=dtype)
            else:
                packed = ops.pack_weights(w_poly.detach(), context_codes.detach(),
                                          None if w_target is None else w_target.detach(), dtype=dtype)
        self._c[key] = (stamp, packed)
        return packed


class PolyAttention(nn.Module):
    """K additive attentions over the clicked-news history (model.py:141-185)."""

    def __init__(self, in_embed_dim: int, num_context_codes: int, context_code_dim: int):
        super().__init__()
        self.linear = nn.Linear(in_features=in_embed_dim, out_features=context_code_dim, bias=False)
        self.context_codes = nn.Parameter(nn.init.xavier_uniform_(
            torch.empty(num_context_codes, context_code_dim), gain=nn.init.calculate_gain('tanh')))
        self.precision = "fp32"
        self._pc = _PackCache()

    def forward(self, embeddings: Tensor, attn_mask: Tensor, bias: Tensor = None) -> Tensor:
        """embeddings [B,L,d], attn_mask [B,L] bool, bias [B,L,C] (or [B,L]) -> [B,K,d] fp32."""
        dt = _PREC[self.precision]
        if bias is not None and bias.dim() == 3:
            bias = bias.mean(dim=2)                                  # model.py:176
        packed = self._pc.get(dt, self.linear.weight, self.context_codes)
        return ops.poly_attention(embeddings.to(dt), attn_mask, packed, his_bias=bias)


class TargetAwareAttention(nn.Module):
    """Candidate-aware re-weighting of the K matching scores (model.py:188-216)."""

    def __init__(self, embed_dim: int):
        super().__init__()
        self.linear = nn.Linear(in_features=embed_dim, out_features=embed_dim, bias=False)
        self.precision = "fp32"
        self._pc = _PackCache()

    def forward(self, query: Tensor, key: Tensor, value: Tensor) -> Tensor:
        """query [B,K,d], key [B,C,d], value [B,C,K] -> [B,C] fp32."""
        dt = _PREC[self.precision]
        packed = self._pc.get(dt, w_target=self.linear.weight)          # W2 alone (model.py:198)
        return ops.target_aware(query.to(dt), key.to(dt), value, packed)


class Miner(nn.Module):
    """Multi-interest matching network (model.py:13-138), scoring path on MI355X."""

    def __init__(self, news_encoder, use_category_bias: bool, num_context_codes: int,
                 context_code_dim: int, score_type: str, dropout: float, num_category: Union[int, None] = None,
                 category_embed_dim: Union[int, None] = None, category_pad_token_id: Union[int, None] = None,
                 category_embed: Union[Tensor, None] = None, precision: str = "fp32"):
        super().__init__()
        self.news_encoder = news_encoder
        self.news_embed_dim = self.news_encoder.embed_dim
        self.use_category_bias = use_category_bias
        if self.use_category_bias:
            self.category_dropout = nn.Dropout(dropout)
            if category_embed is not None:
                self.category_embedding = nn.Embedding.from_pretrained(category_embed, freeze=False,
                                                                       padding_idx=category_pad_token_id)
                self.category_embed_dim = category_embed.shape[1]
            else:
                assert num_category is not None
                self.category_embedding = nn.Embedding(num_embeddings=num_category, embedding_dim=category_embed_dim,
                                                       padding_idx=category_pad_token_id)
                self.category_embed_dim = category_embed_dim
        self.poly_attn = PolyAttention(in_embed_dim=self.news_embed_dim, num_context_codes=num_context_codes,
                                       context_code_dim=context_code_dim)
        self.score_type = score_type
        if self.score_type == 'weighted':
            self.target_aware_attn = TargetAwareAttention(self.news_embed_dim)
        self.dropout = nn.Dropout(dropout)
        self._pc = _PackCache()
        self.set_precision(precision)

    def set_precision(self, precision: str) -> "Miner":
        if precision not in _PREC:
            raise ValueError(f"precision must be one of {sorted(_PREC)}")
        self.precision = precision
        self.poly_attn.precision = precision
        if self.score_type == 'weighted':
            self.target_aware_attn.precision = precision
        return self

    def category_bias(self, category: Tensor, his_category: Tensor) -> Tensor:
        """model.py:113-119: cosine(his_cat, cand_cat) [B,L,C]."""
        his = self.category_dropout(self.category_embedding(his_category))
        cand = self.category_dropout(self.category_embedding(category))
        return pairwise_cosine_similarity(his, cand)

    def score(self, history_repr: Tensor, his_mask: Tensor, candidate_repr: Tensor, *,
              cand_offsets: Tensor = None, category_bias: Tensor = None, return_user: bool = True):
        """Scoring after the news encoder (model.py:113-138).

        history_repr [B,L,d], his_mask [B,L] bool, candidate_repr [B,C,d] (or [N,d] with
        cand_offsets [B+1] int32), category_bias [B,L,C] or [B,L] (mean over candidates) or None.
        Returns (multi_user_interest [B,K,d] fp32, matching_scores [B,C] fp32) like forward, or the
        scores alone when return_user=False.
        """
        if self.score_type not in ('weighted', 'max', 'mean'):
            raise ValueError('Invalid method of aggregating matching score')     # model.py:136
        dt = _PREC[self.precision]
        if category_bias is not None and category_bias.dim() == 3:
            category_bias = category_bias.mean(dim=2)                           # model.py:176
        w2 = self.target_aware_attn.linear.weight if self.score_type == 'weighted' else None
        packed = self._pc.get(dt, self.poly_attn.linear.weight, self.poly_attn.context_codes, w2)
        out = ops.score(history_repr.to(dt), his_mask, candidate_repr.to(dt), packed,
                        score_type=self.score_type, cand_offsets=cand_offsets, his_bias=category_bias,
                        return_user=return_user)
        if return_user:
            scores, mui = out
            return mui, scores
        return out

    def forward(self, title: Tensor, title_mask: Tensor, his_title: Tensor, his_title_mask: Tensor,
                his_mask: Tensor, sapo: Union[Tensor, None] = None, sapo_mask: Union[Tensor, None] = None,
                his_sapo: Union[Tensor, None] = None, his_sapo_mask: Union[Tensor, None] = None,
                category: Union[Tensor, None] = None, his_category: Union[Tensor, None] = None):
        """Same contract as the reference forward (model.py:61-138): (mui [B,K,d], scores [B,C])."""
        batch_size, num_candidates, his_length = title.shape[0], title.shape[1], his_title.shape[1]
        title = title.view(batch_size * num_candidates, -1)
        title_mask = title_mask.view(batch_size * num_candidates, -1)
        sapo = sapo.view(batch_size * num_candidates, -1)          # unconditional, as model.py:93-94
        sapo_mask = sapo_mask.view(batch_size * num_candidates, -1)
        candidate_repr = self.news_encoder(title_encoding=title, title_attn_mask=title_mask,
                                           sapo_encoding=sapo, sapo_attn_mask=sapo_mask)
        candidate_repr = candidate_repr.view(batch_size, num_candidates, -1)
        his_title = his_title.view(batch_size * his_length, -1)
        his_title_mask = his_title_mask.view(batch_size * his_length, -1)
        his_sapo = his_sapo.view(batch_size * his_length, -1)
        his_sapo_mask = his_sapo_mask.view(batch_size * his_length, -1)
        history_repr = self.news_encoder(title_encoding=his_title, title_attn_mask=his_title_mask,
                                         sapo_encoding=his_sapo, sapo_attn_mask=his_sapo_mask)
        history_repr = history_repr.view(batch_size, his_length, -1)
        bias = self.category_bias(category, his_category) if self.use_category_bias else None
        return self.score(history_repr, his_mask, candidate_repr, category_bias=bias, return_user=True)
