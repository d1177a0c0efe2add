"""News-side precompute path, backed by libminer_hip.so (include/miner_news.h).

The reference scores an impression from the news encoder's output for its history and candidates
(src/model/model.py:113-138). Two of its products depend on one news item only:

* ``logits[n] = tanh(W1 e_n) · Qᵀ``   (PolyAttention.forward, model.py:171-174)
* ``proj[n]   = W2 e_n``              (TargetAwareAttention's linear, model.py:212, before GELU)

Over a news table they are computed once per news item (``precompute``); by linearity
``mui · W2ᵀ = A · proj[his]``, so ``score`` only gathers rows and runs the contractions over the
history and the candidates:

    nt = precompute(news_table, packed)          # once per table (or per model update)
    scores = score(nt, his_ids, his_mask, cand_ids)                  # [B, C] fp32
    scores, mui = score(nt, ..., return_user=True)                  # + multi_user_interest

Device tensors only: there is no CPU path. float32 is the parity mode, bfloat16 the throughput mode.
"""
from __future__ import annotations

import dataclasses
import os
from typing import Optional

import torch
from torch import Tensor

from . import _lib
from .ops import (PackedWeights, _as_packed, _contig, _dtype_code, _ptr, _require_device, _stream,
                  check_offsets)

MAX_CAND = 512          # MINER_NEWS_MAX_CAND: candidates per impression
X2W_MAX_L = 128         # MINER_NEWS_X2W_MAX_L: the fp32 pair-plane kernel's wide form (news_score_x2w)
X2W_MAX_K = 64          # MINER_NEWS_X2W_MAX_K
FUSED_MAX_K = 32        # the per-news precompute's packed Q (miner_pack_weights) holds K <= 32 rows


@dataclasses.dataclass
class PairPlanes:
    """fp32 tables as exact-sum fp16 pairs (miner_news_split_x2): the operands of the fp32 scoring
    kernel on the fp16 matrix cores (news_x2.hip). Same bytes as fp32; row r holds x / unit[r], one
    power-of-two unit per row (``*_unit``)."""
    table2: Tensor                # [n_news, 2d] fp16 (per 64-column chunk: 64 hi | 64 lo)
    table_unit: Tensor            # [n_news] fp32 row units
    proj2: Optional[Tensor]
    proj_unit: Optional[Tensor]


@dataclasses.dataclass
class NewsTable:
    """A news-embedding table with its per-news precompute (miner_news_precompute output)."""
    table: Tensor                 # [n_news, d] dtype
    logits: Tensor                # [n_news, K] fp32
    proj: Optional[Tensor]        # [n_news, d] dtype, None when built without w_target
    K: int
    x2: Optional[PairPlanes] = None   # fp32 tables only: the pair planes of table and proj

    @property
    def dtype(self) -> torch.dtype:
        return self.table.dtype

    @property
    def n_news(self) -> int:
        return self.table.shape[0]

    @property
    def d(self) -> int:
        return self.table.shape[1]


def supported(dtype: torch.dtype, L: int, d: int, Dc: int, K: int) -> bool:
    return _lib.lib().miner_news_supported(_dtype_code(dtype), L, d, Dc, K) == 0


def wide_supported(dtype: torch.dtype, L: int, d: int, Dc: int, K: int, n_news: Optional[int] = None) -> bool:
    """Shapes past the news kernels' K <= 32 / L <= 64 that the fp32 pair-plane kernel scores in its
    wide form (news_score_x2w: K <= 64, L <= 128, K % 4 == 0): fp32 tables with pair planes only
    (not under MINER_NEWS_FP32=mfma32), no in-kernel disagreement (the eval loss uses mui). With
    ``n_news``, the table must also fit the pair planes' 32-bit row offsets (x2_fits): precompute
    builds no pair planes past them, and the wide form has no other input."""
    return (dtype == torch.float32 and x2_enabled() and not supported(dtype, L, d, Dc, K)
            and 0 < L <= X2W_MAX_L and 0 < K <= X2W_MAX_K and K % 4 == 0
            and supported(dtype, 1, d, Dc, min(K, FUSED_MAX_K))
            and (n_news is None or x2_fits(n_news, d)))


def path_supported(dtype: torch.dtype, L: int, d: int, Dc: int, K: int, n_news: Optional[int] = None) -> bool:
    """The news-id path takes (dtype, L, d, Dc, K[, n_news]): the news kernels or the wide pair-plane form."""
    return supported(dtype, L, d, Dc, K) or wide_supported(dtype, L, d, Dc, K, n_news)


def _check_shape(dt: int, L: int, d: int, Dc: int, K: int) -> None:
    code = _lib.lib().miner_news_supported(dt, L, d, Dc, K)
    if code != 0:
        raise ValueError(f"news path: L={L} d={d} Dc={Dc} K={K}: {_lib.lib().miner_strerror(code).decode()} "
                         "(L <= 64, K <= 32 and K % 4 == 0, d % 64 == 0)")


def x2_enabled() -> bool:
    """fp32 scoring on the fp16 matrix cores (news_x2.hip) unless MINER_NEWS_FP32=mfma32 selects the
    fp32-MFMA kernel news_score32 (A/B and the exact-fp32 sub-line of the bench)."""
    return os.environ.get("MINER_NEWS_FP32", "x2") != "mfma32"


def x2_fits(n_news: int, d: int) -> bool:
    """The pair planes of an [n_news, d] table fit the x2 kernel's 32-bit row offsets
    (miner_score_news_x2 returns MINER_ESHAPE past n_news·d·4 = 2^32 - 1, e.g. > 1.39M news at d = 768)."""
    return n_news * d * 4 <= 0xFFFFFFFF


def split_x2(src: Tensor, out: Optional[Tensor] = None, unit: Optional[Tensor] = None):
    """fp32 [n, d] -> (pairs [n, 2d] fp16, row units [n] fp32) (miner_news_split_x2)."""
    _require_device(src)
    src = _contig(src)
    if src.dtype != torch.float32 or src.dim() != 2:
        raise ValueError("split_x2 takes an fp32 [n, d] table")
    n, d = src.shape
    if out is None or tuple(out.shape) != (n, 2 * d):
        out = torch.empty((n, 2 * d), device=src.device, dtype=torch.float16)
    if unit is None or unit.numel() != n:
        unit = torch.empty((n,), device=src.device, dtype=torch.float32)
    with torch.cuda.device(src.device):
        rc = _lib.lib().miner_news_split_x2(_stream(src.device), _ptr(src), n, d, _ptr(out), _ptr(unit))
    _lib.check(rc, "miner_news_split_x2")
    return out, unit


def precompute(news_table: Tensor, w_poly, context_codes: Optional[Tensor] = None,
               w_target: Optional[Tensor] = None, *, with_proj: bool = True,
               out: Optional[NewsTable] = None, x2: Optional[bool] = None) -> NewsTable:
    """logits = tanh(E·W1ᵀ)·Qᵀ [n_news, K] fp32 and proj = E·W2ᵀ [n_news, d] for a news table
    (model.py:171-174, :212). ``w_poly`` is a PackedWeights or the raw weights
    (w_poly [Dc,d], context_codes [K,Dc], w_target [d,d]); ``out`` reuses its buffers.
    fp32 tables also get their fp16 pair planes (``x2``, default: x2_enabled()), the operands of
    the fp32 scoring kernel on the fp16 matrix cores."""
    _require_device(news_table, context_codes, w_target)
    if not isinstance(w_poly, PackedWeights):
        _require_device(w_poly)
    table = _contig(news_table)
    dtype = table.dtype
    dt = _dtype_code(dtype)
    pw = _as_packed(w_poly, context_codes, w_target if with_proj else None, dtype)
    if with_proj and not pw.has_target:
        raise ValueError("with_proj needs weights packed with w_target (target_aware_attn.linear.weight)")
    n_news, d = table.shape
    if pw.d != d:
        raise ValueError(f"packed weights are for d={pw.d}, the table has d={d}")
    wide_k = pw.K > FUSED_MAX_K
    if wide_k:
        # K > 32 (the wide pair-plane kernel): the logits in 32-interest slices of Q, each through the
        # same precompute kernel (tanh(W1·e)·Q_sliceᵀ, exact fp32 per element as for K <= 32)
        if not (0 < pw.K <= X2W_MAX_K and pw.K % 4 == 0) or pw.src is None or pw.src[0] is None:
            raise ValueError(f"news path: K={pw.K} needs K <= {X2W_MAX_K}, K % 4 == 0 and the source weights")
        _check_shape(dt, 1, d, pw.Dc, FUSED_MAX_K)
    else:
        _check_shape(dt, 1, d, pw.Dc, pw.K)
    if out is not None and out.table.data_ptr() == table.data_ptr() and tuple(out.logits.shape) == (n_news, pw.K) \
            and (out.proj is not None) == with_proj:
        logits, proj = out.logits, out.proj
    else:
        logits = torch.empty((n_news, pw.K), device=table.device, dtype=torch.float32)
        proj = torch.empty((n_news, d), device=table.device, dtype=dtype) if with_proj else None
    want_x2 = dtype == torch.float32 and (x2_enabled() if x2 is None else x2)
    if want_x2 and not x2_fits(n_news, d):
        # the pair-plane kernel addresses a row piece with a 32-bit byte offset (news_x2.hip,
        # MINER_ESHAPE past it): such a table scores on the fp32-MFMA kernel instead
        if x2:
            raise ValueError(f"x2=True: a {n_news} x {d} table is past the pair-plane kernel's 4 GiB "
                             "row-offset range (n_news * d * 4 < 2^32)")
        want_x2 = False
    # fp32: the products on fp16 pairs for the pair-plane kernel (MINER_DTYPE_F32), on the fp32 MFMA
    # for the fp32-MFMA scoring kernel (MINER_DTYPE_F32_MFMA)
    pre_dt = _lib.DTYPE_F32_MFMA if dt == _lib.DTYPE_F32 and not want_x2 else dt
    with torch.cuda.device(table.device):
        if not wide_k:
            rc = _lib.lib().miner_news_precompute(_stream(table.device), pre_dt, _ptr(table), n_news, _ptr(pw.buf), d,
                                                  pw.Dc, pw.K, _ptr(logits), _ptr(proj))
        else:
            from .ops import pack_weights
            w1, q, w2 = pw.src
            for k0 in range(0, pw.K, FUSED_MAX_K):
                k1 = min(k0 + FUSED_MAX_K, pw.K)
                first = k0 == 0
                part = pack_weights(w1, q[k0:k1], w2 if (first and with_proj) else None, dtype=dtype)
                lg = torch.empty((n_news, k1 - k0), device=table.device, dtype=torch.float32)
                rc = _lib.lib().miner_news_precompute(_stream(table.device), pre_dt, _ptr(table), n_news, _ptr(part.buf),
                                                      d, pw.Dc, k1 - k0, _ptr(lg), _ptr(proj) if first else None)
                if rc != 0:
                    break
                logits[:, k0:k1].copy_(lg)
    _lib.check(rc, "miner_news_precompute")
    planes = None
    if want_x2:
        o = out.x2 if out is not None and out.x2 is not None else None
        t2, tws = split_x2(table, None if o is None else o.table2, None if o is None else o.table_unit)
        p2, pws = (split_x2(proj, None if o is None else o.proj2, None if o is None else o.proj_unit)
                   if proj is not None else (None, None))
        planes = PairPlanes(t2, tws, p2, pws)
    return NewsTable(table, logits, proj, pw.K, planes)


def score(nt: NewsTable, his_ids: Tensor, his_mask: Tensor, cand_ids: Optional[Tensor] = None, *,
          score_type: str = "weighted", cand_offsets: Optional[Tensor] = None,
          his_bias: Optional[Tensor] = None, return_user: bool = False, validate: bool = True,
          user_out: Optional[Tensor] = None, x2: Optional[bool] = None, disagreement: bool = False):
    """Miner.forward after the news encoder (model.py:113-138) for impressions given as news ids.

    his_ids [B, L] int, his_mask [B, L] bool (True = real click), cand_ids [B, C] (dense) or [N]
    with cand_offsets [B+1] int32 (ragged), his_bias [B, L] fp32 (category bias averaged over the
    candidates, model.py:176) or None. Returns scores ([B, C] / [N] fp32) and, if return_user,
    mui [B, K, d] fp32. score_type 'none' returns mui only. ``validate`` checks ids / offsets;
    ``user_out`` is an optional caller-owned fp32 [>= B, K, d] buffer for mui. fp32 tables with
    pair planes score on the fp16 matrix cores (``x2``, default x2_enabled()), else on the fp32 MFMA.
    ``disagreement`` (fp32 pair-plane tables only) also returns D [B] fp32, the eval loss's
    per-impression mean pairwise cosine of the K interests with the diagonal zeroed (loss.py:81),
    formed in the kernel without writing mui; it is appended to the returned tuple.
    """
    st = _lib.SCORE_TYPES.get(score_type)
    if st is None:
        raise ValueError("Invalid method of aggregating matching score")  # model.py:136
    _require_device(his_ids, his_mask, cand_ids, cand_offsets, his_bias)
    dt = _dtype_code(nt.dtype)
    B, L = his_ids.shape
    d, K = nt.d, nt.K
    wide = not supported(nt.dtype, L, d, 1, K)
    if wide:
        if not (nt.dtype == torch.float32 and 0 < L <= X2W_MAX_L and 0 < K <= X2W_MAX_K and K % 4 == 0):
            _check_shape(dt, L, d, 1, K)
        if nt.x2 is None or not (x2_enabled() if x2 is None else x2):
            raise ValueError(f"news path: L={L} K={K} is past the news kernels (L <= 64, K <= 32); the wide "
                             "form needs an fp32 table with pair planes (news.precompute(x2=True))")
        if disagreement:
            raise ValueError("disagreement=True: the wide form (L > 64 or K > 32) writes mui instead "
                             "(return_user=True)")
    if st == _lib.SCORE_WEIGHTED and nt.proj is None:
        raise ValueError("score_type='weighted' needs the table precomputed with w_target (with_proj=True)")
    dev = nt.table.device
    hid = _contig(his_ids, torch.int32)
    mask = _contig(his_mask)
    if mask.dtype != torch.bool:
        mask = mask != 0
    if tuple(mask.shape) != (B, L):
        raise ValueError(f"his_mask must be [{B},{L}]")
    mask = mask.view(torch.uint8)
    if his_bias is not None:
        his_bias = _contig(his_bias, torch.float32)
        if tuple(his_bias.shape) != (B, L):
            raise ValueError(f"his_bias must be [{B},{L}] (category bias averaged over candidates)")
    cid, offs, C, scores = None, None, 0, None
    if st != _lib.SCORE_NONE:
        if cand_ids is None:
            raise ValueError("cand_ids required")
        if cand_offsets is None:
            if cand_ids.dim() != 2 or cand_ids.shape[0] != B:
                raise ValueError(f"dense cand_ids must be [{B},C]")
            C = cand_ids.shape[1]
            if C > MAX_CAND:
                raise ValueError(f"at most {MAX_CAND} candidates per impression on the news path (got {C})")
            cid = _contig(cand_ids, torch.int32)
            scores = torch.empty((B, C), device=dev, dtype=torch.float32)
        else:
            cid = _contig(cand_ids.reshape(-1), torch.int32)
            offs = _contig(cand_offsets, torch.int32)
            if validate:
                check_offsets(offs, B, cid.numel())
                if B and int((offs[1:] - offs[:-1]).max()) > MAX_CAND:
                    raise ValueError(f"at most {MAX_CAND} candidates per impression on the news path")
            scores = torch.empty((cid.numel(),), device=dev, dtype=torch.float32)
    if validate:
        for ids, what in ((hid, "his_ids"), (cid, "cand_ids")):
            if ids is not None and ids.numel() and (int(ids.min()) < 0 or int(ids.max()) >= nt.n_news):
                raise ValueError(f"{what} must index the news table [0, {nt.n_news})")
    mui = None
    if return_user or (st == _lib.SCORE_NONE and not disagreement):
        if user_out is not None:        # a caller-owned [>= B, K, d] fp32 buffer, reused across calls
            if user_out.dtype != torch.float32 or user_out.dim() != 3 or user_out.shape[0] < B or \
                    tuple(user_out.shape[1:]) != (K, d) or not user_out.is_contiguous():
                raise ValueError(f"user_out must be a contiguous fp32 [>={B},{K},{d}] tensor")
            mui = user_out[:B]
        else:
            mui = torch.empty((B, K, d), device=dev, dtype=torch.float32)
    use_x2 = nt.x2 is not None and dt == _lib.DTYPE_F32 and (x2_enabled() if x2 is None else x2)
    dis = None
    if disagreement:
        if not use_x2:
            raise ValueError("disagreement=True needs an fp32 table with pair planes (news.precompute(x2=True))")
        dis = torch.empty((B,), device=dev, dtype=torch.float32)
    with torch.cuda.device(dev):
        if use_x2:
            px = nt.x2
            rc = _lib.lib().miner_score_news_x2(_stream(dev), st, _ptr(px.table2), _ptr(px.table_unit), _ptr(nt.logits),
                                                _ptr(px.proj2), _ptr(px.proj_unit), nt.n_news, _ptr(hid), _ptr(mask),
                                                _ptr(his_bias), _ptr(cid), _ptr(offs), B, L, C, d, K, _ptr(scores),
                                                _ptr(mui), _ptr(dis))
        else:
            # MINER_NEWS_F32X6=1 (read per call, a Python-side switch): news_score32's bf16x6 form
            kdt = _lib.DTYPE_F32_X6 if dt == _lib.DTYPE_F32 and os.environ.get("MINER_NEWS_F32X6") else dt
            rc = _lib.lib().miner_score_news(_stream(dev), kdt, st, _ptr(nt.table), _ptr(nt.logits), _ptr(nt.proj),
                                             nt.n_news, _ptr(hid), _ptr(mask), _ptr(his_bias), _ptr(cid), _ptr(offs),
                                             B, L, C, d, K, _ptr(scores), _ptr(mui))
    _lib.check(rc, "miner_score_news_x2" if use_x2 else "miner_score_news")
    if st == _lib.SCORE_NONE:
        return (mui, dis) if disagreement else mui
    out = (scores, mui) if return_user else (scores,)
    if disagreement:
        out = out + (dis,)
    return out if len(out) > 1 else out[0]
