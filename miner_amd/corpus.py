"""Full-corpus ranking on MI355X (BASELINE config 5: 1M users x 200k news, history 200, K=64,
d=768, fp16), backed by libminer_hip.so (include/miner_corpus.h).

    packed = pack_encoder(w_poly, context_codes, w_target, dtype=torch.float16)
    mui, proj = encode_users(history, his_mask, packed)                 # or table + his_ids
    top_scores, top_ids = rank_topk(mui, proj, news_table, topk=100)   # never materialises U x N

The click score of (user, news) is the reference's (src/model/model.py:127-134, 213-214) with the
impression's candidate set replaced by the whole news table; ties rank the lower news id first.
Device tensors only: there is no CPU path.
"""
from __future__ import annotations

import dataclasses
import os
from typing import Optional

import torch
from torch import Tensor

from . import _lib
from .ops import _contig, _ptr, _require_device, _stream

_DT = {torch.float32: _lib.DTYPE_F32, torch.bfloat16: _lib.DTYPE_BF16, torch.float16: _lib.DTYPE_F16}
MAX_L, MAX_K, MAX_TOPK = 256, 64, 256


def _code(dtype: torch.dtype) -> int:
    try:
        return _DT[dtype]
    except KeyError:
        raise TypeError(f"unsupported dtype {dtype}: float32 (parity), bfloat16 or float16")


@dataclasses.dataclass
class EncoderWeights:
    """miner_encoder_pack() output."""
    buf: Tensor
    dtype: torch.dtype
    d: int
    Dc: int
    K: int
    has_target: bool


def pack_encoder(w_poly: Tensor, context_codes: Tensor, w_target: Optional[Tensor] = None,
                 dtype: Optional[torch.dtype] = None) -> EncoderWeights:
    """poly_attn.linear.weight [Dc,d], poly_attn.context_codes [K,Dc], target_aware_attn.linear.weight
    [d,d] (model.py:155-157, :198) -> the user encoder's packed layout (K <= 64, Dc <= 256)."""
    _require_device(w_poly, context_codes, w_target)
    dtype = dtype or w_poly.dtype
    dt = _code(dtype)
    w1, q, w2 = _contig(w_poly, dtype), _contig(context_codes, dtype), _contig(w_target, dtype)
    Dc, d = w1.shape
    K = q.shape[0]
    if q.shape[1] != Dc or (w2 is not None and tuple(w2.shape) != (d, d)):
        raise ValueError("weight shapes do not match (w_poly [Dc,d], context_codes [K,Dc], w_target [d,d])")
    nbytes = _lib.lib().miner_encoder_packed_bytes(dt, d, Dc, K)
    if nbytes == 0:
        raise ValueError(f"d={d} Dc={Dc} K={K} not supported (K <= 64, Dc <= 256, d <= 768, d % 64 == 0)")
    buf = torch.empty(nbytes, dtype=torch.uint8, device=w1.device)
    with torch.cuda.device(w1.device):
        rc = _lib.lib().miner_encoder_pack(_stream(w1.device), dt, _ptr(w1), _ptr(q), _ptr(w2), d, Dc, K, _ptr(buf))
    _lib.check(rc, "miner_encoder_pack")
    return EncoderWeights(buf, dtype, d, Dc, K, w2 is not None)


def encode_users(history: Tensor, his_mask: Tensor, packed: EncoderWeights, *, his_ids: Optional[Tensor] = None,
                 his_bias: Optional[Tensor] = None, with_proj: bool = True, return_f32: bool = False):
    """PolyAttention (model.py:159-185) per user, and proj = gelu(mui · W2ᵀ) (model.py:212).

    history [U,L,d] (dense), or the news table [n_news,d] with his_ids [U,L]; his_mask [U,L] bool;
    his_bias [U,L] fp32 or None. Returns (mui, proj) in the packed dtype ([U,K,d]; proj None when
    with_proj is False), plus mui in fp32 when return_f32.
    """
    _require_device(history, his_mask, his_ids, his_bias)
    dt = _code(packed.dtype)
    src = _contig(history, packed.dtype)
    mask = _contig(his_mask, torch.bool).view(torch.uint8)
    U, L = mask.shape
    d, K = packed.d, packed.K
    ids = None
    n_news = 0
    if his_ids is not None:
        ids = _contig(his_ids, torch.int32)
        n_news = src.shape[0]
        if ids.numel() and (int(ids.min()) < 0 or int(ids.max()) >= n_news):
            raise IndexError(f"his_ids out of range [0, {n_news})")
    elif tuple(src.shape) != (U, L, d):
        raise ValueError(f"history must be [{U},{L},{d}]")
    if not 1 <= L <= MAX_L:
        raise ValueError(f"history length {L} outside [1, {MAX_L}]")
    if with_proj and not packed.has_target:
        raise ValueError("the packed weights hold no w_target: pass with_proj=False")
    bias = _contig(his_bias, torch.float32)
    dev = src.device
    mui = torch.empty(U, K, d, dtype=packed.dtype, device=dev)
    proj = torch.empty(U, K, d, dtype=packed.dtype, device=dev) if with_proj else None
    m32 = torch.empty(U, K, d, dtype=torch.float32, device=dev) if return_f32 else None
    with torch.cuda.device(dev):
        rc = _lib.lib().miner_encode_users(_stream(dev), dt, _ptr(src), _ptr(ids), n_news, _ptr(mask), _ptr(bias),
                                           _ptr(packed.buf), U, L, d, packed.Dc, K, _ptr(m32), _ptr(mui), _ptr(proj))
    _lib.check(rc, "miner_encode_users")
    return (mui, proj, m32) if return_f32 else (mui, proj)


def rank_topk(user_mui: Tensor, user_proj: Optional[Tensor], news: Tensor, topk: int, *,
              score_type: str = "weighted"):
    """Top-k news per user by the click score, best first: (scores [U,topk] fp32, ids [U,topk]
    int32); entries past the table size are (-inf, -1)."""
    st = _lib.SCORE_TYPES.get(score_type)
    if st is None or st == _lib.SCORE_NONE:
        raise ValueError("Invalid method of aggregating matching score")  # model.py:136
    _require_device(user_mui, user_proj, news)
    dtype = user_mui.dtype
    dt = _code(dtype)
    mui = _contig(user_mui, dtype)
    proj = _contig(user_proj, dtype) if st == _lib.SCORE_WEIGHTED else None
    if st == _lib.SCORE_WEIGHTED and proj is None:
        raise ValueError("score_type 'weighted' needs user_proj")
    tab = _contig(news, dtype)
    U, K, d = mui.shape
    N = tab.shape[0]
    if tab.shape[1] != d or (proj is not None and proj.shape != mui.shape):
        raise ValueError("shape mismatch between user vectors and the news table")
    if not 1 <= topk <= MAX_TOPK:
        raise ValueError(f"topk must be in [1, {MAX_TOPK}]")
    dev = mui.device
    top_s = torch.empty(U, topk, dtype=torch.float32, device=dev)
    top_i = torch.empty(U, topk, dtype=torch.int32, device=dev)
    # a workspace only where the split form runs: the library's recommendation (U <= 510 on a 256-CU
    # device), or MINER_RK_SPLIT=1 / 0 (read here, per call: a test / A/B switch) forcing either form
    lib = _lib.lib()
    force = os.environ.get("MINER_RK_SPLIT", "")
    split = force == "1" if force in ("0", "1") else bool(lib.miner_rank_topk_split_recommended(U))
    nws = int(lib.miner_rank_topk_workspace_bytes(U, topk)) if split else 0
    ws = torch.empty(nws, dtype=torch.uint8, device=dev) if nws else None
    with torch.cuda.device(dev):
        rc = _lib.lib().miner_rank_topk_ws(_stream(dev), dt, st, _ptr(mui), _ptr(proj), _ptr(tab), U, N, d, K, topk,
                                           _ptr(top_s), _ptr(top_i), _ptr(ws), nws)
    _lib.check(rc, "miner_rank_topk")
    return top_s, top_i


def rank_corpus(news: Tensor, his_ids: Tensor, his_mask: Tensor, packed: EncoderWeights, topk: int, *,
                his_bias: Optional[Tensor] = None, score_type: str = "weighted", batch: int = 16384,
                out: Optional[tuple] = None):
    """BASELINE config 5 on one GPU's share of the users: every user (his_ids [U,L] into the news
    table [N,d], his_mask [U,L]) encoded and ranked against the whole table, ``batch`` users per
    encode + rank pair so that the [batch,K,d] user vectors are all that is ever held (125,000 users
    at K = 64, d = 768, fp16 would be 24.6 GB of mui + proj at once). Returns (scores [U,topk] fp32,
    ids [U,topk] int32), best first: each user's list is independent of the batching
    (tests/test_gpu_fullsize.py). ``out`` = preallocated (scores, ids) to write into."""
    if batch <= 0:
        raise ValueError("batch must be positive")
    U = his_ids.shape[0]
    dev = news.device
    top_s, top_i = out if out is not None else (torch.empty(U, topk, dtype=torch.float32, device=dev),
                                                torch.empty(U, topk, dtype=torch.int32, device=dev))
    with_proj = score_type == "weighted"
    for u0 in range(0, U, batch):
        u1 = min(U, u0 + batch)
        mui, proj = encode_users(news, his_mask[u0:u1], packed, his_ids=his_ids[u0:u1],
                                 his_bias=None if his_bias is None else his_bias[u0:u1], with_proj=with_proj)
        s, i = rank_topk(mui, proj, news, topk, score_type=score_type)
        top_s[u0:u1] = s
        top_i[u0:u1] = i
    return top_s, top_i
