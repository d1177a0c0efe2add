"""torch-facing wrappers of the C ABI (include/miner_score.h).

PyTorch is plumbing here: it owns device memory and the current HIP stream; the arithmetic runs in
libminer_hip.so. Every call enqueues on ``torch.cuda.current_stream()`` and returns without
synchronising. Inputs must be device tensors: there is no CPU path.

Weights go through ``pack_weights`` once (the kernel's tiled layout); ``score`` also accepts the
raw ``(w_poly, context_codes, w_target)`` tensors and packs them on the fly.
"""
from __future__ import annotations

import dataclasses
import os

import torch

from . import _lib

_DTYPES = {torch.float32: _lib.DTYPE_F32, torch.bfloat16: _lib.DTYPE_BF16}
FUSED_MAX_K, FUSED_MAX_L = 32, 64       # miner_fused (miner_score.h); past them: the wide path
WIDE_MAX_K, WIDE_MAX_L = 64, 256        # miner_encode_users + miner_score_wide (miner_wide.h)


def _ptr(t):
    return None if t is None else t.data_ptr()


def _require_device(*ts):
    for t in ts:
        if t is not None and isinstance(t, torch.Tensor) and t.device.type != "cuda":
            raise RuntimeError("miner_amd ops run on the GPU only (got a tensor on %s); the scoring "
                               "path has no CPU fallback" % t.device)


def _contig(t, dtype=None):
    if t is None:
        return None
    if dtype is not None and t.dtype != dtype:
        t = t.to(dtype)
    return t.contiguous()


def _kernel_dtype(dt: int) -> int:
    """The dtype code a dense-row launch passes: fp32 runs its S1 / S5 contractions as bf16x6 by
    default; MINER_DENSE_FP32=mfma32 (read per call, a Python-side switch) asks the library for the
    exact fp32-MFMA form (MINER_DTYPE_F32_MFMA)."""
    if dt == _lib.DTYPE_F32 and os.environ.get("MINER_DENSE_FP32") == "mfma32":
        return _lib.DTYPE_F32_MFMA
    return dt


def _dtype_code(dtype: torch.dtype) -> int:
    try:
        return _DTYPES[dtype]
    except KeyError:
        raise TypeError(f"unsupported dtype {dtype}: use float32 (parity) or bfloat16 (throughput)")


def _stream(dev):
    return torch.cuda.current_stream(dev).cuda_stream


def check_offsets(cand_offsets: torch.Tensor, B: int, N: int) -> None:
    """Host-side validation of CSR candidate offsets (one device->host copy)."""
    o = cand_offsets.detach().to("cpu", torch.int64)
    if o.numel() != B + 1 or int(o[0]) != 0 or int(o[-1]) != N or bool((o[1:] < o[:-1]).any()):
        raise ValueError(f"cand_offsets must be a non-decreasing int32 [B+1] array from 0 to {N}")


@dataclasses.dataclass
class PackedWeights:
    """miner_pack_weights() output: one device buffer holding W1, Q and W2 in the kernel layout.

    ``buf`` is None when (d, Dc, K) is past the fused kernel (K > 32): such weights are scored by
    the wide path (include/miner_wide.h), whose user-encoder pack is built from ``src`` on first use.
    """
    buf: torch.Tensor | None
    dtype: torch.dtype
    d: int
    Dc: int
    K: int
    has_target: bool
    src: tuple | None = None                     # (w_poly, context_codes, w_target), dtype, detached
    wide: object | None = dataclasses.field(default=None, repr=False)   # corpus.EncoderWeights cache


def pack_weights(w_poly: torch.Tensor, context_codes: torch.Tensor, w_target: torch.Tensor | None = None,
                 dtype: torch.dtype | None = None) -> PackedWeights:
    """Pack poly_attn.linear.weight [Dc,d], poly_attn.context_codes [K,Dc] and (optionally)
    target_aware_attn.linear.weight [d,d] (model.py:155-157, :198) for the kernels."""
    _require_device(w_poly, context_codes, w_target)
    dtype = dtype or w_poly.dtype
    dt = _dtype_code(dtype)
    w1 = _contig(w_poly, dtype)
    q = _contig(context_codes, dtype)
    w2 = _contig(w_target, dtype)
    Dc, d = w1.shape
    K = q.shape[0]
    if q.shape[1] != Dc:
        raise ValueError(f"context_codes must be [K,{Dc}], got {tuple(q.shape)}")
    if w2 is not None and tuple(w2.shape) != (d, d):
        raise ValueError(f"w_target must be [{d},{d}], got {tuple(w2.shape)}")
    src = tuple(None if t is None else t.detach() for t in (w1, q, w2))
    nbytes = _lib.lib().miner_packed_weights_bytes(dt, d, Dc, K)
    if nbytes == 0:
        if _lib.lib().miner_wide_supported(dt, 1, d, Dc, K) != 0:
            raise ValueError(f"weights d={d} Dc={Dc} K={K} not supported by this build "
                             f"(K <= {WIDE_MAX_K}, Dc <= 256, d <= 768)")
        return PackedWeights(None, dtype, d, Dc, K, w2 is not None, src)      # wide path only
    buf = torch.empty(nbytes, dtype=torch.uint8, device=w1.device)
    with torch.cuda.device(w1.device):
        rc = _lib.lib().miner_pack_weights(_stream(w1.device), dt, _ptr(w1), _ptr(q), _ptr(w2), d, Dc, K, _ptr(buf))
    _lib.check(rc, "miner_pack_weights")
    return PackedWeights(buf, dtype, d, Dc, K, w2 is not None, src)


def pack_target_weights(w_target: torch.Tensor, dtype: torch.dtype | None = None) -> PackedWeights:
    """Pack target_aware_attn.linear.weight [d,d] (model.py:198) alone, for ``target_aware``
    (TargetAwareAttention on its own has no PolyAttention weights: Dc = K = 0 in the result)."""
    _require_device(w_target)
    dtype = dtype or w_target.dtype
    dt = _dtype_code(dtype)
    w2 = _contig(w_target, dtype)
    if w2.dim() != 2 or w2.shape[0] != w2.shape[1]:
        raise ValueError(f"w_target must be [d,d], got {tuple(w2.shape)}")
    d = w2.shape[0]
    nbytes = _lib.lib().miner_target_weights_bytes(dt, d)
    if nbytes == 0:
        raise ValueError(f"w_target d={d} not supported by this build (d % 32 == 0, d <= 1024)")
    buf = torch.empty(nbytes, dtype=torch.uint8, device=w2.device)
    with torch.cuda.device(w2.device):
        rc = _lib.lib().miner_pack_target_weights(_stream(w2.device), dt, _ptr(w2), d, _ptr(buf))
    _lib.check(rc, "miner_pack_target_weights")
    return PackedWeights(buf, dtype, d, 0, 0, True, (None, None, w2.detach()))


def _check_mask_bias(his_mask: torch.Tensor, his_bias, B: int, L: int):
    """his_mask [B,L] (bool or 0/1) -> contiguous uint8 view; his_bias [B,L] fp32 or None."""
    mask = _contig(his_mask)
    if mask.dtype != torch.bool:
        mask = mask != 0
    if tuple(mask.shape) != (B, L):
        raise ValueError(f"his_mask must be [{B},{L}], got {tuple(mask.shape)}")
    if his_bias is not None:
        his_bias = _contig(his_bias, torch.float32)
        if tuple(his_bias.shape) != (B, L):
            raise ValueError(f"his_bias must be [{B},{L}] (category bias averaged over candidates), "
                             f"got {tuple(his_bias.shape)}")
    return mask.view(torch.uint8), his_bias


def _as_packed(w_poly, context_codes, w_target, dtype) -> PackedWeights:
    if isinstance(w_poly, PackedWeights):
        if w_poly.dtype != dtype:
            raise TypeError(f"packed weights are {w_poly.dtype}, activations {dtype}")
        return w_poly
    return pack_weights(w_poly, context_codes, w_target, dtype=dtype)


def _fused_or_wide(dt: int, L: int, d: int, Dc: int, K: int) -> bool:
    """True when the fused kernel takes the shape, False when the wide path does; raises when
    neither does (the reference itself has no limit: model.py:18-21, :159-185)."""
    code = _lib.lib().miner_supported(dt, L, d, Dc, K)
    if code == 0:
        return True
    if _lib.lib().miner_wide_supported(dt, L, d, Dc, K) == 0:
        return False
    raise ValueError(f"shape L={L} d={d} Dc={Dc} K={K}: {_lib.lib().miner_strerror(code).decode()} "
                     f"(fused kernel: L <= {FUSED_MAX_L}, K <= {FUSED_MAX_K}; wide path: L <= {WIDE_MAX_L}, "
                     f"K <= {WIDE_MAX_K}, Dc <= 256, d <= 768)")


def _wide_encoder(pw: PackedWeights):
    """The user-encoder pack (miner_encoder_pack, corpus.h) of these weights, built once."""
    if pw.wide is None:
        if pw.src is None or pw.src[0] is None:
            raise ValueError("these packed weights carry no PolyAttention source tensors for the wide path")
        from . import corpus
        pw.wide = corpus.pack_encoder(pw.src[0], pw.src[1], pw.src[2], dtype=pw.dtype)
    return pw.wide


def _score_wide(pw: PackedWeights, st: int, rows: torch.Tensor, his_ids, mask_u8: torch.Tensor, his_bias,
                cand: torch.Tensor, cand_ids, offs, B: int, C: int, n_out: int, return_user: bool):
    """Wide path (include/miner_wide.h): miner_encode_users (PolyAttention and, for 'weighted',
    gelu(mui·W2ᵀ); model.py:159-185, :212) then miner_score_wide (model.py:127-136, :213-214)."""
    from . import corpus
    enc = _wide_encoder(pw)
    weighted = st == _lib.SCORE_WEIGHTED
    if weighted and not enc.has_target:
        raise ValueError("score_type='weighted' needs weights packed with w_target")
    f32 = pw.dtype == torch.float32
    res = corpus.encode_users(rows, mask_u8.view(torch.bool), enc, his_ids=his_ids, his_bias=his_bias,
                              with_proj=weighted, return_f32=return_user and not f32)
    mui, proj = res[0], res[1]
    d, K = pw.d, pw.K
    dev = rows.device
    shape = (B, C) if offs is None else (n_out,)
    scores = torch.empty(shape, device=dev, dtype=torch.float32)
    n_news = rows.shape[0] if cand_ids is not None else 0
    with torch.cuda.device(dev):
        rc = _lib.lib().miner_score_wide(_stream(dev), _dtype_code(pw.dtype), st, _ptr(mui), _ptr(proj), _ptr(cand),
                                         _ptr(cand_ids), n_news, _ptr(offs), None, B, C, d, K, _ptr(scores))
    _lib.check(rc, "miner_score_wide")
    if return_user:
        return scores, (mui if f32 else res[2])
    return scores


def score(history: torch.Tensor, his_mask: torch.Tensor, candidates: torch.Tensor,
          w_poly, context_codes: torch.Tensor | None = None, w_target: torch.Tensor | None = None, *,
          score_type: str = "weighted", cand_offsets: torch.Tensor | None = None,
          his_bias: torch.Tensor | None = None, return_user: bool = False,
          validate_offsets: bool = True):
    """Fused PolyAttention -> Cand·muiᵀ -> aggregation (src/model/model.py:113-138).

    history [B,L,d], his_mask [B,L] bool, candidates [B,C,d] (dense) or [N,d] with
    cand_offsets [B+1] int32 (ragged). ``w_poly`` is a PackedWeights, or the raw weight tensors are
    passed as (w_poly, context_codes, w_target). Activations float32 (parity) or bfloat16.
    Returns scores ([B,C] dense / [N] ragged, fp32) and, if return_user, mui [B,K,d] fp32.
    """
    st = _lib.SCORE_TYPES.get(score_type)
    if st is None or st == _lib.SCORE_NONE:
        raise ValueError("Invalid method of aggregating matching score")  # model.py:136
    _require_device(history, his_mask, candidates, context_codes, w_target, cand_offsets, his_bias)
    if not isinstance(w_poly, PackedWeights):
        _require_device(w_poly)
    tdt = history.dtype
    dt = _dtype_code(tdt)
    history = _contig(history)
    candidates = _contig(candidates, tdt)
    B, L, d = history.shape
    if isinstance(w_poly, PackedWeights):
        Dc, K = w_poly.Dc, w_poly.K
    else:
        K, Dc = context_codes.shape
        if tuple(w_poly.shape) != (Dc, d):
            raise ValueError(f"w_poly must be [{Dc},{d}], got {tuple(w_poly.shape)}")
    fused = _fused_or_wide(dt, L, d, Dc, K)
    if st == _lib.SCORE_WEIGHTED and not isinstance(w_poly, PackedWeights) and w_target is None:
        raise ValueError("score_type='weighted' needs w_target (target_aware_attn.linear.weight)")
    pw = _as_packed(w_poly, context_codes, w_target if st == _lib.SCORE_WEIGHTED else None, tdt)
    fused = fused and pw.buf is not None
    if pw.d != d:
        raise ValueError(f"packed weights are for d={pw.d}, history has d={d}")
    if pw.Dc == 0:
        raise ValueError("packed weights hold no PolyAttention part (pack_target_weights output)")
    if st == _lib.SCORE_WEIGHTED and not pw.has_target:
        raise ValueError("score_type='weighted' needs weights packed with w_target")
    mask, his_bias = _check_mask_bias(his_mask, his_bias, B, L)
    if cand_offsets is None:
        if candidates.dim() != 3 or candidates.shape[0] != B or candidates.shape[2] != d:
            raise ValueError(f"dense candidates must be [{B},C,{d}]")
        C = candidates.shape[1]
        scores = torch.empty((B, C), device=history.device, dtype=torch.float32)
        offs = None
    else:
        if candidates.dim() != 2 or candidates.shape[1] != d:
            raise ValueError(f"ragged candidates must be [N,{d}]")
        offs = _contig(cand_offsets, torch.int32)
        if validate_offsets:
            check_offsets(offs, B, candidates.shape[0])
        C = 0
        scores = torch.empty((candidates.shape[0],), device=history.device, dtype=torch.float32)
    if not fused:
        return _score_wide(pw, st, history, None, mask, his_bias, candidates, None, offs, B, C,
                           scores.numel(), return_user)
    mui = torch.empty((B, K, d), device=history.device, dtype=torch.float32) if return_user else None
    with torch.cuda.device(history.device):
        rc = _lib.lib().miner_score(_stream(history.device), _kernel_dtype(dt), st, _ptr(history), _ptr(mask), _ptr(his_bias),
                                    _ptr(candidates), _ptr(offs), _ptr(pw.buf), B, L, C, d, Dc, K,
                                    _ptr(scores), _ptr(mui))
    _lib.check(rc, "miner_score")
    return (scores, mui) if return_user else scores


def _check_ids(ids: torch.Tensor, n: int, what: str) -> None:
    if ids.numel() and (int(ids.min()) < 0 or int(ids.max()) >= n):
        raise ValueError(f"{what} must index the news table [0, {n})")


def score_gather(news_table: torch.Tensor, his_ids: torch.Tensor, his_mask: torch.Tensor, cand_ids: torch.Tensor,
                 w_poly, context_codes: torch.Tensor | None = None, w_target: torch.Tensor | None = None, *,
                 score_type: str = "weighted", cand_offsets: torch.Tensor | None = None,
                 his_bias: torch.Tensor | None = None, return_user: bool = False, validate: bool = True):
    """``score`` with the news rows gathered by id from a device news-embedding table.

    news_table [n_news, d] (the news encoder's output for every news item, float32 or bfloat16),
    his_ids [B, L] int, his_mask [B, L] bool, cand_ids [B, C] (dense) or [N] with cand_offsets [B+1].
    The reference re-encodes every sample's news (src/model/model.py:104-111 fed by
    src/reader.py:366-379); with the table computed once, the kernel DMAs the rows by id.
    Returns what ``score`` returns. ``validate`` checks ids / offsets on the device first.
    """
    st = _lib.SCORE_TYPES.get(score_type)
    if st is None or st == _lib.SCORE_NONE:
        raise ValueError("Invalid method of aggregating matching score")  # model.py:136
    _require_device(news_table, his_ids, his_mask, cand_ids, context_codes, w_target, cand_offsets, his_bias)
    if not isinstance(w_poly, PackedWeights):
        _require_device(w_poly)
    tdt = news_table.dtype
    dt = _dtype_code(tdt)
    table = _contig(news_table)
    n_news, d = table.shape
    B, L = his_ids.shape
    hid = _contig(his_ids, torch.int32)
    if isinstance(w_poly, PackedWeights):
        Dc, K = w_poly.Dc, w_poly.K
    else:
        K, Dc = context_codes.shape
    fused = _fused_or_wide(dt, L, d, Dc, K)
    if st == _lib.SCORE_WEIGHTED and not isinstance(w_poly, PackedWeights) and w_target is None:
        raise ValueError("score_type='weighted' needs w_target (target_aware_attn.linear.weight)")
    pw = _as_packed(w_poly, context_codes, w_target if st == _lib.SCORE_WEIGHTED else None, tdt)
    fused = fused and pw.buf is not None
    if pw.d != d:
        raise ValueError(f"packed weights are for d={pw.d}, the news table has d={d}")
    if pw.Dc == 0:
        raise ValueError("packed weights hold no PolyAttention part (pack_target_weights output)")
    if st == _lib.SCORE_WEIGHTED and not pw.has_target:
        raise ValueError("score_type='weighted' needs weights packed with w_target")
    mask, his_bias = _check_mask_bias(his_mask, his_bias, B, L)
    if cand_offsets is None:
        if cand_ids.dim() != 2 or cand_ids.shape[0] != B:
            raise ValueError(f"dense cand_ids must be [{B},C]")
        C = cand_ids.shape[1]
        cid = _contig(cand_ids, torch.int32)
        scores = torch.empty((B, C), device=table.device, dtype=torch.float32)
        offs = None
    else:
        cid = _contig(cand_ids.reshape(-1), torch.int32)
        offs = _contig(cand_offsets, torch.int32)
        if validate:
            check_offsets(offs, B, cid.numel())
        C = 0
        scores = torch.empty((cid.numel(),), device=table.device, dtype=torch.float32)
    if validate:
        _check_ids(hid, n_news, "his_ids")
        _check_ids(cid, n_news, "cand_ids")
    if not fused:
        return _score_wide(pw, st, table, hid, mask, his_bias, table, cid, offs, B, C, scores.numel(), return_user)
    mui = torch.empty((B, K, d), device=table.device, dtype=torch.float32) if return_user else None
    with torch.cuda.device(table.device):
        rc = _lib.lib().miner_score_gather(_stream(table.device), _kernel_dtype(dt), st, _ptr(table), n_news, _ptr(hid), _ptr(mask),
                                           _ptr(his_bias), _ptr(cid), _ptr(offs), _ptr(pw.buf), B, L, C, d, Dc, K,
                                           _ptr(scores), _ptr(mui))
    _lib.check(rc, "miner_score_gather")
    return (scores, mui) if return_user else scores


def poly_attention(history: torch.Tensor, his_mask: torch.Tensor, w_poly, context_codes: torch.Tensor | None = None,
                   his_bias: torch.Tensor | None = None) -> torch.Tensor:
    """PolyAttention.forward (src/model/model.py:159-185) -> mui [B,K,d] fp32."""
    _require_device(history, his_mask, context_codes, his_bias)
    tdt = history.dtype
    dt = _dtype_code(tdt)
    history = _contig(history)
    pw = _as_packed(w_poly, context_codes, None, tdt)
    if history.dim() != 3:
        raise ValueError(f"history must be [B,L,d], got {tuple(history.shape)}")
    B, L, d = history.shape
    Dc, K = pw.Dc, pw.K
    if pw.d != d or Dc == 0:
        raise ValueError(f"packed weights are for d={pw.d} (Dc={Dc}), history has d={d}")
    mask, his_bias = _check_mask_bias(his_mask, his_bias, B, L)
    if not _fused_or_wide(dt, L, d, Dc, K) or pw.buf is None:
        from . import corpus
        res = corpus.encode_users(history, mask.view(torch.bool), _wide_encoder(pw), his_bias=his_bias,
                                  with_proj=False, return_f32=tdt != torch.float32)
        return res[0] if tdt == torch.float32 else res[2]
    mui = torch.empty((B, K, d), device=history.device, dtype=torch.float32)
    with torch.cuda.device(history.device):
        rc = _lib.lib().miner_score(_stream(history.device), _kernel_dtype(dt), _lib.SCORE_NONE, _ptr(history), _ptr(mask),
                                    _ptr(his_bias), None, None, _ptr(pw.buf), B, L, 0, d, Dc, K, None, _ptr(mui))
    _lib.check(rc, "miner_score(PolyAttention)")
    return mui


def target_aware(query: torch.Tensor, key: torch.Tensor, value: torch.Tensor, w_target,
                 cand_offsets: torch.Tensor | None = None, validate_offsets: bool = True) -> torch.Tensor:
    """TargetAwareAttention.forward (src/model/model.py:200-216).

    query [B,K,d], key [B,C,d] (or [N,d] + cand_offsets), value [B,C,K] (or [N,K]) -> [B,C] / [N].
    ``w_target`` is the [d,d] weight or a PackedWeights that holds it.
    """
    _require_device(query, key, value, cand_offsets)
    tdt = query.dtype
    dt = _dtype_code(tdt)
    query = _contig(query)
    key = _contig(key, tdt)
    value = _contig(value, torch.float32)
    if query.dim() != 3:
        raise ValueError(f"query must be [B,K,d], got {tuple(query.shape)}")
    B, K, d = query.shape
    if isinstance(w_target, PackedWeights):
        pw = w_target
        if not pw.has_target or pw.dtype != tdt:
            raise ValueError("packed weights must hold w_target in the query dtype")
        if pw.d != d:
            raise ValueError(f"packed w_target is for d={pw.d}, query has d={d}")
        if pw.K and pw.K != K:
            raise ValueError(f"packed weights are for K={pw.K}, query has K={K}")
    else:
        _require_device(w_target)
        if tuple(w_target.shape) != (d, d):
            raise ValueError(f"w_target must be [{d},{d}], got {tuple(w_target.shape)}")
        pw = pack_target_weights(w_target, dtype=tdt)          # TAA alone needs only W2
    if cand_offsets is None:
        C = key.shape[1]
        if tuple(key.shape) != (B, C, d) or tuple(value.shape) != (B, C, K):
            raise ValueError("key must be [B,C,d] and value [B,C,K]")
        out = torch.empty((B, C), device=query.device, dtype=torch.float32)
        offs = None
    else:
        if key.dim() != 2 or key.shape[1] != d or tuple(value.shape) != (key.shape[0], K):
            raise ValueError("ragged key must be [N,d] and value [N,K]")
        offs = _contig(cand_offsets, torch.int32)
        if validate_offsets:
            check_offsets(offs, B, key.shape[0])
        C = 0
        out = torch.empty((key.shape[0],), device=query.device, dtype=torch.float32)
    if K > FUSED_MAX_K:
        # wide path: proj = gelu(query · W2ᵀ) (model.py:212), then the weighted aggregation of the given
        # value (model.py:213-214) — include/miner_wide.h
        if K > WIDE_MAX_K or d % 64:
            raise ValueError(f"TargetAwareAttention with K={K} d={d}: K <= {WIDE_MAX_K} and d % 64 == 0 past K = "
                             f"{FUSED_MAX_K}")
        w2 = pw.src[2] if pw.src is not None else None
        if w2 is None:
            raise ValueError("these packed weights carry no w_target source tensor for K > 32")
        proj = torch.empty_like(query)
        with torch.cuda.device(query.device):
            rc = _lib.lib().miner_wide_proj(_stream(query.device), dt, _ptr(query), _ptr(_contig(w2, tdt)), B * K, d,
                                            _ptr(proj))
            _lib.check(rc, "miner_wide_proj")
            rc = _lib.lib().miner_score_wide(_stream(query.device), dt, _lib.SCORE_WEIGHTED, None, _ptr(proj),
                                             _ptr(key), None, 0, _ptr(offs), _ptr(value), B, C, d, K, _ptr(out))
        _lib.check(rc, "miner_score_wide")
        return out
    with torch.cuda.device(query.device):
        rc = _lib.lib().miner_target_aware(_stream(query.device), _kernel_dtype(dt), _ptr(query), _ptr(key), _ptr(value), _ptr(offs),
                                           _ptr(pw.buf), pw.Dc, B, C, d, K, _ptr(out))
    _lib.check(rc, "miner_target_aware")
    return out
