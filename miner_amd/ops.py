"""torch-facing wrappers of the C ABI (include/miner_score.h).

PyTorch is plumbing here: it owns device memory and the current HIP stream; the arithmetic runs in
libminer_hip.so. Every call enqueues on ``torch.cuda.current_stream()`` and returns without
synchronising. Inputs must be device tensors: there is no CPU path.
"""
from __future__ import annotations

import torch

from . import _lib

_DTYPES = {torch.float32: _lib.DTYPE_F32, torch.bfloat16: _lib.DTYPE_BF16}


def _ptr(t):
    return None if t is None else ctypes_ptr(t)


def ctypes_ptr(t: torch.Tensor) -> int:
    return t.data_ptr()


def _require_device(*ts):
    for t in ts:
        if t is not None and t.device.type != "cuda":
            raise RuntimeError("miner_amd ops run on the GPU only (got a tensor on %s); the scoring "
                               "path has no CPU fallback" % t.device)


def _contig(t, dtype=None):
    if t is None:
        return None
    if dtype is not None and t.dtype != dtype:
        t = t.to(dtype)
    return t.contiguous()


def _dtype_code(t: torch.Tensor) -> int:
    try:
        return _DTYPES[t.dtype]
    except KeyError:
        raise TypeError(f"unsupported dtype {t.dtype}: use float32 (parity) or bfloat16 (throughput)")


def check_offsets(cand_offsets: torch.Tensor, B: int, N: int) -> None:
    """Host-side validation of CSR candidate offsets (one device->host copy)."""
    o = cand_offsets.detach().to("cpu", torch.int64)
    if o.numel() != B + 1 or int(o[0]) != 0 or int(o[-1]) != N or bool((o[1:] < o[:-1]).any()):
        raise ValueError(f"cand_offsets must be a non-decreasing int32 [B+1] array from 0 to {N}")


def score(history: torch.Tensor, his_mask: torch.Tensor, candidates: torch.Tensor,
          w_poly: torch.Tensor, context_codes: torch.Tensor, w_target: torch.Tensor | None = None, *,
          score_type: str = "weighted", cand_offsets: torch.Tensor | None = None,
          his_bias: torch.Tensor | None = None, return_user: bool = False,
          validate_offsets: bool = True):
    """Fused PolyAttention -> Cand·muiᵀ -> aggregation (src/model/model.py:113-138).

    history [B,L,d], his_mask [B,L] bool, candidates [B,C,d] (dense) or [N,d] with
    cand_offsets [B+1] int32 (ragged). Weights in the activation dtype (float32 or bfloat16).
    Returns scores ([B,C] dense / [N] ragged, fp32) and, if return_user, mui [B,K,d] fp32.
    """
    st = _lib.SCORE_TYPES.get(score_type)
    if st is None or st == _lib.SCORE_NONE:
        raise ValueError("Invalid method of aggregating matching score")  # model.py:136
    _require_device(history, his_mask, candidates, w_poly, context_codes, w_target, cand_offsets, his_bias)
    dt = _dtype_code(history)
    tdt = history.dtype
    history = _contig(history)
    candidates = _contig(candidates, tdt)
    w_poly = _contig(w_poly, tdt)
    context_codes = _contig(context_codes, tdt)
    w_target = _contig(w_target, tdt) if st == _lib.SCORE_WEIGHTED else None
    if st == _lib.SCORE_WEIGHTED and w_target is None:
        raise ValueError("score_type='weighted' needs w_target (target_aware_attn.linear.weight)")
    B, L, d = history.shape
    K, Dc = context_codes.shape
    if tuple(w_poly.shape) != (Dc, d):
        raise ValueError(f"w_poly must be [{Dc},{d}], got {tuple(w_poly.shape)}")
    if w_target is not None and tuple(w_target.shape) != (d, d):
        raise ValueError(f"w_target must be [{d},{d}]")
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
    code = _lib.lib().miner_supported(dt, L, d, Dc, K)
    if code != 0:
        raise ValueError(f"shape L={L} d={d} Dc={Dc} K={K}: {_lib.lib().miner_strerror(code).decode()}")
    mui = torch.empty((B, K, d), device=history.device, dtype=torch.float32) if return_user else None
    stream = torch.cuda.current_stream(history.device).cuda_stream
    with torch.cuda.device(history.device):
        rc = _lib.lib().miner_score(stream, dt, st, _ptr(history), _ptr(mask), _ptr(his_bias),
                                    _ptr(candidates), _ptr(offs), _ptr(w_poly), _ptr(context_codes),
                                    _ptr(w_target), B, L, C, d, Dc, K, _ptr(scores), _ptr(mui))
    _lib.check(rc, "miner_score")
    return (scores, mui) if return_user else scores


def poly_attention(history: torch.Tensor, his_mask: torch.Tensor, w_poly: torch.Tensor,
                   context_codes: torch.Tensor, his_bias: torch.Tensor | None = None) -> torch.Tensor:
    """PolyAttention.forward (src/model/model.py:159-185) -> mui [B,K,d] fp32."""
    _require_device(history, his_mask, w_poly, context_codes, his_bias)
    dt = _dtype_code(history)
    tdt = history.dtype
    history = _contig(history)
    w_poly = _contig(w_poly, tdt)
    context_codes = _contig(context_codes, tdt)
    B, L, d = history.shape
    K, Dc = context_codes.shape
    mask = _contig(his_mask)
    if mask.dtype != torch.bool:
        mask = mask != 0
    mask = mask.view(torch.uint8)
    if his_bias is not None:
        his_bias = _contig(his_bias, torch.float32)
    code = _lib.lib().miner_supported(dt, L, d, Dc, K)
    if code != 0:
        raise ValueError(f"shape L={L} d={d} Dc={Dc} K={K}: {_lib.lib().miner_strerror(code).decode()}")
    mui = torch.empty((B, K, d), device=history.device, dtype=torch.float32)
    stream = torch.cuda.current_stream(history.device).cuda_stream
    with torch.cuda.device(history.device):
        rc = _lib.lib().miner_score(stream, dt, _lib.SCORE_NONE, _ptr(history), _ptr(mask), _ptr(his_bias),
                                    None, None, _ptr(w_poly), _ptr(context_codes), None,
                                    B, L, 0, d, Dc, K, None, _ptr(mui))
    _lib.check(rc, "miner_score(PolyAttention)")
    return mui


def target_aware(query: torch.Tensor, key: torch.Tensor, value: torch.Tensor, w_target: torch.Tensor,
                 cand_offsets: torch.Tensor | None = None, validate_offsets: bool = True) -> torch.Tensor:
    """TargetAwareAttention.forward (src/model/model.py:200-216).

    query [B,K,d], key [B,C,d] (or [N,d] + cand_offsets), value [B,C,K] (or [N,K]) -> [B,C] / [N].
    """
    _require_device(query, key, value, w_target, cand_offsets)
    dt = _dtype_code(query)
    tdt = query.dtype
    query = _contig(query)
    key = _contig(key, tdt)
    w_target = _contig(w_target, tdt)
    value = _contig(value, torch.float32)
    B, K, d = query.shape
    if cand_offsets is None:
        C = key.shape[1]
        if tuple(key.shape) != (B, C, d) or tuple(value.shape) != (B, C, K):
            raise ValueError("key must be [B,C,d] and value [B,C,K]")
        out = torch.empty((B, C), device=query.device, dtype=torch.float32)
        offs = None
    else:
        offs = _contig(cand_offsets, torch.int32)
        if validate_offsets:
            check_offsets(offs, B, key.shape[0])
        C = 0
        out = torch.empty((key.shape[0],), device=query.device, dtype=torch.float32)
    stream = torch.cuda.current_stream(query.device).cuda_stream
    with torch.cuda.device(query.device):
        rc = _lib.lib().miner_target_aware(stream, dt, _ptr(query), _ptr(key), _ptr(value), _ptr(offs),
                                           _ptr(w_target), B, C, d, K, _ptr(out))
    _lib.check(rc, "miner_target_aware")
    return out
