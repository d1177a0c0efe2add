"""FastFormer user encoder on MI355X (BASELINE config 4), backed by the fused
HIP kernel of libminer_hip.so (include/miner_fastformer.h).

Ops (torch-facing wrappers of the C ABI; device tensors only, enqueued on the current stream):

* ``flatten_params(state_dict)``  FastformerEncoder.state_dict() -> the flat fp32 blob of the ABI;
* ``pack(params, dtype)``         -> ``FFPacked`` (the kernel's tiled layout, once per model);
* ``score(...)`` / ``score_gather(...)``  user vectors and scores = candidates · user.

Drop-in modules with the reference's class names, constructor arguments and parameter names (so a
reference ``fast_attn`` / ``FastFormer`` state_dict loads as-is):

* ``FastformerEncoder``  src/model/model.py:482-545 (+ FastformerLayer :469-480, FastAttention
  :458-467, FastSelfAttention :373-455, AttentionPooling :345-371, HF BertSelfOutput /
  BertIntermediate / BertOutput);
* ``FastFormer``         src/model/model.py:223-341 (``forward`` returns matching_scores [B,C]).

No CPU fallback: calling them with CPU tensors raises.
"""
from __future__ import annotations

import dataclasses
from typing import Dict, Optional, Union

import torch
import torch.nn as nn
from torch import Tensor

from . import _lib
from .ops import _contig, _dtype_code, _ptr, _require_device, _stream, check_offsets

HIDDEN, HEADS, MAX_L, LAYERS = 256, 16, 64, 2
_PREC = {"fp32": torch.float32, "bf16": torch.bfloat16}


def _layer_params(i: int):
    p = f"encoders.{i}."
    s = p + "attention.self."
    H = HIDDEN
    return [(s + "query.weight", (H, H)), (s + "query.bias", (H,)),
            (s + "query_att.weight", (HEADS, H)), (s + "query_att.bias", (HEADS,)),
            (s + "key.weight", (H, H)), (s + "key.bias", (H,)),
            (s + "key_att.weight", (HEADS, H)), (s + "key_att.bias", (HEADS,)),
            (s + "transform.weight", (H, H)), (s + "transform.bias", (H,)),
            (p + "attention.output.dense.weight", (H, H)), (p + "attention.output.dense.bias", (H,)),
            (p + "attention.output.LayerNorm.weight", (H,)), (p + "attention.output.LayerNorm.bias", (H,)),
            (p + "intermediate.dense.weight", (H, H)), (p + "intermediate.dense.bias", (H,)),
            (p + "output.dense.weight", (H, H)), (p + "output.dense.bias", (H,)),
            (p + "output.LayerNorm.weight", (H,)), (p + "output.LayerNorm.bias", (H,))]


# FastformerEncoder.state_dict() order (model.py:482-495 construction order)
PARAMS = ([e for i in range(LAYERS) for e in _layer_params(i)]
          + [("position_embeddings.weight", (HIDDEN, HIDDEN)), ("LayerNorm.weight", (HIDDEN,)),
             ("LayerNorm.bias", (HIDDEN,)), ("poolers.0.att_fc1.weight", (HIDDEN, HIDDEN)),
             ("poolers.0.att_fc1.bias", (HIDDEN,)), ("poolers.0.att_fc2.weight", (1, HIDDEN)),
             ("poolers.0.att_fc2.bias", (1,))])
PARAM_FLOATS = sum(int(torch.Size(s).numel()) for _, s in PARAMS)
assert PARAM_FLOATS == 940097


def flatten_params(state_dict: Dict[str, Tensor], device=None) -> Tensor:
    """FastformerEncoder.state_dict() (keys as the reference's, with or without a ``fast_attn.``
    prefix) -> the flat fp32 blob [940097] of miner_fastformer_pack."""
    parts = []
    for name, shape in PARAMS:
        t = state_dict.get(name)
        if t is None:
            t = state_dict.get("fast_attn." + name)
        if t is None:
            raise KeyError(f"FastFormer parameter {name!r} missing")
        if tuple(t.shape) != shape:
            raise ValueError(f"{name}: expected shape {shape}, got {tuple(t.shape)}")
        parts.append(t.detach().reshape(-1).to(device or t.device, torch.float32))
    return torch.cat(parts).contiguous()


@dataclasses.dataclass
class FFPacked:
    """miner_fastformer_pack() output."""
    buf: Tensor
    dtype: torch.dtype


def pack(params: Union[Tensor, Dict[str, Tensor]], dtype: torch.dtype = torch.float32) -> FFPacked:
    """Pack the FastFormer user encoder's parameters (flat blob or state_dict, on the GPU)."""
    if not isinstance(params, Tensor):
        params = flatten_params(params)
    _require_device(params)
    if params.dtype != torch.float32 or params.numel() != PARAM_FLOATS:
        raise ValueError(f"params must be a float32 blob of {PARAM_FLOATS} values")
    dt = _dtype_code(dtype)
    params = params.contiguous()
    nbytes = _lib.lib().miner_fastformer_packed_bytes(dt)
    buf = torch.empty(nbytes, dtype=torch.uint8, device=params.device)
    with torch.cuda.device(params.device):
        rc = _lib.lib().miner_fastformer_pack(_stream(params.device), dt, _ptr(params), _ptr(buf))
    _lib.check(rc, "miner_fastformer_pack")
    return FFPacked(buf, dtype)


def _offsets(cand_offsets, B, N, validate):
    if cand_offsets is None:
        return None
    cand_offsets = _contig(cand_offsets, torch.int32)
    if validate:
        check_offsets(cand_offsets, B, N)
    return cand_offsets


def _check_ids(ids: Tensor, n: int, what: str) -> None:
    if ids.numel() and (int(ids.min()) < 0 or int(ids.max()) >= n):
        raise IndexError(f"{what} out of range [0, {n})")


def score(history: Tensor, his_mask: Tensor, candidates: Optional[Tensor], packed: FFPacked, *,
          cand_offsets: Optional[Tensor] = None, return_user: bool = False, validate: bool = True):
    """FastformerEncoder(history, his_mask) -> user [B,256]; scores = candidates · user
    (model.py:318-322).

    history [B,L,256], his_mask [B,L] bool, candidates [B,C,256] (dense) or [N,256] with
    cand_offsets [B+1] int32, or None (user vectors only). Returns scores (fp32 [B,C] / [N]),
    (scores, user) with return_user, or user alone when candidates is None.
    """
    _require_device(history, his_mask, candidates, cand_offsets)
    dt = _dtype_code(packed.dtype)
    if history.dim() != 3 or history.shape[2] != HIDDEN:
        raise ValueError(f"history must be [B,L,{HIDDEN}], got {tuple(history.shape)}")
    B, L, _ = history.shape
    if not 1 <= L <= MAX_L:
        raise ValueError(f"history length {L} outside [1, {MAX_L}]")
    hist = _contig(history, packed.dtype)
    mask = _contig(his_mask, torch.bool).view(torch.uint8)
    if tuple(mask.shape) != (B, L):
        raise ValueError(f"his_mask must be [{B},{L}]")
    dev = hist.device
    user = torch.empty(B, HIDDEN, dtype=torch.float32, device=dev) if (return_user or candidates is None) else None
    cand = offs = scores = None
    C = 0
    if candidates is not None:
        cand = _contig(candidates, packed.dtype)
        if cand_offsets is None:
            if cand.dim() != 3 or cand.shape[0] != B or cand.shape[2] != HIDDEN:
                raise ValueError(f"candidates must be [{B},C,{HIDDEN}] without cand_offsets")
            C = cand.shape[1]
            scores = torch.empty(B, C, dtype=torch.float32, device=dev)
        else:
            if cand.dim() != 2 or cand.shape[1] != HIDDEN:
                raise ValueError(f"candidates must be [N,{HIDDEN}] with cand_offsets")
            offs = _offsets(cand_offsets, B, cand.shape[0], validate)
            scores = torch.empty(cand.shape[0], dtype=torch.float32, device=dev)
    with torch.cuda.device(dev):
        rc = _lib.lib().miner_fastformer_score(_stream(dev), dt, _ptr(hist), _ptr(mask), _ptr(cand), _ptr(offs),
                                               _ptr(packed.buf), B, L, C, _ptr(scores), _ptr(user))
    _lib.check(rc, "miner_fastformer_score")
    if candidates is None:
        return user
    return (scores, user) if return_user else scores


def score_gather(news_table: Tensor, his_ids: Tensor, his_mask: Tensor, cand_ids: Optional[Tensor],
                 packed: FFPacked, *, cand_offsets: Optional[Tensor] = None, return_user: bool = False,
                 validate: bool = True):
    """``score`` with history / candidate rows taken by id from news_table [n_news,256]
    (his_ids [B,L], cand_ids [B,C] dense or [N] with cand_offsets)."""
    _require_device(news_table, his_ids, his_mask, cand_ids, cand_offsets)
    dt = _dtype_code(packed.dtype)
    table = _contig(news_table, packed.dtype)
    if table.dim() != 2 or table.shape[1] != HIDDEN:
        raise ValueError(f"news_table must be [n_news,{HIDDEN}]")
    n_news = table.shape[0]
    B, L = his_ids.shape
    if not 1 <= L <= MAX_L:
        raise ValueError(f"history length {L} outside [1, {MAX_L}]")
    hid = _contig(his_ids, torch.int32)
    mask = _contig(his_mask, torch.bool).view(torch.uint8)
    if validate:
        _check_ids(hid, n_news, "his_ids")
    dev = table.device
    user = torch.empty(B, HIDDEN, dtype=torch.float32, device=dev) if (return_user or cand_ids is None) else None
    cid = offs = scores = None
    C = 0
    if cand_ids is not None:
        cid = _contig(cand_ids, torch.int32)
        if validate:
            _check_ids(cid, n_news, "cand_ids")
        if cand_offsets is None:
            if cid.dim() != 2 or cid.shape[0] != B:
                raise ValueError(f"cand_ids must be [{B},C] without cand_offsets")
            C = cid.shape[1]
            scores = torch.empty(B, C, dtype=torch.float32, device=dev)
        else:
            offs = _offsets(cand_offsets, B, cid.numel(), validate)
            scores = torch.empty(cid.numel(), dtype=torch.float32, device=dev)
    with torch.cuda.device(dev):
        rc = _lib.lib().miner_fastformer_score_gather(_stream(dev), dt, _ptr(table), n_news, _ptr(hid), _ptr(mask),
                                                      _ptr(cid), _ptr(offs), _ptr(packed.buf), B, L, C,
                                                      _ptr(scores), _ptr(user))
    _lib.check(rc, "miner_fastformer_score_gather")
    if cand_ids is None:
        return user
    return (scores, user) if return_user else scores


# ---------------------------------------------------------------------------------------------
# drop-in modules (parameter names of the reference)
# ---------------------------------------------------------------------------------------------
class _SelfAttention(nn.Module):          # FastSelfAttention (model.py:373-407)
    def __init__(self):
        super().__init__()
        self.query = nn.Linear(HIDDEN, HIDDEN)
        self.query_att = nn.Linear(HIDDEN, HEADS)
        self.key = nn.Linear(HIDDEN, HIDDEN)
        self.key_att = nn.Linear(HIDDEN, HEADS)
        self.transform = nn.Linear(HIDDEN, HIDDEN)


class _DenseLN(nn.Module):                # BertSelfOutput / BertOutput
    def __init__(self, eps):
        super().__init__()
        self.dense = nn.Linear(HIDDEN, HIDDEN)
        self.LayerNorm = nn.LayerNorm(HIDDEN, eps=eps)


class _Dense(nn.Module):                  # BertIntermediate
    def __init__(self):
        super().__init__()
        self.dense = nn.Linear(HIDDEN, HIDDEN)


class _Attention(nn.Module):              # FastAttention (model.py:458-467)
    def __init__(self, eps):
        super().__init__()
        self.self = _SelfAttention()
        self.output = _DenseLN(eps)


class _Layer(nn.Module):                  # FastformerLayer (model.py:469-480)
    def __init__(self, eps):
        super().__init__()
        self.attention = _Attention(eps)
        self.intermediate = _Dense()
        self.output = _DenseLN(eps)


class _Pooling(nn.Module):                # AttentionPooling (model.py:345-359)
    def __init__(self):
        super().__init__()
        self.att_fc1 = nn.Linear(HIDDEN, HIDDEN)
        self.att_fc2 = nn.Linear(HIDDEN, 1)


class _PackCache:
    """pack() output per (dtype, device), re-packed when a parameter changes (version counters
    and storage pointers)."""

    def __init__(self):
        self._c = {}

    def get(self, module: nn.Module, dtype: torch.dtype) -> FFPacked:
        params = list(module.parameters())
        key = (dtype, params[0].device)
        stamp = tuple((t._version, t.data_ptr()) for t in params)
        hit = self._c.get(key)
        if hit is not None and hit[0] == stamp:
            return hit[1]
        with torch.no_grad():
            packed = pack(flatten_params(module.state_dict()), dtype)
        self._c[key] = (stamp, packed)
        return packed


class FastformerEncoder(nn.Module):
    """model.py:482-545 with the reference's BertConfig (model.py:245-266): hidden 256, 16 heads,
    intermediate 256, 2 layers, max positions 256, layer_norm_eps 1e-12, one weight pooler."""

    def __init__(self, config=None, pooler_count: int = 1, precision: str = "fp32"):
        super().__init__()
        get = (lambda k, d: getattr(config, k, d)) if config is not None else (lambda k, d: d)
        if (get("hidden_size", HIDDEN), get("num_attention_heads", HEADS), get("intermediate_size", HIDDEN),
                get("num_hidden_layers", LAYERS)) != (HIDDEN, HEADS, HIDDEN, LAYERS) or pooler_count != 1:
            raise ValueError("the fused kernel implements the reference's FastFormer config only "
                             "(hidden 256, 16 heads, intermediate 256, 2 layers, one pooler)")
        eps = get("layer_norm_eps", 1e-12)
        if eps != 1e-12:
            raise ValueError("layer_norm_eps must be 1e-12 (model.py:255)")
        self.encoders = nn.ModuleList([_Layer(eps) for _ in range(LAYERS)])
        self.position_embeddings = nn.Embedding(get("max_position_embeddings", 256), HIDDEN)
        self.LayerNorm = nn.LayerNorm(HIDDEN, eps=eps)
        self.poolers = nn.ModuleList([_Pooling()])
        self.apply(self._init_weights)
        self.precision = precision
        self._pc = _PackCache()

    def _init_weights(self, module):      # model.py:497-509 (initializer_range 0.02)
        if isinstance(module, (nn.Linear, nn.Embedding)):
            module.weight.data.normal_(mean=0.0, std=0.02)
        elif isinstance(module, nn.LayerNorm):
            module.bias.data.zero_()
            module.weight.data.fill_(1.0)
        if isinstance(module, nn.Linear) and module.bias is not None:
            module.bias.data.zero_()

    def packed(self) -> FFPacked:
        return self._pc.get(self, _PREC[self.precision])

    def forward(self, input_embs: Tensor, attention_mask: Tensor, pooler_index: int = 0) -> Tensor:
        """model.py:511-545: [B,L,256] history embeddings, [B,L] mask -> user vectors [B,256] fp32."""
        if pooler_index != 0:
            raise ValueError("one pooler")
        packed = self.packed()
        return score(input_embs.to(packed.dtype), attention_mask, None, packed)


class FastFormer(nn.Module):
    """FastFormer user-encoder model (model.py:223-341), scoring path on MI355X."""

    def __init__(self, news_encoder, score_type: str, dropout: float, precision: str = "fp32"):
        super().__init__()
        self.news_encoder = news_encoder
        self.news_embed_dim = self.news_encoder.embed_dim
        self.fast_attn = FastformerEncoder(precision=precision)
        self.score_type = score_type
        self.dropout = nn.Dropout(dropout)
        self.set_precision(precision)

    def set_precision(self, precision: str) -> "FastFormer":
        if precision not in _PREC:
            raise ValueError(f"precision must be one of {sorted(_PREC)}")
        self.precision = precision
        self.fast_attn.precision = precision
        return self

    def score(self, history_repr: Tensor, his_mask: Tensor, candidate_repr: Tensor, *,
              cand_offsets: Tensor = None, return_user: bool = False):
        """Scoring after the news encoder (model.py:318-322): matching_scores [B,C] fp32
        (or [N] with cand_offsets), plus the user vectors with return_user."""
        packed = self.fast_attn.packed()
        return score(history_repr.to(packed.dtype), his_mask, candidate_repr.to(packed.dtype), packed,
                     cand_offsets=cand_offsets, return_user=return_user)

    def forward(self, title: Tensor, title_mask: Tensor, his_title: Tensor, his_title_mask: Tensor,
                his_mask: Tensor, sapo: Union[Tensor, None] = None, sapo_mask: Union[Tensor, None] = None,
                his_sapo: Union[Tensor, None] = None, his_sapo_mask: Union[Tensor, None] = None,
                category: Union[Tensor, None] = None, his_category: Union[Tensor, None] = None):
        """Same contract as the reference forward (model.py:274-341): matching_scores [B,C]."""
        batch_size, num_candidates, his_length = title.shape[0], title.shape[1], his_title.shape[1]
        candidate_repr = self.news_encoder(title_encoding=title.view(batch_size * num_candidates, -1),
                                           title_attn_mask=title_mask.view(batch_size * num_candidates, -1),
                                           sapo_encoding=sapo.view(batch_size * num_candidates, -1),
                                           sapo_attn_mask=sapo_mask.view(batch_size * num_candidates, -1))
        candidate_repr = candidate_repr.view(batch_size, num_candidates, -1)
        history_repr = self.news_encoder(title_encoding=his_title.view(batch_size * his_length, -1),
                                         title_attn_mask=his_title_mask.view(batch_size * his_length, -1),
                                         sapo_encoding=his_sapo.view(batch_size * his_length, -1),
                                         sapo_attn_mask=his_sapo_mask.view(batch_size * his_length, -1))
        history_repr = history_repr.view(batch_size, his_length, -1)
        return self.score(history_repr, his_mask, candidate_repr)
