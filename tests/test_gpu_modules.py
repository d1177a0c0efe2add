"""The drop-in nn.Modules at the north_star boundary (miner_amd.model: Miner.forward / Miner.score,
PolyAttention.forward, TargetAwareAttention.forward — src/model/model.py:61-138, :159-185,
:200-216) against the reference's own outputs in the golden fixtures — needs an MI355X.

Weights enter through ``load_state_dict`` with the reference's parameter names; ``Miner.forward``
runs with the stub news encoder of make_golden.py (token 0 of a title is a news-table row).
Tolerances as tests/test_gpu_parity.py: fp32 |x - ref| <= 1e-5·|ref| + 1e-5·rms(ref); bf16 mode
against the oracle on the same bf16-rounded inputs and weights, 7e-3·|ref| + 2e-2·rms(ref).
"""
import numpy as np
import pytest
import torch
import torch.nn as nn

from oracle import miner_oracle as orc
from tests.conftest import golden_names, load_golden

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


class StubNewsEncoder(nn.Module):
    """Stands in for NewsEncoder (news_encoder.py:60-106) as make_golden.py does."""

    def __init__(self, table):
        super().__init__()
        self.embed_dim = table.shape[1]
        self.register_buffer("table", table)

    def forward(self, title_encoding, title_attn_mask, sapo_encoding=None, sapo_attn_mask=None):
        return self.table[title_encoding[:, 0]]


def _model(g, precision="fp32"):
    from miner_amd import model
    table = torch.from_numpy(g["table"])
    use_bias = bool(g["use_bias"])
    kw = {}
    if use_bias:
        ce = torch.from_numpy(g["category_embedding"])
        kw = dict(num_category=ce.shape[0], category_embed_dim=ce.shape[1], category_pad_token_id=0)
    m = model.Miner(StubNewsEncoder(table), use_bias, g["K"], g["Dc"], g["score_type"], 0.0, **kw)
    sd = {"poly_attn.linear.weight": torch.from_numpy(g["W1"]), "poly_attn.context_codes": torch.from_numpy(g["Q"])}
    if g["score_type"] == "weighted":
        sd["target_aware_attn.linear.weight"] = torch.from_numpy(g["W2"])
    if use_bias:
        sd["category_embedding.weight"] = torch.from_numpy(g["category_embedding"])
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert all(k.startswith("news_encoder.") for k in missing), missing
    return m.to(DEV).eval().set_precision(precision)


def _tokens(ids, C_or_L):
    """[B, n] news rows -> title tokens [B, n, 4] (token 0 = row) and an all-ones mask."""
    t = torch.zeros(ids.shape + (4,), dtype=torch.int64)
    t[..., 0] = torch.from_numpy(ids)
    return t.to(DEV), torch.ones_like(t).to(DEV)


@pytest.mark.parametrize("name", golden_names())
def test_miner_forward_matches_reference(name):
    g = load_golden(name)
    m = _model(g)
    title, tmask = _tokens(g["cand_ids"], g["C"])
    his_title, hmask = _tokens(g["his_ids"], g["L"])
    kw = {}
    if g["use_bias"]:
        kw = dict(category=torch.from_numpy(g["cand_cat"]).to(DEV), his_category=torch.from_numpy(g["his_cat"]).to(DEV))
    with torch.no_grad():
        mui, scores = m(title=title, title_mask=tmask, his_title=his_title, his_title_mask=hmask,
                        his_mask=torch.from_numpy(g["his_mask"]).to(DEV), sapo=title, sapo_mask=tmask,
                        his_sapo=his_title, his_sapo_mask=hmask, **kw)
    torch.cuda.synchronize()
    ok, worst = orc.parity_ok(scores.cpu().numpy(), g["scores"])
    assert ok, f"{name}: Miner.forward scores off by {worst:.2f}x the tolerance"
    ok, worst = orc.parity_ok(mui.cpu().numpy(), g["mui"])
    assert ok, f"{name}: Miner.forward mui off by {worst:.2f}x the tolerance"


@pytest.mark.parametrize("name", golden_names())
def test_miner_score_matches_reference(name):
    g = load_golden(name)
    m = _model(g)
    bias = torch.from_numpy(g["bias"]).to(DEV) if g["use_bias"] else None
    with torch.no_grad():
        mui, scores = m.score(torch.from_numpy(g["E"]).to(DEV), torch.from_numpy(g["his_mask"]).to(DEV),
                              torch.from_numpy(g["cand"]).to(DEV), category_bias=bias)
    torch.cuda.synchronize()
    assert orc.parity_ok(scores.cpu().numpy(), g["scores"])[0]
    assert orc.parity_ok(mui.cpu().numpy(), g["mui"])[0]


@pytest.mark.parametrize("name", golden_names())
def test_poly_attention_module(name):
    g = load_golden(name)
    m = _model(g)
    bias = torch.from_numpy(g["bias"]).to(DEV) if g["use_bias"] else None
    with torch.no_grad():
        mui = m.poly_attn(torch.from_numpy(g["E"]).to(DEV), torch.from_numpy(g["his_mask"]).to(DEV), bias=bias)
    torch.cuda.synchronize()
    ok, worst = orc.parity_ok(mui.cpu().numpy(), g["mui"])
    assert ok, f"{name}: PolyAttention.forward off by {worst:.2f}x the tolerance"


@pytest.mark.parametrize("name", [n for n in golden_names() if load_golden(n)["score_type"] == "weighted"])
def test_target_aware_module(name):
    """TargetAwareAttention.forward with the reference's mui as query and Cand·muiᵀ as value; the
    module packs W2 alone (miner_pack_target_weights) — no dummy PolyAttention block."""
    g = load_golden(name)
    m = _model(g)
    mui, cand = torch.from_numpy(g["mui"]), torch.from_numpy(g["cand"])
    value = torch.matmul(cand, mui.permute(0, 2, 1))
    ref = orc.target_aware_torch(mui, cand, value, torch.from_numpy(g["W2"]))
    with torch.no_grad():
        out = m.target_aware_attn(mui.to(DEV), cand.to(DEV), value.to(DEV))
    torch.cuda.synchronize()
    ok, worst = orc.parity_ok(out.cpu().numpy(), ref.numpy())
    assert ok, f"{name}: TargetAwareAttention.forward off by {worst:.2f}x the tolerance"
    # the last stage of the full path: the reference's scores from its own mui
    ok, worst = orc.parity_ok(out.cpu().numpy(), g["scores"])
    assert ok, f"{name}: TAA(reference mui) vs reference scores off by {worst:.2f}x"
    pk = m.target_aware_attn._pc.get(torch.float32, w_target=m.target_aware_attn.linear.weight)
    assert pk.Dc == 0 and pk.has_target


def _bf16(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(torch.bfloat16).to(torch.float32)


@pytest.mark.parametrize("name", golden_names())
def test_miner_score_bf16(name):
    g = load_golden(name)
    m = _model(g, "bf16")
    bias = torch.from_numpy(g["bias"]) if g["use_bias"] else None
    E, Cd = _bf16(g["E"]), _bf16(g["cand"])
    W1, Q = _bf16(g["W1"]), _bf16(g["Q"])
    W2 = _bf16(g["W2"]) if g["score_type"] == "weighted" else None
    rmui, rs = orc.score_torch(E, torch.from_numpy(g["his_mask"]), Cd, W1, Q, W2, score_type=g["score_type"],
                               bias=bias)
    with torch.no_grad():
        mui, scores = m.score(E.to(DEV), torch.from_numpy(g["his_mask"]).to(DEV), Cd.to(DEV),
                              category_bias=None if bias is None else bias.to(DEV))
    torch.cuda.synchronize()
    ok, worst = orc.parity_ok(scores.cpu().numpy(), rs.numpy(), rtol=7e-3, rms_floor=2e-2)
    assert ok, f"{name}: bf16 scores off by {worst:.2f}x the bf16 tolerance"


def test_repack_after_parameter_update():
    g = load_golden("cfg1_demo")
    m = _model(g)
    E, M, Cd = (torch.from_numpy(g[k]).to(DEV) for k in ("E", "his_mask", "cand"))
    with torch.no_grad():
        s0 = m.score(E, M, Cd, return_user=False).clone()
        m.target_aware_attn.linear.weight.mul_(0.5)
        s1 = m.score(E, M, Cd, return_user=False)
        m.target_aware_attn.linear.weight.mul_(2.0)
        s2 = m.score(E, M, Cd, return_user=False)
    torch.cuda.synchronize()
    assert not torch.equal(s0, s1)
    assert torch.equal(s0, s2)
