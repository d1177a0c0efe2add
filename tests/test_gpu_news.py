"""News-side precompute path (miner_news_precompute + miner_score_news) — needs an
MI355X. The kernel computes the reference's products in a different association
(mui·W2ᵀ = A·(E·W2ᵀ), logits per news row), so parity is checked against the reference's own
outputs (golden fixtures, fp32) and the oracle, never bit-for-bit against the dense kernel.

Tolerances (as tests/test_gpu_parity.py):
* fp32: |x - ref| <= 1e-5*|ref| + 1e-5*rms(ref)   (north_star 1e-5 relative + SURVEY §8c floor)
* bf16: against the oracle on the same bf16-rounded table and weights, |x - ref| <= 7e-3*|ref| +
  2e-2*rms(ref) (the kernel rounds the attention weights, proj rows and the GELU output to bf16
  MFMA operands).
"""
import os

import numpy as np
import pytest
import torch

from miner_amd import news, ops, synthetic
from oracle import miner_oracle as orc
from tests.conftest import load_golden, news_golden_names

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
BF_RTOL, BF_FLOOR = 7e-3, 2e-2


def _dev(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a)).to(DEV)
    return t if dtype is None else t.to(dtype)


def _setup(seed, B, L, d, n_news, dtype, C=40, ragged=None, Dc=200, K=32):
    g = torch.Generator(device="cpu").manual_seed(seed)
    table = (torch.randn((n_news, d), generator=g) / d ** 0.5).to(DEV, dtype)
    his_ids = torch.randint(0, n_news, (B, L), generator=g)
    lens = torch.randint(0, L + 1, (B,), generator=g)
    mask = torch.arange(L)[None, :] >= (L - lens)[:, None]
    his_ids[~mask] = 0                      # left padding = the pad news (row 0), reader.py:369
    if ragged:
        sizes = torch.randint(ragged[0], ragged[1] + 1, (B,), generator=g)
        offs = torch.zeros(B + 1, dtype=torch.int32)
        offs[1:] = torch.cumsum(sizes, 0)
        cand_ids = torch.randint(0, n_news, (int(offs[-1]),), generator=g)
    else:
        cand_ids = torch.randint(0, n_news, (B, C), generator=g)
        offs = None
    W1, Q, W2 = synthetic.init_weights(seed, d, Dc, K, device=DEV)
    return (table, his_ids.to(DEV), mask.to(DEV), cand_ids.to(DEV), None if offs is None else offs.to(DEV),
            W1.to(dtype), Q.to(dtype), W2.to(dtype))


def _oracle(table, hid, mask, cid, offs, W1, Q, W2, score_type="weighted", bias=None):
    """fp32 oracle on the (possibly bf16-rounded) inputs: (mui [B,K,d], scores dense [B,C] / ragged [N])."""
    T = table.float().cpu()
    E = T[hid.cpu().long()]
    m = mask.cpu()
    w = [x.float().cpu() if x is not None else None for x in (W1, Q, W2)]
    b = None if bias is None else bias.cpu()
    if offs is None:
        return orc.score_torch(E, m, T[cid.cpu().long()], *w, score_type, b)
    mui = orc.poly_attention_torch(E, m, w[0], w[1], b)
    o = offs.cpu().tolist()
    cids = cid.cpu().long()
    out = []
    for i in range(len(o) - 1):
        cd = T[cids[o[i]:o[i + 1]]].unsqueeze(0)
        if cd.shape[1] == 0:
            continue
        _, s = orc.score_torch(E[i:i + 1], m[i:i + 1], cd, *w, score_type, None if b is None else b[i:i + 1])
        out.append(s.reshape(-1))
    return mui, torch.cat(out) if out else torch.zeros(0)


def _ok(x, ref, dtype, what):
    x = x.detach().cpu().numpy()
    ref = ref.detach().cpu().numpy() if isinstance(ref, torch.Tensor) else ref
    if dtype == torch.float32:
        ok, worst = orc.parity_ok(x, ref)
    else:
        ok, worst = orc.parity_ok(x, ref, rtol=BF_RTOL, rms_floor=BF_FLOOR)
    assert ok, f"{what}: off by {worst:.2f}x the tolerance"
    return worst


FP32_KERNELS = ["x2", "mfma32"]     # fp16-pair operands on the fp16 MFMA (default) / fp32 MFMA (news_score32)


# ---- parity against the reference's own outputs (fp32) ------------------------------------------
@pytest.mark.parametrize("kern", FP32_KERNELS)
@pytest.mark.parametrize("name", news_golden_names())
def test_fp32_matches_reference(name, kern, monkeypatch):
    monkeypatch.setenv("MINER_NEWS_FP32", kern)
    g = load_golden(name)
    weighted = g["score_type"] == "weighted"
    W2 = _dev(g["W2"]) if "W2" in g else None
    nt = news.precompute(_dev(g["table"]), _dev(g["W1"]), _dev(g["Q"]), W2 if weighted else None, with_proj=weighted)
    bias = _dev(g["bias"], torch.float32) if g["use_bias"] else None
    scores, mui = news.score(nt, _dev(g["his_ids"]), _dev(g["his_mask"]), _dev(g["cand_ids"]),
                             score_type=g["score_type"], his_bias=bias, return_user=True)
    torch.cuda.synchronize()
    _ok(scores, g["scores"], torch.float32, f"{name} scores")
    _ok(mui, g["mui"], torch.float32, f"{name} mui")


@pytest.mark.parametrize("name", news_golden_names())
def test_fp32_bf16x6_matches_reference(name, monkeypatch):
    """The optional bf16x6 form of the fp32 kernel (MINER_NEWS_F32X6=1: every fp32 operand cut exactly
    into three bf16 terms, six bf16 MFMAs per contraction) at the same fp32 bar as the default."""
    monkeypatch.setenv("MINER_NEWS_F32X6", "1")
    test_fp32_matches_reference(name, "mfma32", monkeypatch)


def _f64_scores(table, hid, mask, cid, W1, Q, W2, score_type="weighted"):
    T = table.double().cpu()
    E, Cd = T[hid.cpu().long()], T[cid.cpu().long()]
    w1, q, w2 = (x.double().cpu() for x in (W1, Q, W2))
    s = torch.tanh(E @ w1.T) @ q.T                                       # [B, L, K]
    s = s.masked_fill(~mask.cpu()[:, :, None], 1e-30)
    a = torch.softmax(s, dim=1)
    mui = torch.einsum("blk,bld->bkd", a, E)
    x = torch.nn.functional.gelu(mui @ w2.T)
    m = Cd @ mui.transpose(1, 2)
    if score_type == "max":
        return m.max(-1).values
    lg = torch.softmax(Cd @ x.transpose(1, 2), dim=-1)
    return (lg * m).sum(-1)


@pytest.mark.parametrize("form", ["x2", "mfma32", "x6"])
def test_fp32_config3_vs_f64(form, monkeypatch):
    """Config-3 shape (L=50, C=40, K=32, d=768) against a float64 evaluation of the same products:
    every fp32 form (fp16 pairs on the fp16 MFMA, fp32 MFMA fma chains, bf16x6) stays well inside
    the fp32 parity bar."""
    monkeypatch.setenv("MINER_NEWS_FP32", "x2" if form == "x2" else "mfma32")
    if form == "x6":
        monkeypatch.setenv("MINER_NEWS_F32X6", "1")
    table, hid, mask, cid, offs, W1, Q, W2 = _setup(33, 300, 50, 768, 5000, torch.float32)
    nt = news.precompute(table, W1, Q, W2)
    scores = news.score(nt, hid, mask, cid)
    torch.cuda.synchronize()
    ref = _f64_scores(table, hid, mask, cid, W1, Q, W2)
    _ok(scores, ref, torch.float32, f"config-3 fp32 ({form}) vs float64")


@pytest.mark.parametrize("scale,score_type", [(1.0, "weighted"), (3e3, "max"), (2e-4, "weighted")])
def test_x2_error_vs_fp32_mfma(scale, score_type, monkeypatch):
    """The fp16-pair kernel is as accurate as the fp32-MFMA kernel: against float64, its worst and
    rms score errors stay within 1.5x those of the exact fp32 fma chains (tables scaled by 3e3 and
    2e-4 exercise the power-of-two pair scale; at 3e3 the 'weighted' softmax over K is one-hot and
    ill-conditioned in any fp32 form, so that scale is checked on 'max')."""
    table, hid, mask, cid, offs, W1, Q, W2 = _setup(34, 400, 50, 768, 6000, torch.float32)
    table = table * scale
    ref = _f64_scores(table, hid, mask, cid, W1, Q, W2, score_type)
    rms = float(ref.pow(2).mean().sqrt())
    errs = {}
    for kern in FP32_KERNELS:
        monkeypatch.setenv("MINER_NEWS_FP32", kern)
        nt = news.precompute(table, W1, Q, W2)
        s = news.score(nt, hid, mask, cid, score_type=score_type)
        torch.cuda.synchronize()
        e = (s.double().cpu() - ref).abs()
        # the parity bar's shape (|x - ref| <= 1e-5·|ref| + 1e-5·rms): error per unit of that bar
        errs[kern] = (float((e / (ref.abs() + rms)).max()), float(e.pow(2).mean().sqrt()))
        _ok(s, ref, torch.float32, f"{kern} at table scale {scale}")
    assert errs["x2"][0] <= 1.5 * errs["mfma32"][0] + 1e-7, errs
    assert errs["x2"][1] <= 1.5 * errs["mfma32"][1] + 1e-8 * rms, errs


def test_x2_weighted_large_scale_vs_reference_fp32(monkeypatch):
    """The case test_x2_error_vs_fp32_mfma leaves to 'max': a table scaled by 3e3 under 'weighted',
    where the softmax over K is one-hot and ill-conditioned in any fp32 form. Both fp32 kernels'
    worst and rms errors against float64 stay within 1.5x those of the reference's own fp32
    arithmetic (the oracle's CPU restatement of model.py:159-216, ATen ops in the reference's order)
    on the same inputs."""
    table, hid, mask, cid, offs, W1, Q, W2 = _setup(34, 400, 50, 768, 6000, torch.float32)
    table = table * 3e3
    ref = _f64_scores(table, hid, mask, cid, W1, Q, W2)
    rms = float(ref.pow(2).mean().sqrt())

    def err(x):
        e = (x.double().cpu() - ref).abs()
        return float((e / (ref.abs() + rms)).max()), float(e.pow(2).mean().sqrt() / rms)

    re = err(_oracle(table, hid, mask, cid, None, W1, Q, W2)[1])
    for kern in FP32_KERNELS:
        monkeypatch.setenv("MINER_NEWS_FP32", kern)
        s = news.score(news.precompute(table, W1, Q, W2), hid, mask, cid)
        torch.cuda.synchronize()
        ke = err(s)
        print(f"scale 3e3 weighted (max rel, rms rel): {kern} {ke}, reference fp32 {re}")
        assert ke[0] <= 1.5 * re[0] + 1e-7 and ke[1] <= 1.5 * re[1] + 1e-8, (kern, ke, re)


def _heavy_tailed(seed, B=240, L=50, d=768, n_news=4000, C=40):
    """A news table with the outliers encoder outputs have: three dimensions 100x the rest in every
    row, row 1 at 1e4x and row 2 at 1e5x the median row norm; impressions 0-79 touch the outlier
    rows (in the history: 0-19 row 1, 20-39 row 2; as a candidate: 40-59 row 1, 60-79 row 2),
    the rest never do."""
    g = torch.Generator().manual_seed(seed)
    t = torch.randn((n_news, d), generator=g) / d ** 0.5
    t[:, [5, 77, d // 2 + 16]] *= 100.0
    t[1] *= 1e4
    t[2] *= 1e5
    hid = torch.randint(3, n_news, (B, L), generator=g)
    lens = torch.randint(1, L + 1, (B,), generator=g)
    mask = torch.arange(L)[None, :] >= (L - lens)[:, None]
    hid[~mask] = 0
    cid = torch.randint(3, n_news, (B, C), generator=g)
    hid[0:20, L - 1] = 1
    hid[20:40, L - 1] = 2
    cid[40:60, 7] = 1
    cid[60:80, 3] = 2
    W1, Q, W2 = synthetic.init_weights(seed, d, 200, 32, device=DEV)
    return t.to(DEV), hid.to(DEV), mask.to(DEV), cid.to(DEV), W1, Q, W2


def test_x2_split_rows_exact_sum():
    """miner_news_split_x2: every row r is (hi + lo)·unit[r] with unit[r] a power of two and
    max|row| / unit[r] in [2^13, 2^14); each element within 2^-22 of itself (2^-24·unit absolute
    where lo falls below the fp16 normals), whatever the magnitude of the other rows."""
    table, *_ = _heavy_tailed(36, n_news=600, d=256)
    table[7] = 0.0                                    # an all-zero row
    table[8] *= 1e-20                                 # a tiny row
    t2, unit = news.split_x2(table)
    torch.cuda.synchronize()
    t2, unit, x = t2.cpu().float(), unit.cpu().double(), table.cpu().double()
    n, d = x.shape
    pl = t2.view(n, d // 64, 2, 64)
    back = (pl[:, :, 0, :].double() + pl[:, :, 1, :].double()).reshape(n, d) * unit[:, None]
    m = x.abs().max(dim=1).values
    e = torch.log2(unit)
    assert torch.equal(e, e.round()), "units are powers of two"
    nz = m > 0
    ratio = m[nz] / unit[nz]
    assert bool(((ratio >= 2 ** 13) & (ratio < 2 ** 14)).all()), ratio
    err = (back - x).abs()
    bound = torch.maximum(x.abs() * 2.0 ** -22, unit[:, None] * 2.0 ** -24)
    assert bool((err <= bound).all()), float((err / bound).max())


@pytest.mark.parametrize("score_type", ["max", "weighted"])
def test_x2_heavy_tailed(score_type, monkeypatch):
    """Heavy-tailed tables (rows 1e4x and 1e5x the median norm, a few dimensions 100x the rest):
    the fp16-pair kernel against float64 on the impressions that never touch the outlier rows, with
    the fp32 bar's rms taken over those impressions alone (an outlier row must not hide the error of
    the ordinary rows behind its own magnitude), and within 1.5x the fp32-MFMA kernel's error there;
    on the impressions that touch the outliers the same fp32 bar (rms over that subset) for both
    score types, and under 'weighted' (a one-hot, ill-conditioned softmax over K) also within 1.5x
    the error of the reference's own fp32 arithmetic, the oracle's CPU restatement."""
    table, hid, mask, cid, W1, Q, W2 = _heavy_tailed(35)
    ref = _f64_scores(table, hid, mask, cid, W1, Q, W2, score_type)
    subsets = {"ordinary": slice(80, None), "outlier": slice(0, 80)}
    errs = {}
    for kern in FP32_KERNELS:
        monkeypatch.setenv("MINER_NEWS_FP32", kern)
        nt = news.precompute(table, W1, Q, W2)
        s = news.score(nt, hid, mask, cid, score_type=score_type).double().cpu()
        torch.cuda.synchronize()
        for name, sl in subsets.items():
            r, x = ref[sl], s[sl]
            rms = float(r.pow(2).mean().sqrt())
            e = (x - r).abs()
            errs[(kern, name)] = (float((e / (r.abs() + rms)).max()), float(e.pow(2).mean().sqrt() / rms))
            _ok(x, r, torch.float32, f"{kern} {score_type} on the {name} impressions")
    for name in subsets:
        xe, me = errs[("x2", name)], errs[("mfma32", name)]
        assert xe[0] <= 1.5 * me[0] + 1e-7, (name, errs)
        assert xe[1] <= 1.5 * me[1] + 1e-8, (name, errs)
    if score_type == "weighted":
        # the outlier impressions under 'weighted', pinned to the reference's own arithmetic: the
        # oracle's fp32 restatement of model.py:159-216 (ATen ops in the reference's order, CPU) has
        # an error against float64 on them too, and both kernels stay within 1.5x of it
        sl = subsets["outlier"]
        r = ref[sl]
        rms = float(r.pow(2).mean().sqrt())
        x32 = _oracle(table, hid, mask, cid, None, W1, Q, W2, score_type)[1].double()[sl]
        e = (x32 - r).abs()
        re = (float((e / (r.abs() + rms)).max()), float(e.pow(2).mean().sqrt() / rms))
        print(f"outlier/weighted error (max rel, rms rel): reference fp32 {re}, "
              f"x2 {errs[('x2', 'outlier')]}, mfma32 {errs[('mfma32', 'outlier')]}")
        for kern in FP32_KERNELS:
            ke = errs[(kern, "outlier")]
            assert ke[0] <= 1.5 * re[0] + 1e-7 and ke[1] <= 1.5 * re[1] + 1e-8, (kern, ke, re)


@pytest.mark.parametrize("dtype", ["x2", "mfma32", torch.bfloat16])
@pytest.mark.parametrize("d,Dc,K", [(64, 32, 4), (256, 200, 32), (768, 200, 32), (192, 72, 16)])
def test_precompute_vs_f64(dtype, d, Dc, K, monkeypatch):
    """fp32 precompute in both forms (x2: the products on fp16 pairs, MINER_DTYPE_F32; mfma32: on the
    fp32 MFMA, MINER_DTYPE_F32_MFMA) and bf16, against float64."""
    if isinstance(dtype, str):
        monkeypatch.setenv("MINER_NEWS_FP32", dtype)
        dtype = torch.float32
    g = torch.Generator().manual_seed(d + K)
    n = 333
    table = (torch.randn((n, d), generator=g) / d ** 0.5).to(DEV, dtype)
    W1, Q, W2 = [w.to(dtype) for w in synthetic.init_weights(5, d, Dc, K, device=DEV)]
    nt = news.precompute(table, W1, Q, W2)
    torch.cuda.synchronize()
    E = table.double().cpu()
    logits = torch.tanh(E @ W1.double().cpu().T) @ Q.double().cpu().T
    proj = E @ W2.double().cpu().T
    _ok(nt.logits, logits, dtype, "logits")
    if dtype == torch.float32:
        _ok(nt.proj.float(), proj, dtype, "proj")
    else:   # proj is stored in bf16: one rounding of an fp32-accumulated product
        rel = float((nt.proj.double().cpu() - proj).abs().max() / proj.abs().max())
        assert rel < 1e-2, rel


def test_precompute_pairs_heavy_tailed():
    """The pair form of the fp32 precompute carries one power-of-two unit per table row: rows scaled
    by 2^-60 .. 2^60 keep the fp32 MFMA form's accuracy (within 1.5x its max and rms error against
    float64, relative to each row's own magnitude), and a row holding an infinity or a NaN gives the
    reference fp32 arithmetic's pattern of non-finite outputs without touching the other rows of its
    32-row tile."""
    d, Dc, K, n = 768, 200, 32, 96
    g = torch.Generator().manual_seed(606)
    base = torch.randn((n, d), generator=g) / d ** 0.5
    scale = torch.pow(2.0, torch.randint(-60, 61, (n, 1), generator=g).double()).float()
    table = base * scale
    table[3, 100] = float("inf")
    table[40, 5] = float("-inf")
    table[41, 9] = float("nan")
    W1, Q, W2 = synthetic.init_weights(7, d, Dc, K, device="cpu")
    W2[11, 100] = 0.0                                  # inf·0 = NaN in the reference's row 3, column 11
    out = {}
    for form in ("x2", "mfma32"):
        os.environ["MINER_NEWS_FP32"] = form
        try:
            nt = news.precompute(table.to(DEV), W1.to(DEV), Q.to(DEV), W2.to(DEV))
            torch.cuda.synchronize()
            out[form] = (nt.logits.double().cpu(), nt.proj.double().cpu())
        finally:
            os.environ.pop("MINER_NEWS_FP32", None)
    bad = torch.zeros(n, dtype=torch.bool)
    bad[[3, 40, 41]] = True
    E = table.double()
    ref = (torch.tanh(E @ W1.double().T) @ Q.double().T, E @ W2.double().T)
    ref32 = (torch.tanh(table @ W1.T) @ Q.T, table @ W2.T)
    for i, name in enumerate(("logits", "proj")):
        for form in ("x2", "mfma32"):
            got = out[form][i]
            # non-finite rows: the reference fp32 pattern (NaN where it is NaN, the same infinities)
            r32 = ref32[i][bad].double()
            assert torch.equal(torch.isnan(got[bad]), torch.isnan(r32)), (form, name)
            fin = torch.isfinite(r32)
            assert torch.equal(torch.isfinite(got[bad]), fin), (form, name)
            inf = torch.isinf(r32)
            assert torch.equal(got[bad][inf], r32[inf]), (form, name)
        # finite rows: error relative to each row's own magnitude
        r = ref[i][~bad]
        rms = r.pow(2).mean(dim=1, keepdim=True).sqrt()
        errs = {}
        for form in ("x2", "mfma32"):
            e = (out[form][i][~bad] - r).abs() / rms
            errs[form] = (float(e.max()), float(e.pow(2).mean().sqrt()))
        print(f"{name}: pairs {errs['x2']}, fp32 MFMA {errs['mfma32']}")
        assert errs["x2"][0] <= 1.5 * errs["mfma32"][0] + 1e-7, (name, errs)
        assert errs["x2"][1] <= 1.5 * errs["mfma32"][1] + 1e-8, (name, errs)


def test_precompute_infinite_row_bf16():
    """bf16 precompute (news_pre2), Dc = 200 (W1 padded to 224 rows): a table row holding an infinity
    saturates tanh as in the reference (finite logits), and a NaN row gives NaN logits; the padded
    rows' zero weights do not turn the infinite row NaN."""
    d, Dc, K, n = 768, 200, 32, 300
    g = torch.Generator().manual_seed(607)
    table = (torch.randn((n, d), generator=g) / d ** 0.5).to(torch.bfloat16)
    table[3, 100] = float("inf")
    table[260, 5] = float("-inf")
    table[261, 9] = float("nan")
    W1, Q, W2 = [w.to(torch.bfloat16) for w in synthetic.init_weights(8, d, Dc, K, device="cpu")]
    nt = news.precompute(table.to(DEV), W1.to(DEV), Q.to(DEV), W2.to(DEV))
    torch.cuda.synchronize()
    lg = nt.logits.cpu()
    ref = torch.tanh(table.float() @ W1.float().T) @ Q.float().T
    assert torch.equal(torch.isnan(lg), torch.isnan(ref))
    assert torch.isfinite(lg[[3, 260]]).all() and torch.isnan(lg[261]).all()
    ok = torch.ones(n, dtype=torch.bool)
    ok[[3, 260, 261]] = False
    _ok(lg[ok], ref[ok], torch.bfloat16, "logits of the finite rows")


# ---- shapes and layouts against the oracle --------------------------------------------------------
@pytest.mark.parametrize("dtype", ["x2", "mfma32", torch.bfloat16])
@pytest.mark.parametrize("B,L,d,C,K,Dc", [
    (300, 50, 768, 40, 32, 200),     # config 3 shape
    (700, 50, 256, 40, 32, 200),     # config 2 shape, several impressions per workgroup
    (257, 20, 64, 5, 4, 32),         # config 1 shape: one 64-column chunk (no prefetch overlap)
    (90, 64, 128, 33, 8, 48),        # L = 64, two chunks
    (64, 1, 192, 1, 32, 72),         # L = 1, C = 1
    (40, 37, 320, 150, 12, 64),      # three candidate passes
])
def test_vs_oracle(dtype, B, L, d, C, K, Dc, monkeypatch):
    if isinstance(dtype, str):
        monkeypatch.setenv("MINER_NEWS_FP32", dtype)
        dtype = torch.float32
    table, hid, mask, cid, offs, W1, Q, W2 = _setup(B + d, B, L, d, 2000, dtype, C=C, K=K, Dc=Dc)
    nt = news.precompute(table, W1, Q, W2)
    s, mui = news.score(nt, hid, mask, cid, return_user=True)
    torch.cuda.synchronize()
    ref_mui, ref = _oracle(table, hid, mask, cid, offs, W1, Q, W2)
    _ok(s, ref, dtype, "scores")
    _ok(mui, ref_mui, dtype, "mui")


@pytest.mark.parametrize("score_type", ["weighted", "max", "mean"])
@pytest.mark.parametrize("dtype", ["x2", "mfma32", torch.bfloat16])
def test_ragged_bias(score_type, dtype, monkeypatch):
    if isinstance(dtype, str):
        monkeypatch.setenv("MINER_NEWS_FP32", dtype)
        dtype = torch.float32
    table, hid, mask, cid, offs, W1, Q, W2 = _setup(7, 211, 50, 768, 3000, dtype, ragged=(0, 150))
    bias = torch.rand(hid.shape, device=DEV) - 0.5
    w2 = W2 if score_type == "weighted" else None
    nt = news.precompute(table, W1, Q, w2, with_proj=w2 is not None)
    s = news.score(nt, hid, mask, cid, score_type=score_type, cand_offsets=offs, his_bias=bias)
    torch.cuda.synchronize()
    _, ref = _oracle(table, hid, mask, cid, offs, W1, Q, w2, score_type, bias)
    _ok(s, ref, dtype, f"{score_type} scores")


@pytest.mark.parametrize("dtype", ["x2", "mfma32", torch.bfloat16])
def test_masked_slot_groups(dtype, monkeypatch):
    """The news kernels gather and contract the masked history slots holding one news id (the left
    padding) once, with a multiplicity (news_x2.hip dedupe_prep). Irregular inputs against the oracle:
    masks that are not left-aligned, several different ids under the mask, a masked slot sharing a
    clicked slot's id, repeated clicked ids, all-masked and no-masked histories, with category bias."""
    if isinstance(dtype, str):
        monkeypatch.setenv("MINER_NEWS_FP32", dtype)
        dtype = torch.float32
    B, L = 240, 50
    table, hid, mask, cid, offs, W1, Q, W2 = _setup(12, B, L, 768, 3000, dtype)
    g = torch.Generator(device="cpu").manual_seed(12)
    h = hid.cpu().clone()
    m = mask.cpu().clone()
    m[:60] = torch.rand((60, L), generator=g) < 0.5                   # scattered masks
    h[:60] = torch.randint(0, 6, (60, L), generator=g)                 # few ids: repeats everywhere
    h[60:120][~m[60:120]] = torch.randint(0, 3, (60, L), generator=g)[~m[60:120]]   # mixed ids under the mask
    h[120:150, :] = h[120:150, :1]                                     # every slot one id, masked or not
    m[150:170] = False                                                 # all masked, assorted ids
    h[150:170] = torch.randint(0, 3000, (20, L), generator=g)
    m[170:190] = True                                                  # nothing masked
    bias = torch.rand((B, L), generator=g) - 0.5
    hid, mask, bias = h.to(DEV), m.to(DEV), bias.to(DEV)
    nt = news.precompute(table, W1, Q, W2)
    s, mui = news.score(nt, hid, mask, cid, his_bias=bias, return_user=True)
    s_plain = news.score(nt, hid, mask, cid)
    torch.cuda.synchronize()
    ref_mui, ref = _oracle(table, hid, mask, cid, None, W1, Q, W2, bias=bias)
    _ok(s, ref, dtype, "scores")
    _ok(mui, ref_mui, dtype, "mui")
    _, ref_plain = _oracle(table, hid, mask, cid, None, W1, Q, W2)
    _ok(s_plain, ref_plain, dtype, "plain scores")


def test_spread_gram_nonfinite_row_isolated():
    """The spread Gram (MIND-shape LOSS kernel) hands each chunk's interest-tile-1 operand to the
    tile-0 wave through ring rows the history product reads times an attention weight of 0: an
    impression whose history holds an infinite table element must not leak NaN into the impressions
    that the same workgroup scores after it (4 per workgroup here). Its own D is not finite, as the
    reference's cosines of an infinite mui (utils.py:9-29); every other impression's D and scores
    match the oracle at the fp32 bar."""
    from miner_amd import evaluation
    B, L, d, n_news = 4 * 256, 50, 768, 3000
    table, hid, mask, cid, offs, W1, Q, W2 = _setup(717, B, L, d, n_news, torch.float32)
    bad_row, bad_imp = n_news - 1, 5
    hid[hid == bad_row] = 1
    cid[cid == bad_row] = 1
    hid[bad_imp, -1] = bad_row
    mask[bad_imp, -1] = True
    table[bad_row, 7] = float("inf")
    nt = news.precompute(table, W1, Q, W2, x2=True)
    s, dis = news.score(nt, hid, mask, cid, x2=True, disagreement=True)
    torch.cuda.synchronize()
    assert not torch.isfinite(dis[bad_imp]).item()
    keep = torch.ones(B, dtype=torch.bool, device=DEV)
    keep[bad_imp] = False
    ref_mui, ref_s = _oracle(table, hid[keep], mask[keep], cid[keep], None, W1, Q, W2)
    _ok(s[keep], ref_s, torch.float32, "scores of the other impressions")
    ref = evaluation.disagreement(ref_mui.double()).float()
    _ok(dis[keep], ref, torch.float32, "disagreement of the other impressions")


def test_x2_nan_logit_propagates(monkeypatch):
    """A NaN in a clicked slot's logit (here through the category bias) makes the reference's softmax
    over the history NaN for that impression (torch softmax propagates it, model.py:176-181), so every
    score of the impression is NaN; the x2 kernel's exp clamp must not turn it into a zero weight
    (fmaxf(NaN, -104) = -104). The other impressions stay at the fp32 bar."""
    monkeypatch.setenv("MINER_NEWS_FP32", "x2")
    B, L = 64, 50
    table, hid, mask, cid, offs, W1, Q, W2 = _setup(21, B, L, 768, 2000, torch.float32)
    mask[:, -1] = True                                   # the last slot is a click in every impression
    bias = (torch.rand(hid.shape, device=DEV) - 0.5)
    bad = torch.tensor([3, 17, 40], device=DEV)
    bias[bad, -1] = float("nan")
    nt = news.precompute(table, W1, Q, W2)
    s = news.score(nt, hid, mask, cid, his_bias=bias)
    torch.cuda.synchronize()
    _, ref = _oracle(table, hid, mask, cid, None, W1, Q, W2, bias=bias)
    s, ref = s.cpu().reshape(B, -1), ref.reshape(B, -1)
    assert torch.isnan(ref[bad.cpu()]).all()
    assert torch.equal(torch.isnan(s), torch.isnan(ref)), "NaN pattern differs from the reference"
    keep = torch.ones(B, dtype=torch.bool)
    keep[bad.cpu()] = False
    _ok(s[keep], ref[keep], torch.float32, "finite impressions")


def test_mui_only_and_all_padded():
    table, hid, mask, cid, offs, W1, Q, W2 = _setup(8, 50, 30, 256, 500, torch.float32)
    mask[:10] = False                      # all-padded histories: uniform average of pad rows
    hid[:10] = 0
    nt = news.precompute(table, W1, Q, W2)
    mui = news.score(nt, hid, mask, score_type="none")
    torch.cuda.synchronize()
    ref_mui, _ = _oracle(table, hid, mask, cid, None, W1, Q, W2)
    _ok(mui, ref_mui, torch.float32, "mui")


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_launch_invariance(dtype):
    """A big launch equals the same impressions scored a few at a time (bit-exact: the per-impression
    arithmetic does not depend on the workgroup an impression lands on)."""
    table, hid, mask, cid, offs, W1, Q, W2 = _setup(9, 3000, 50, 768, 20000, dtype)
    nt = news.precompute(table, W1, Q, W2)
    big = news.score(nt, hid, mask, cid)
    parts = torch.cat([news.score(nt, hid[i:i + 37], mask[i:i + 37], cid[i:i + 37]) for i in range(0, 3000, 37)])
    torch.cuda.synchronize()
    assert torch.isfinite(big).all()
    assert torch.equal(big, parts)


def test_agrees_with_dense_kernel_bf16():
    """The news path and the fused dense kernel (weights per impression) on the same inputs agree to
    bf16 rounding (they round different intermediates)."""
    table, hid, mask, cid, offs, W1, Q, W2 = _setup(10, 200, 50, 768, 4000, torch.bfloat16)
    nt = news.precompute(table, W1, Q, W2)
    a = news.score(nt, hid, mask, cid)
    b = ops.score_gather(table, hid, mask, cid, W1, Q, W2)
    torch.cuda.synchronize()
    err = float((a - b).abs().max() / b.pow(2).mean().sqrt())
    assert err < 0.1, err


def test_bad_inputs_raise():
    table, hid, mask, cid, offs, W1, Q, W2 = _setup(11, 8, 10, 256, 100, torch.bfloat16, C=5)
    nt = news.precompute(table, W1, Q, W2)
    bad = hid.clone()
    bad[3, 4] = 100
    with pytest.raises(ValueError, match="his_ids"):
        news.score(nt, bad, mask, cid)
    with pytest.raises(ValueError, match="at most"):
        news.score(nt, hid, mask, torch.zeros((8, 513), dtype=torch.int32, device=DEV))
    with pytest.raises(ValueError, match="Invalid method"):
        news.score(nt, hid, mask, cid, score_type="sum")
    with pytest.raises(ValueError, match="news path"):
        news.precompute(table[:, :96].contiguous(), W1[:, :96].contiguous(), Q, None, with_proj=False)


@pytest.mark.parametrize("shp_rt", [True, False])
@pytest.mark.parametrize("B,L,d,C,K,ragged", [
    (300, 50, 768, 40, 32, None),      # config 3 shape (compile-time MIND-shape LOSS kernel unless shp_rt)
    (700, 50, 256, 40, 32, None),      # config 2 shape (compile-time d = 256 LOSS kernel unless shp_rt)
    (257, 20, 64, 5, 4, None),         # config 1 shape: one chunk per row, K = 4
    (90, 64, 128, 33, 16, None),       # L = 64, K = 16 (interest tile 1 empty)
    (40, 37, 320, 150, 12, None),      # three candidate passes
    (211, 50, 768, None, 32, (0, 150)),  # ragged 0..150 candidates (compile-time LOSS kernel unless shp_rt)
    (130, 50, 768, 150, 32, None),     # MIND shape, three candidate passes per impression (spread Gram)
])
def test_fused_disagreement(B, L, d, C, K, ragged, shp_rt):
    """The eval loss's disagreement term formed inside the fp32 scoring kernel (the Gram matrix of
    mui, no mui written) equals the reference formula on the reference's own mui (float64), and the
    scores of the loss variant match the plain kernel's at the fp32 bar. The MIND shape (L = 50,
    K = 32, no bias, no mui output) runs the compile-time LOSS kernels (news_score_x2<WEIGHTED, *,
    12 | 4, 2, true>, the Gram spread over the four mui waves) that eval_loop's fused-loss path
    launches by default; shp_rt adds an all-zero category bias, which adds exactly 0 to every logit
    and selects the run-time-shape form (the Gram on two waves): both forms' D and scores must agree."""
    from miner_amd import evaluation
    table, hid, mask, cid, offs, W1, Q, W2 = _setup(B + d + K, B, L, d, 2000, torch.float32, C=C or 40, K=K,
                                                    ragged=ragged)
    zb = torch.zeros(hid.shape, device=DEV) if shp_rt else None
    nt = news.precompute(table, W1, Q, W2, x2=True)
    s_plain = news.score(nt, hid, mask, cid, cand_offsets=offs, x2=True)
    s, dis = news.score(nt, hid, mask, cid, cand_offsets=offs, his_bias=zb, x2=True, disagreement=True)
    torch.cuda.synchronize()
    # same arithmetic; hipcc may contract a multiply-add differently in the two instantiations
    _ok(s, s_plain, torch.float32, "loss-variant scores vs the plain kernel")
    ref_mui, ref_s = _oracle(table, hid, mask, cid, offs, W1, Q, W2)
    _ok(s, ref_s, torch.float32, "loss-variant scores vs the oracle")
    ref = evaluation.disagreement(ref_mui.double()).float()
    _ok(dis, ref, torch.float32, "disagreement")
    if not shp_rt:
        # the compile-time-shape kernels against the run-time form on the same inputs
        s_rt, dis_rt = news.score(nt, hid, mask, cid, cand_offsets=offs, his_bias=torch.zeros(hid.shape, device=DEV),
                                  x2=True, disagreement=True)
        torch.cuda.synchronize()
        _ok(s, s_rt, torch.float32, "compile-time-shape LOSS scores vs the run-time form")
        _ok(dis, dis_rt, torch.float32, "compile-time-shape disagreement vs the run-time form")
    # mui-only launch with the loss epilogue (score type 'none')
    m2, d2 = news.score(nt, hid, mask, score_type="none", x2=True, disagreement=True)
    torch.cuda.synchronize()
    _ok(d2, ref, torch.float32, "disagreement (none)")
