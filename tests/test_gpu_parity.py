"""HIP kernel parity vs the reference (golden fixtures) and the oracle — needs an MI355X.

Tolerances:
* fp32 mode (MINER_DTYPE_F32): |x - ref| <= 1e-5*|ref| + 1e-5*rms(ref)   (north_star 1e-5 relative;
  SURVEY.md §8c absolute floor for near-zero scores).
* bf16 mode: compared with the oracle evaluated in fp32 on the SAME bf16-rounded inputs and weights;
  the kernel also rounds its on-chip intermediates (tanh(E·W1ᵀ), attention weights, mui, gelu
  output) to bf16 MFMA operands, so the bound is |x - ref| <= 7e-3*|ref| + 2e-2*rms(ref) (3x tighter
  than round 1, set from the observed worst case: profiles/r02_tolerance_margins.txt), and the
  AUC computed from bf16 scores must stay within 5e-3 of the fp32 AUC.
"""
import numpy as np
import pytest
import torch

from oracle import miner_oracle as orc
from tests.conftest import golden_names, load_golden

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _ops():
    from miner_amd import ops
    return ops


def _dev(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a)).to(DEV)
    return t if dtype is None else t.to(dtype)


def _inputs(g, dtype):
    W2 = _dev(g["W2"], dtype) if "W2" in g else None
    bias = _dev(g["bias"], torch.float32) if g["use_bias"] else None
    return (_dev(g["E"], dtype), _dev(g["his_mask"]), _dev(g["cand"], dtype), _dev(g["W1"], dtype),
            _dev(g["Q"], dtype), W2, bias)


@pytest.mark.parametrize("form", ["x6", "mfma32"])
@pytest.mark.parametrize("name", golden_names())
def test_fp32_matches_reference(name, form, monkeypatch):
    """fp32 mode in both forms of the dense kernel: bf16x6 products on the bf16 matrix cores (the
    default) and the exact fp32-MFMA fma chains (MINER_DENSE_FP32=mfma32)."""
    if form == "mfma32":
        monkeypatch.setenv("MINER_DENSE_FP32", "mfma32")
    else:
        monkeypatch.delenv("MINER_DENSE_FP32", raising=False)
    g = load_golden(name)
    E, M, Cd, W1, Q, W2, bias = _inputs(g, torch.float32)
    scores, mui = _ops().score(E, M, Cd, W1, Q, W2, score_type=g["score_type"], his_bias=bias, return_user=True)
    torch.cuda.synchronize()
    ok, worst = orc.parity_ok(scores.cpu().numpy(), g["scores"])
    assert ok, f"{name}: scores off by {worst:.2f}x the tolerance"
    ok, worst = orc.parity_ok(mui.cpu().numpy(), g["mui"])
    assert ok, f"{name}: mui off by {worst:.2f}x the tolerance"


@pytest.mark.parametrize("name", golden_names())
def test_poly_attention_alone(name):
    g = load_golden(name)
    E, M, _, W1, Q, _, bias = _inputs(g, torch.float32)
    mui = _ops().poly_attention(E, M, W1, Q, his_bias=bias)
    torch.cuda.synchronize()
    ok, worst = orc.parity_ok(mui.cpu().numpy(), g["mui"])
    assert ok, f"{name}: mui off by {worst:.2f}x the tolerance"


@pytest.mark.parametrize("name", [n for n in golden_names() if load_golden(n)["score_type"] == "weighted"])
def test_target_aware_alone(name):
    g = load_golden(name)
    mui = torch.from_numpy(g["mui"])
    cand = torch.from_numpy(g["cand"])
    W2 = torch.from_numpy(g["W2"])
    value = torch.matmul(cand, mui.permute(0, 2, 1))
    ref = orc.target_aware_torch(mui, cand, value, W2)
    out = _ops().target_aware(mui.to(DEV), cand.to(DEV), value.to(DEV), W2.to(DEV))
    torch.cuda.synchronize()
    ok, worst = orc.parity_ok(out.cpu().numpy(), ref.numpy())
    assert ok, f"{name}: TAA off by {worst:.2f}x the tolerance"


def _bf16_round(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(torch.bfloat16).to(torch.float32)


@pytest.mark.parametrize("name", golden_names())
def test_bf16_within_tolerance(name):
    g = load_golden(name)
    E, M, Cd, W1, Q, W2, bias = _inputs(g, torch.bfloat16)
    scores = _ops().score(E, M, Cd, W1, Q, W2, score_type=g["score_type"], his_bias=bias)
    torch.cuda.synchronize()
    _, ref = orc.score_torch(_bf16_round(g["E"]), torch.from_numpy(g["his_mask"]), _bf16_round(g["cand"]),
                             _bf16_round(g["W1"]), _bf16_round(g["Q"]),
                             _bf16_round(g["W2"]) if "W2" in g else None, g["score_type"],
                             torch.from_numpy(g["bias"]) if g["use_bias"] else None)
    ok, worst = orc.parity_ok(scores.cpu().numpy(), ref.numpy(), rtol=7e-3, rms_floor=2e-2)
    assert ok, f"{name}: bf16 scores off by {worst:.2f}x the bf16 tolerance"


def test_ragged_equals_dense():
    g = load_golden("cfg3_slice")
    E, M, Cd, W1, Q, W2, _ = _inputs(g, torch.float32)
    dense = _ops().score(E, M, Cd, W1, Q, W2)
    B, C, d = Cd.shape
    # drop a different number of trailing candidates per impression -> ragged CSR batch
    keep = [C - 3 * b for b in range(B)]
    packed = torch.cat([Cd[b, :keep[b]] for b in range(B)])
    offs = torch.tensor([0] + list(np.cumsum(keep)), dtype=torch.int32, device=DEV)
    rag = _ops().score(E, M, packed, W1, Q, W2, cand_offsets=offs)
    torch.cuda.synchronize()
    want = torch.cat([dense[b, :keep[b]] for b in range(B)])
    ok, worst = orc.parity_ok(rag.cpu().numpy(), want.cpu().numpy())
    assert ok, worst


def test_many_candidates_chunked():
    """C > 64 exercises the multi-chunk S6/S7 loop; compared with the fp64 oracle."""
    rng = np.random.default_rng(11)
    B, L, K, d, Dc, C = 3, 30, 32, 128, 64, 150
    E = (rng.standard_normal((B, L, d)) / np.sqrt(d)).astype(np.float32)
    cand = (rng.standard_normal((B, C, d)) / np.sqrt(d)).astype(np.float32)
    mask = rng.random((B, L)) < 0.7
    W1 = ((rng.random((Dc, d)) * 2 - 1) / np.sqrt(d)).astype(np.float32)
    Q = ((rng.random((K, Dc)) * 2 - 1) * 0.2).astype(np.float32)
    W2 = ((rng.random((d, d)) * 2 - 1) / np.sqrt(d)).astype(np.float32)
    s = _ops().score(_dev(E), _dev(mask), _dev(cand), _dev(W1), _dev(Q), _dev(W2))
    torch.cuda.synchronize()
    _, ref = orc.score_f64(E, mask, cand, W1, Q, W2)
    ok, worst = orc.parity_ok(s.cpu().numpy(), ref)
    assert ok, worst


def test_config3_batch_properties():
    """Full config-3 shapes (L=50, K=32, d=768, Dc=200, C=40), several thousand impressions:
    a strided sample is checked against the oracle, and every impression's score is independent
    of the batch it is scored in (a shuffled sub-batch reproduces it)."""
    from miner_amd import synthetic
    B = 4096
    imp = synthetic.impressions(36, 0, B, L=50, d=768, C=40, device=DEV)
    W1, Q, W2 = synthetic.init_weights(36, 768, 200, 32, device=DEV)
    s = _ops().score(imp.history, imp.his_mask, imp.candidates, W1, Q, W2)
    idx = torch.arange(0, B, 97, device=DEV)
    _, ref = orc.score_torch(imp.history[idx].cpu(), imp.his_mask[idx].cpu(), imp.candidates[idx].cpu(),
                             W1.cpu(), Q.cpu(), W2.cpu())
    ok, worst = orc.parity_ok(s[idx].cpu().numpy(), ref.numpy())
    assert ok, worst
    perm = torch.randperm(B, device=DEV)[:1000]
    s2 = _ops().score(imp.history[perm], imp.his_mask[perm], imp.candidates[perm], W1, Q, W2)
    ok, worst = orc.parity_ok(s2.cpu().numpy(), s[perm].cpu().numpy(), rtol=1e-6, rms_floor=1e-6)
    assert ok, worst
    assert torch.isfinite(s).all()


def test_bf16_config3_auc_delta():
    from miner_amd import synthetic
    from miner_amd.evaluation import auc_score
    B = 2048
    imp = synthetic.impressions(36, 0, B, L=50, d=768, C=40, device=DEV)
    W1, Q, W2 = synthetic.init_weights(36, 768, 200, 32, device=DEV)
    s32 = _ops().score(imp.history, imp.his_mask, imp.candidates, W1, Q, W2)
    bf = torch.bfloat16
    s16 = _ops().score(imp.history.to(bf), imp.his_mask, imp.candidates.to(bf), W1.to(bf), Q.to(bf), W2.to(bf))
    lab = imp.labels.reshape(-1).cpu().numpy()
    a32 = auc_score(lab, torch.sigmoid(s32).reshape(-1).cpu().numpy())
    a16 = auc_score(lab, torch.sigmoid(s16).reshape(-1).cpu().numpy())
    assert abs(a32 - a16) < 5e-3, (a32, a16)


def test_unsupported_shape_raises():
    E = torch.zeros((2, 4, 64), device=DEV)
    M = torch.ones((2, 4), dtype=torch.bool, device=DEV)
    C = torch.zeros((2, 3, 64), device=DEV)
    W1 = torch.zeros((8, 64), device=DEV)
    Q = torch.zeros((65, 8), device=DEV)   # K = 65: past the fused kernel (32) and the wide path (64)
    W2 = torch.zeros((64, 64), device=DEV)
    with pytest.raises(ValueError):
        _ops().score(E, M, C, W1, Q, W2)
    with pytest.raises(ValueError):
        _ops().score(E, M, C, W1, Q[:4], W2, score_type="bogus")


def test_cpu_tensors_fail_loudly():
    E = torch.zeros((2, 4, 64))
    with pytest.raises(RuntimeError):
        _ops().score(E, torch.ones((2, 4), dtype=torch.bool), torch.zeros((2, 3, 64)),
                     torch.zeros((8, 64)), torch.zeros((4, 8)), torch.zeros((64, 64)))


@pytest.mark.parametrize("scale,score_type", [(1.0, "weighted"), (1.0, "max"), (1e-3, "weighted"), (300.0, "max")])
def test_x6_error_vs_fp32_mfma(scale, score_type, monkeypatch):
    """The dense fp32 kernel's bf16x6 products are as accurate as the fp32 MFMA: against float64
    (oracle.score_f64) the worst error per unit of the parity bar (|x - ref| / (|ref| + rms)) and the
    rms error stay within 1.5x those of the exact fp32 fma chains (bf16 keeps fp32's exponent range,
    so the row scale does not matter; 300 and 1e-3 check that — at 300 the 'weighted' softmax over K
    is one-hot and ill-conditioned in any fp32 form, so that scale is checked on 'max')."""
    g = torch.Generator().manual_seed(61)
    B, L, C, d, Dc, K = 96, 50, 40, 768, 200, 32
    E = torch.randn((B, L, d), generator=g) / d ** 0.5 * scale
    cand = torch.randn((B, C, d), generator=g) / d ** 0.5 * scale
    lens = torch.randint(1, L + 1, (B,), generator=g)
    mask = torch.arange(L)[None, :] >= (L - lens)[:, None]
    W1 = torch.randn((Dc, d), generator=g) * (2.0 / (Dc + d)) ** 0.5
    Q = torch.randn((K, Dc), generator=g) * (2.0 / (K + Dc)) ** 0.5
    W2 = torch.randn((d, d), generator=g) * (1.0 / d) ** 0.5
    _, ref = orc.score_f64(E.numpy(), mask.numpy(), cand.numpy(), W1.numpy(), Q.numpy(), W2.numpy(), score_type)
    ref = torch.from_numpy(ref)
    rms = float(ref.pow(2).mean().sqrt())
    errs = {}
    for form in ("x6", "mfma32"):
        if form == "mfma32":
            monkeypatch.setenv("MINER_DENSE_FP32", "mfma32")
        else:
            monkeypatch.delenv("MINER_DENSE_FP32", raising=False)
        s = _ops().score(E.to(DEV), mask.to(DEV), cand.to(DEV), W1.to(DEV), Q.to(DEV), W2.to(DEV), score_type=score_type)
        torch.cuda.synchronize()
        e = (s.double().cpu() - ref).abs()
        errs[form] = (float((e / (ref.abs() + rms)).max()), float(e.pow(2).mean().sqrt()))
        ok, worst = orc.parity_ok(s.cpu().numpy(), ref.numpy())
        assert ok, f"{form} at scale {scale} ({score_type}): off by {worst:.2f}x the tolerance"
    assert errs["x6"][0] <= 1.5 * errs["mfma32"][0] + 1e-7, errs
    assert errs["x6"][1] <= 1.5 * errs["mfma32"][1] + 1e-8 * rms, errs


def test_x6_infinite_history_element(monkeypatch):
    """An infinite element in a history row: the bf16x6 split of S1 (W1·Eᵀ) keeps hi =
    ±inf with finite residuals (cdna4_common.h split3_pair), so tanh(W1·e) saturates as in the
    reference instead of turning the impression NaN: mui equals the oracle's (torch fp32, the
    reference op order) — ±inf exactly in the affected column, the fp32 bar everywhere else — and
    the other impressions are untouched."""
    monkeypatch.delenv("MINER_DENSE_FP32", raising=False)
    g = torch.Generator().manual_seed(71)
    B, L, C, d, Dc, K = 8, 20, 5, 256, 64, 16
    E = torch.randn((B, L, d), generator=g) / d ** 0.5
    cand = torch.randn((B, C, d), generator=g) / d ** 0.5
    mask = torch.ones((B, L), dtype=torch.bool)
    W1 = torch.randn((Dc, d), generator=g) * (2.0 / (Dc + d)) ** 0.5
    Q = torch.randn((K, Dc), generator=g) * (2.0 / (K + Dc)) ** 0.5
    W2 = torch.randn((d, d), generator=g) * (1.0 / d) ** 0.5
    E[3, 7, 11] = float("inf")
    E[5, 2, 100] = float("-inf")
    s, mui = _ops().score(E.to(DEV), mask.to(DEV), cand.to(DEV), W1.to(DEV), Q.to(DEV), W2.to(DEV), return_user=True)
    torch.cuda.synchronize()
    ref_mui, ref = orc.score_torch(E, mask, cand, W1, Q, W2)
    mui = mui.cpu()
    assert torch.equal(torch.isnan(mui), torch.isnan(ref_mui)), "NaN pattern of mui differs from the reference"
    assert torch.equal(torch.isinf(mui), torch.isinf(ref_mui)), "inf pattern of mui differs from the reference"
    assert torch.equal(mui[torch.isinf(ref_mui)], ref_mui[torch.isinf(ref_mui)])
    fin = torch.isfinite(ref_mui)
    assert orc.parity_ok(mui[fin].numpy(), ref_mui[fin].numpy())[0]
    ok_rows = [b for b in range(B) if b not in (3, 5)]
    assert orc.parity_ok(s.cpu()[ok_rows].numpy(), ref[ok_rows].numpy())[0]


@pytest.mark.parametrize("where", ["history", "w_target"])
def test_pairs_nan_propagates(where, monkeypatch):
    """A NaN input stays NaN through the fp16-pair operands of the default fp32 form (S1 and S5):
    the pair clamp keeps it (v_med3 alone would return a finite bound), so the NaN pattern of mui and
    the scores is the reference's (torch fp32, the reference op order): one impression for a NaN
    history element, every score for a NaN in W2; everything finite matches at the fp32 bar."""
    monkeypatch.delenv("MINER_DENSE_FP32", raising=False)
    g = torch.Generator().manual_seed(72)
    B, L, C, d, Dc, K = 8, 20, 5, 256, 64, 16
    E = torch.randn((B, L, d), generator=g) / d ** 0.5
    cand = torch.randn((B, C, d), generator=g) / d ** 0.5
    mask = torch.ones((B, L), dtype=torch.bool)
    W1 = torch.randn((Dc, d), generator=g) * (2.0 / (Dc + d)) ** 0.5
    Q = torch.randn((K, Dc), generator=g) * (2.0 / (K + Dc)) ** 0.5
    W2 = torch.randn((d, d), generator=g) * (1.0 / d) ** 0.5
    if where == "history":
        E[3, 7, 11] = float("nan")
    else:
        W2[40, 9] = float("nan")
    s, mui = _ops().score(E.to(DEV), mask.to(DEV), cand.to(DEV), W1.to(DEV), Q.to(DEV), W2.to(DEV), return_user=True)
    torch.cuda.synchronize()
    ref_mui, ref = orc.score_torch(E, mask, cand, W1, Q, W2)
    mui, s = mui.cpu(), s.cpu()
    assert torch.isnan(ref).any()
    assert torch.equal(torch.isnan(mui), torch.isnan(ref_mui)), "NaN pattern of mui differs from the reference"
    assert torch.equal(torch.isnan(s), torch.isnan(ref)), "NaN pattern of the scores differs from the reference"
    fin = torch.isfinite(ref_mui)
    assert orc.parity_ok(mui[fin].numpy(), ref_mui[fin].numpy())[0]
    fs = torch.isfinite(ref)
    assert orc.parity_ok(s[fs].numpy(), ref[fs].numpy())[0]


@pytest.mark.parametrize("score_type", ["weighted", "max"])
def test_fp32_pairs_heavy_tailed(score_type, monkeypatch):
    """The default fp32 form runs S1 (W1·Eᵀ) and S5 (W2·muiᵀ) on fp16 pairs with a power-of-two unit
    per operand row (history row, mui row, weight row). Heavy-tailed inputs, as encoder outputs have
    them: three dimensions 100x the rest in every row, history / candidate rows 1e4x and 1e5x the
    median norm in impressions 0-79 (0-19 / 20-39 in the history, 40-59 / 60-79 as a candidate),
    and weight rows 30x the rest. Against float64 (oracle.score_f64), on the impressions that touch
    the outliers and on the others separately (each with its own rms, so an outlier row cannot hide
    the error of the ordinary ones): within 1.5x the fp32 MFMA's error, and the fp32 bar — except on
    the outlier impressions under 'weighted', where the softmax over K is one-hot and ill-conditioned
    in any fp32 arithmetic: there the pair form stays within 1.5x the error of the reference's own
    fp32 path (the oracle's CPU restatement, ATen ops in model.py's order)."""
    g = torch.Generator().manual_seed(83)
    B, L, C, d, Dc, K, n = 160, 50, 40, 768, 200, 32, 3000
    T = torch.randn((n, d), generator=g) / d ** 0.5
    T[:, [5, 77, d // 2 + 16]] *= 100.0
    T[1] *= 1e4
    T[2] *= 1e5
    hid = torch.randint(3, n, (B, L), generator=g)
    lens = torch.randint(1, L + 1, (B,), generator=g)
    mask = torch.arange(L)[None, :] >= (L - lens)[:, None]
    hid[~mask] = 0
    cid = torch.randint(3, n, (B, C), generator=g)
    hid[0:20, L - 1] = 1
    hid[20:40, L - 1] = 2
    cid[40:60, 7] = 1
    cid[60:80, 3] = 2
    E, cand = T[hid], T[cid]
    W1 = torch.randn((Dc, d), generator=g) * (2.0 / (Dc + d)) ** 0.5
    Q = torch.randn((K, Dc), generator=g) * (2.0 / (K + Dc)) ** 0.5
    W2 = torch.randn((d, d), generator=g) * (1.0 / d) ** 0.5
    W1[:4] *= 30.0
    W2[:16] *= 30.0
    _, ref = orc.score_f64(E.numpy(), mask.numpy(), cand.numpy(), W1.numpy(), Q.numpy(), W2.numpy(), score_type)
    ref = torch.from_numpy(ref)
    subsets = {"outlier": slice(0, 80), "ordinary": slice(80, None)}
    errs = {}
    for form in ("pairs", "mfma32"):
        if form == "mfma32":
            monkeypatch.setenv("MINER_DENSE_FP32", "mfma32")
        else:
            monkeypatch.delenv("MINER_DENSE_FP32", raising=False)
        s = _ops().score(E.to(DEV), mask.to(DEV), cand.to(DEV), W1.to(DEV), Q.to(DEV), W2.to(DEV),
                         score_type=score_type).double().cpu()
        torch.cuda.synchronize()
        for name, sl in subsets.items():
            r, x = ref[sl], s[sl]
            rms = float(r.pow(2).mean().sqrt())
            e = (x - r).abs()
            errs[(form, name)] = (float((e / (r.abs() + rms)).max()), float(e.pow(2).mean().sqrt() / rms))
            if score_type == "weighted" and name == "outlier":
                continue
            ok, worst = orc.parity_ok(x.numpy(), r.numpy())
            assert ok, f"{form} {score_type} on the {name} impressions: off by {worst:.2f}x the tolerance"
    for name in subsets:
        pe, me = errs[("pairs", name)], errs[("mfma32", name)]
        assert pe[0] <= 1.5 * me[0] + 1e-7, (name, errs)
        assert pe[1] <= 1.5 * me[1] + 1e-8, (name, errs)
    if score_type == "weighted":
        sl = subsets["outlier"]
        r = ref[sl]
        rms = float(r.pow(2).mean().sqrt())
        x32 = orc.score_torch(E, mask, cand, W1, Q, W2, score_type)[1].double()[sl]
        e = (x32 - r).abs()
        re = (float((e / (r.abs() + rms)).max()), float(e.pow(2).mean().sqrt() / rms))
        print(f"outlier/weighted error (max rel, rms rel): reference fp32 {re}, pairs {errs[('pairs', 'outlier')]}, "
              f"mfma32 {errs[('mfma32', 'outlier')]}")
        fe = errs[("pairs", "outlier")]      # (the fp32 MFMA form is looser here: its fma order)
        assert fe[0] <= 1.5 * re[0] + 1e-7 and fe[1] <= 1.5 * re[1] + 1e-8, (fe, re)
