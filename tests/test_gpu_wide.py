"""The wide path (include/miner_wide.h: miner_encode_users + miner_score_wide, miner_wide_proj) for
reference-legal shapes past the fused kernels' K <= 32 / L <= 64 — needs an MI355X.

The reference has no such limits (num_context_codes free, model.py:18-21; PolyAttention shape-generic,
:159-185). The golden wide_* fixtures are the reference's own outputs (make_golden.py) and run through
every -m gpu test that iterates the golden fixtures (ops, modules, metrics); this file adds the input
modes and sizes those do not reach. fp32 bar: |x - ref| <= 1e-5·|ref| + 1e-5·rms(ref); 16-bit: the
oracle on the same rounded inputs, 7e-3·|ref| + 2e-2·rms(ref) (the bf16 bar of test_gpu_parity.py).
"""
import numpy as np
import pytest
import torch

from oracle import miner_oracle as orc
from tests.conftest import load_golden, wide_golden_names

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _ops():
    from miner_amd import ops
    return ops


def _dev(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a)).to(DEV)
    return t if dtype is None else t.to(dtype)


def _weights(rng, d, Dc, K):
    W1 = ((rng.random((Dc, d)) * 2 - 1) / np.sqrt(d)).astype(np.float32)
    Q = ((rng.random((K, Dc)) * 2 - 1) * 0.3).astype(np.float32)
    W2 = ((rng.random((d, d)) * 2 - 1) / np.sqrt(d)).astype(np.float32)
    return W1, Q, W2


@pytest.mark.parametrize("name", wide_golden_names())
def test_gather_equals_dense(name):
    """News-id input (the eval layout) and dense rows give the same scores and mui."""
    g = load_golden(name)
    W2 = _dev(g["W2"]) if "W2" in g else None
    bias = _dev(g["bias"], torch.float32) if g["use_bias"] else None
    dense, mui_d = _ops().score(_dev(g["E"]), _dev(g["his_mask"]), _dev(g["cand"]), _dev(g["W1"]), _dev(g["Q"]), W2,
                                score_type=g["score_type"], his_bias=bias, return_user=True)
    gath, mui_g = _ops().score_gather(_dev(g["table"]), _dev(g["his_ids"]), _dev(g["his_mask"]), _dev(g["cand_ids"]),
                                      _dev(g["W1"]), _dev(g["Q"]), W2, score_type=g["score_type"], his_bias=bias,
                                      return_user=True)
    torch.cuda.synchronize()
    assert torch.equal(dense, gath)
    assert torch.equal(mui_d, mui_g)
    assert orc.parity_ok(gath.cpu().numpy(), g["scores"])[0]


@pytest.mark.parametrize("score_type", ["weighted", "max", "mean"])
def test_ragged_many_candidates(score_type):
    """Ragged candidate counts 0 / 1 / 64 / 65 / 150 (passes of 64), L = 150, K = 48, against float64."""
    rng = np.random.default_rng(21)
    B, L, K, d, Dc = 5, 150, 48, 128, 64
    counts = [0, 150, 65, 1, 64]
    E = (rng.standard_normal((B, L, d)) / np.sqrt(d)).astype(np.float32)
    mask = rng.random((B, L)) < 0.6
    mask[0] = False                                    # an all-padded history
    N = sum(counts)
    cand = (rng.standard_normal((N, d)) / np.sqrt(d)).astype(np.float32)
    offs = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    W1, Q, W2 = _weights(rng, d, Dc, K)
    s = _ops().score(_dev(E), _dev(mask), _dev(cand), _dev(W1), _dev(Q), _dev(W2), score_type=score_type,
                     cand_offsets=_dev(offs))
    torch.cuda.synchronize()
    s = s.cpu().numpy()
    for b in range(B):
        if counts[b] == 0:
            continue
        _, ref = orc.score_f64(E[b:b + 1], mask[b:b + 1], cand[None, offs[b]:offs[b + 1]], W1, Q, W2, score_type)
        ok, worst = orc.parity_ok(s[offs[b]:offs[b + 1]], ref.reshape(-1))
        assert ok, (b, worst)


def test_config5_dims_bf16_and_fp32():
    """K = 64, L = 200, d = 768, Dc = 200 (the config-5 user dims) on 40 impressions x 40 candidates."""
    from miner_amd import synthetic
    rng = np.random.default_rng(22)
    B, L, K, d, Dc, C = 40, 200, 64, 768, 200, 40
    imp = synthetic.impressions(36, 0, B, L=L, d=d, C=C, device=DEV)
    W1, Q, W2 = (_dev(w) for w in _weights(rng, d, Dc, K))
    s32 = _ops().score(imp.history, imp.his_mask, imp.candidates, W1, Q, W2)
    _, ref = orc.score_torch(imp.history.cpu(), imp.his_mask.cpu(), imp.candidates.cpu(), W1.cpu(), Q.cpu(), W2.cpu())
    ok, worst = orc.parity_ok(s32.cpu().numpy(), ref.numpy())
    assert ok, worst
    bf = torch.bfloat16
    s16 = _ops().score(imp.history.to(bf), imp.his_mask, imp.candidates.to(bf), W1.to(bf), Q.to(bf), W2.to(bf))
    r = lambda t: t.to(bf).float().cpu()
    _, ref16 = orc.score_torch(r(imp.history), imp.his_mask.cpu(), r(imp.candidates), r(W1), r(Q), r(W2))
    ok, worst = orc.parity_ok(s16.cpu().numpy(), ref16.numpy(), rtol=7e-3, rms_floor=2e-2)
    assert ok, worst


def test_target_aware_alone_k64():
    """TargetAwareAttention.forward (model.py:200-216) at K = 64: miner_wide_proj + miner_score_wide."""
    rng = np.random.default_rng(23)
    B, K, d, C = 6, 64, 256, 70
    mui = (rng.standard_normal((B, K, d)) / np.sqrt(d)).astype(np.float32)
    cand = (rng.standard_normal((B, C, d)) / np.sqrt(d)).astype(np.float32)
    W2 = ((rng.random((d, d)) * 2 - 1) / np.sqrt(d)).astype(np.float32)
    value = np.matmul(cand, mui.transpose(0, 2, 1)).astype(np.float32)
    ref = orc.target_aware_torch(torch.from_numpy(mui), torch.from_numpy(cand), torch.from_numpy(value),
                                 torch.from_numpy(W2))
    out = _ops().target_aware(_dev(mui), _dev(cand), _dev(value), _dev(W2))
    torch.cuda.synchronize()
    ok, worst = orc.parity_ok(out.cpu().numpy(), ref.numpy())
    assert ok, worst


def test_poly_attention_wide_with_bias():
    rng = np.random.default_rng(24)
    B, L, K, d, Dc = 7, 100, 40, 192, 96
    E = (rng.standard_normal((B, L, d)) / np.sqrt(d)).astype(np.float32)
    mask = rng.random((B, L)) < 0.5
    bias = rng.standard_normal((B, L)).astype(np.float32) * 0.3
    W1, Q, _ = _weights(rng, d, Dc, K)
    mui = _ops().poly_attention(_dev(E), _dev(mask), _dev(W1), _dev(Q), his_bias=_dev(bias))
    ref = orc.poly_attention_torch(torch.from_numpy(E), torch.from_numpy(mask), torch.from_numpy(W1),
                                   torch.from_numpy(Q), torch.from_numpy(bias))
    torch.cuda.synchronize()
    ok, worst = orc.parity_ok(mui.cpu().numpy(), ref.numpy())
    assert ok, worst


def test_launch_invariance():
    """An impression's score does not depend on the batch it is scored in."""
    g = load_golden("wide_k64_l120")
    args = (_dev(g["W1"]), _dev(g["Q"]), _dev(g["W2"]))
    full = _ops().score(_dev(g["E"]), _dev(g["his_mask"]), _dev(g["cand"]), *args)
    part = _ops().score(_dev(g["E"][2:5]), _dev(g["his_mask"][2:5]), _dev(g["cand"][2:5]), *args)
    torch.cuda.synchronize()
    assert torch.equal(full[2:5], part)
