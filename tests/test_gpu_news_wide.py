"""The news-id path past the news kernels' K <= 32 / L <= 64: the per-news
precompute (logits in 32-interest slices of Q, proj = E·W2ᵀ, pair planes) + news_score_x2w, the
wide form of the fp32 pair-plane kernel (news_x2.hip: K <= 64, L <= 128) — needs an MI355X.

The reference limits neither K (num_context_codes, model.py:18-21) nor L (model.py:159-185). Parity:
* the three reference-generated wide_* fixtures (tests/golden/make_golden.py) at the fp32 bar
  |x - ref| <= 1e-5·|ref| + 1e-5·rms(ref), scores and mui;
* the oracle (oracle/miner_oracle.py) on config-3-like and irregular shapes at the same bar;
* the error against float64 within 1.5x the wide path's exact fp32 form (ue_fused + score_wide on the
  fp32 MFMA, which recomputes gelu(mui·W2ᵀ) per user);
* masked-slot groups across the two 64-slot halves, and a batch scored in one launch equals its
  impressions scored in pieces (bit-exact).
"""
import numpy as np
import pytest
import torch

from miner_amd import news, ops, synthetic
from oracle import miner_oracle as orc
from tests.conftest import load_golden, wide_golden_names

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _dev(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a)).to(DEV)
    return t if dtype is None else t.to(dtype)


def _ok(x, ref, what):
    x = x.detach().cpu().numpy() if isinstance(x, torch.Tensor) else x
    ref = ref.detach().cpu().numpy() if isinstance(ref, torch.Tensor) else ref
    ok, worst = orc.parity_ok(x, ref)
    assert ok, f"{what}: off by {worst:.2f}x the tolerance"
    return worst


@pytest.fixture(autouse=True)
def _x2(monkeypatch):
    monkeypatch.setenv("MINER_NEWS_FP32", "x2")


@pytest.mark.parametrize("name", wide_golden_names())
def test_wide_matches_reference(name):
    g = load_golden(name)
    weighted = g["score_type"] == "weighted"
    assert news.wide_supported(torch.float32, int(g["L"]), int(g["d"]), int(g["Dc"]), int(g["K"]))
    W2 = _dev(g["W2"]) if "W2" in g else None
    nt = news.precompute(_dev(g["table"]), _dev(g["W1"]), _dev(g["Q"]), W2 if weighted else None, with_proj=weighted)
    bias = _dev(g["bias"], torch.float32) if g["use_bias"] else None
    scores, mui = news.score(nt, _dev(g["his_ids"]), _dev(g["his_mask"]), _dev(g["cand_ids"]),
                             score_type=g["score_type"], his_bias=bias, return_user=True)
    torch.cuda.synchronize()
    _ok(scores, g["scores"], f"{name} scores")
    _ok(mui, g["mui"], f"{name} mui")


def _case(seed, B, L, K, d, C, n_news=3000, Dc=200, ragged=None, pad=True):
    gen = torch.Generator().manual_seed(seed)
    table = torch.randn((n_news, d), generator=gen) / d ** 0.5
    hid = torch.randint(0, n_news, (B, L), generator=gen)
    lens = torch.randint(0, L + 1, (B,), generator=gen) if pad else torch.full((B,), L)
    mask = torch.arange(L)[None, :] >= (L - lens)[:, None]
    hid[~mask] = 0
    if ragged:
        sizes = torch.randint(ragged[0], ragged[1] + 1, (B,), generator=gen)
        offs = torch.zeros(B + 1, dtype=torch.int32)
        offs[1:] = torch.cumsum(sizes, 0)
        cid = torch.randint(0, n_news, (int(offs[-1]),), generator=gen)
    else:
        offs, cid = None, torch.randint(0, n_news, (B, C), generator=gen)
    W1, Q, W2 = synthetic.init_weights(seed, d, Dc, K)
    return table, hid, mask, cid, offs, W1, Q, W2


def _oracle(table, hid, mask, cid, offs, W1, Q, W2, score_type="weighted", bias=None):
    E = table[hid.long()]
    w2 = W2 if score_type == "weighted" else None
    if offs is None:
        return orc.score_torch(E, mask, table[cid.long()], W1, Q, w2, score_type, bias)
    mui = orc.poly_attention_torch(E, mask, W1, Q, bias)
    o = offs.tolist()
    out = []
    for i in range(len(o) - 1):
        if o[i + 1] == o[i]:
            continue
        _, s = orc.score_torch(E[i:i + 1], mask[i:i + 1], table[cid[o[i]:o[i + 1]].long()].unsqueeze(0), W1, Q, w2,
                               score_type, None if bias is None else bias[i:i + 1])
        out.append(s.reshape(-1))
    return mui, torch.cat(out) if out else torch.zeros(0)


@pytest.mark.parametrize("B,L,K,d,C", [
    (256, 100, 64, 768, 40),     # the verdict's K = 64, L = 100, d = 768 case
    (300, 50, 64, 768, 40),      # K only past the limit
    (300, 100, 32, 768, 40),     # L only past the limit
    (200, 128, 36, 256, 70),     # L = 128 (both halves full), K = 36, two candidate passes
    (64, 65, 40, 64, 1),         # one 64-column chunk (two steps), C = 1
])
def test_wide_vs_oracle(B, L, K, d, C):
    table, hid, mask, cid, offs, W1, Q, W2 = _case(B + L + K, B, L, K, d, C)
    nt = news.precompute(table.to(DEV), W1.to(DEV), Q.to(DEV), W2.to(DEV))
    s, mui = news.score(nt, hid.to(DEV), mask.to(DEV), cid.to(DEV), return_user=True)
    torch.cuda.synchronize()
    ref_mui, ref = _oracle(table, hid, mask, cid, offs, W1, Q, W2)
    _ok(s, ref, "scores")
    _ok(mui, ref_mui, "mui")


@pytest.mark.parametrize("score_type", ["weighted", "max", "mean"])
def test_wide_ragged_bias(score_type):
    """Ragged 0..150 candidates (up to three passes of 64) with category bias, L = 90, K = 48."""
    table, hid, mask, cid, offs, W1, Q, W2 = _case(5, 150, 90, 48, 256, 0, ragged=(0, 150))
    bias = torch.rand(hid.shape, generator=torch.Generator().manual_seed(6)) - 0.5
    w2 = W2.to(DEV) if score_type == "weighted" else None
    nt = news.precompute(table.to(DEV), W1.to(DEV), Q.to(DEV), w2, with_proj=w2 is not None)
    s = news.score(nt, hid.to(DEV), mask.to(DEV), cid.to(DEV), score_type=score_type, cand_offsets=offs.to(DEV),
                   his_bias=bias.to(DEV))
    torch.cuda.synchronize()
    _, ref = _oracle(table, hid, mask, cid, offs, W1, Q, W2, score_type, bias)
    _ok(s, ref, f"{score_type} scores")


def test_wide_masked_groups_across_halves():
    """Masked slots of one id in both 64-slot halves form one group (dedupe over two ballots);
    scattered masks, several ids under the mask, all-masked and unmasked histories, L = 120, K = 64."""
    B, L = 160, 120
    table, hid, mask, cid, offs, W1, Q, W2 = _case(9, B, L, 64, 256, 40)
    g = torch.Generator().manual_seed(9)
    mask[:40] = torch.rand((40, L), generator=g) < 0.5
    hid[:40] = torch.randint(0, 5, (40, L), generator=g)
    mask[40:60] = torch.arange(L)[None, :] >= 100                 # first masked slot 0, group spans both halves
    hid[40:60, :100] = 7
    mask[60:80] = torch.arange(L)[None, :] < 70                   # masked tail in the second half only
    hid[60:80, 70:] = 3
    mask[80:100] = False
    hid[80:100] = torch.randint(0, 3000, (20, L), generator=g)
    mask[100:120] = True
    bias = torch.rand((B, L), generator=g) - 0.5
    nt = news.precompute(table.to(DEV), W1.to(DEV), Q.to(DEV), W2.to(DEV))
    s, mui = news.score(nt, hid.to(DEV), mask.to(DEV), cid.to(DEV), his_bias=bias.to(DEV), return_user=True)
    mui_only = news.score(nt, hid.to(DEV), mask.to(DEV), score_type="none")
    torch.cuda.synchronize()
    ref_mui, ref = _oracle(table, hid, mask, cid, None, W1, Q, W2, bias=bias)
    _ok(s, ref, "scores")
    _ok(mui, ref_mui, "mui")
    ref_mui0, _ = _oracle(table, hid, mask, cid, None, W1, Q, W2)
    _ok(mui_only, ref_mui0, "mui only (no bias)")


def test_wide_launch_invariance():
    """3,000 impressions in one launch == the same impressions scored 37 at a time (bit-exact)."""
    table, hid, mask, cid, offs, W1, Q, W2 = _case(13, 3000, 100, 64, 256, 40)
    nt = news.precompute(table.to(DEV), W1.to(DEV), Q.to(DEV), W2.to(DEV))
    h, m, c = hid.to(DEV), mask.to(DEV), cid.to(DEV)
    full = news.score(nt, h, m, c)
    parts = torch.cat([news.score(nt, h[i:i + 37], m[i:i + 37], c[i:i + 37]) for i in range(0, 3000, 37)])
    torch.cuda.synchronize()
    assert torch.equal(full, parts)


def test_wide_error_vs_fp32_path():
    """Error against float64 within 1.5x that of the wide path's exact-fp32 form (miner_encode_users
    + miner_score_wide on the fp32 MFMA), at K = 64, L = 100, d = 768."""
    table, hid, mask, cid, offs, W1, Q, W2 = _case(17, 96, 100, 64, 768, 40)
    nt = news.precompute(table.to(DEV), W1.to(DEV), Q.to(DEV), W2.to(DEV))
    s = news.score(nt, hid.to(DEV), mask.to(DEV), cid.to(DEV))
    s32 = ops.score_gather(table.to(DEV), hid.to(DEV), mask.to(DEV), cid.to(DEV), W1.to(DEV), Q.to(DEV), W2.to(DEV))
    torch.cuda.synchronize()
    ref = orc.score_f64(table[hid.long()].numpy(), mask.numpy(), table[cid.long()].numpy(), W1.numpy(), Q.numpy(),
                        W2.numpy())[1]
    rms = float(np.sqrt((ref ** 2).mean()))
    e_x2 = float(np.abs(s.double().cpu().numpy() - ref).max()) / rms
    e_32 = float(np.abs(s32.double().cpu().numpy() - ref).max()) / rms
    assert e_x2 <= 1.5 * e_32 + 1e-7, (e_x2, e_32)
    _ok(s, ref, "vs float64")


def test_wide_errors():
    table, hid, mask, cid, offs, W1, Q, W2 = _case(3, 4, 130, 64, 256, 4)
    nt = news.precompute(table.to(DEV), W1.to(DEV), Q.to(DEV), W2.to(DEV))
    with pytest.raises(ValueError):                          # L = 130 > 128
        news.score(nt, hid.to(DEV), mask.to(DEV), cid.to(DEV))
    with pytest.raises(ValueError):                          # no in-kernel disagreement in the wide form
        news.score(nt, hid[:, :100].to(DEV), mask[:, :100].to(DEV), cid.to(DEV), disagreement=True)
