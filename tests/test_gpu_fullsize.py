"""BASELINE.json's configs at their full per-GPU sizes — needs an MI355X.

The CPU oracle cannot score millions of impressions in a test, so the full launches are checked
through size-independent properties:
* a strided sample of each launch against the oracle, at the same bars as the small tests (fp32:
  1e-5·|ref| + 1e-5·rms; 16-bit: against the oracle on the same rounded inputs);
* batch independence: a shuffled sub-batch rescored alone reproduces its scores bit for bit (no
  cross-impression state anywhere in the kernels);
* every score finite.
Config 3 is the whole 3,000,000-impression MIND-large-shaped eval set of one GPU in the bench's
fp32 headline form (news ids over a 104k-row table). Config 2 has 50,000 impressions at d = 256,
config 4 has 50,000 FastFormer impressions, and config 5 is the bench's 2,048 users x 200,000 news
step with the fused top-100.
"""
import numpy as np
import pytest
import torch

from miner_amd import news, synthetic
from oracle import miner_oracle as orc

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _impressions(seed, B, L, C, n_news):
    g = torch.Generator(device=DEV).manual_seed(seed)
    lens = torch.randint(0, L + 1, (B,), generator=g, device=DEV)
    mask = torch.arange(L, device=DEV)[None, :] >= (L - lens)[:, None]
    hid = torch.randint(1, n_news, (B, L), generator=g, device=DEV, dtype=torch.int32)
    hid[~mask] = 0
    cid = torch.randint(1, n_news, (B, C), generator=g, device=DEV, dtype=torch.int32)
    return hid, mask, cid


def _sample_vs_oracle(table, hid, mask, cid, W1, Q, W2, scores, idx, rtol=1e-5, floor=1e-5):
    T = table.float().cpu()
    i = idx.cpu()
    h, m, c = hid.cpu()[i].long(), mask.cpu()[i], cid.cpu()[i].long()
    _, ref = orc.score_torch(T[h], m, T[c], W1.float().cpu(), Q.float().cpu(), W2.float().cpu())
    ok, worst = orc.parity_ok(scores[idx].cpu().numpy(), ref.numpy(), rtol=rtol, rms_floor=floor)
    assert ok, worst
    return worst


def _batch_independent(score_fn, hid, mask, cid, scores, n=20000, seed=3):
    perm = torch.randperm(hid.shape[0], generator=torch.Generator().manual_seed(seed))[:n].to(DEV)
    part = score_fn(hid[perm], mask[perm], cid[perm])
    assert torch.equal(part, scores[perm])


def test_config3_full_eval_set_fp32():
    """3,000,000 impressions (L=50, C=40, K=32, d=768, Dc=200) over a 104,000-row table, fp32."""
    B, L, C, d, n_news = 3_000_000, 50, 40, 768, 104_000
    g = torch.Generator(device=DEV).manual_seed(36)
    table = torch.randn((n_news, d), generator=g, device=DEV) / d ** 0.5
    W1, Q, W2 = synthetic.init_weights(36, d, 200, 32, device=DEV)
    hid, mask, cid = _impressions(36, B, L, C, n_news)
    nt = news.precompute(table, W1, Q, W2)
    scores = news.score(nt, hid, mask, cid, validate=False)
    torch.cuda.synchronize()
    assert torch.isfinite(scores).all()
    _sample_vs_oracle(table, hid, mask, cid, W1, Q, W2, scores, torch.arange(0, B, 9973, device=DEV))
    _batch_independent(lambda h, m, c: news.score(nt, h, m, c, validate=False), hid, mask, cid, scores)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_config2_full(dtype):
    """50,000 impressions at the MIND-small shape (d=256) over a 65,238-row table."""
    B, L, C, d, n_news = 50_000, 50, 40, 256, 65_238
    g = torch.Generator(device=DEV).manual_seed(2)
    t32 = torch.randn((n_news, d), generator=g, device=DEV) / d ** 0.5
    table = t32.to(dtype)
    W1, Q, W2 = (w.to(dtype) for w in synthetic.init_weights(2, d, 200, 32, device=DEV))
    hid, mask, cid = _impressions(2, B, L, C, n_news)
    nt = news.precompute(table, W1, Q, W2)
    scores = news.score(nt, hid, mask, cid, validate=False)
    torch.cuda.synchronize()
    assert torch.isfinite(scores).all()
    bars = {} if dtype == torch.float32 else {"rtol": 7e-3, "floor": 2e-2}
    _sample_vs_oracle(table, hid, mask, cid, W1, Q, W2, scores, torch.arange(0, B, 251, device=DEV), **bars)
    _batch_independent(lambda h, m, c: news.score(nt, h, m, c, validate=False), hid, mask, cid, scores, n=5000)


def test_config4_full_fastformer():
    """50,000 FastFormer impressions (L=50, C=40, hidden 256), bf16: a sample against the oracle on
    the same bf16-rounded inputs and weights, and batch independence."""
    from miner_amd import fastformer as ff
    from oracle import fastformer_oracle as ffo
    B, L, C, H = 50_000, 50, 40, 256
    g = torch.Generator(device=DEV).manual_seed(1000)
    lens = torch.randint(0, L + 1, (B,), generator=g, device=DEV)
    mask = torch.arange(L, device=DEV)[None, :] >= (L - lens)[:, None]
    hist = (torch.randn((B, L, H), generator=g, device=DEV) * 0.0625).to(torch.bfloat16)
    cand = (torch.randn((B, C, H), generator=g, device=DEV) * 0.0625).to(torch.bfloat16)
    params = synthetic.fastformer_params(0)
    packed = ff.pack(params.to(DEV), torch.bfloat16)
    s = ff.score(hist, mask, cand, packed)
    torch.cuda.synchronize()
    assert torch.isfinite(s).all()
    idx = torch.arange(0, B, 997, device=DEV)
    pdict = {n: t.reshape(shape) for (n, shape), t in
             zip(ff.PARAMS, torch.split(params, [int(np.prod(sh)) for _, sh in ff.PARAMS]))}
    pdict = {k: (v.to(torch.bfloat16).float() if (v.dim() == 2 and "position_embeddings" not in k) else v)
             for k, v in pdict.items()}
    with torch.no_grad():
        u = ffo.user_vectors(pdict, hist[idx].float().cpu(), mask[idx].cpu())
        ref = torch.matmul(cand[idx].float().cpu(), u.unsqueeze(-1)).squeeze(-1)
    ok, worst = orc.parity_ok(s[idx].cpu().numpy(), ref.numpy(), rtol=6e-3, rms_floor=1.2e-2)   # test_gpu_fastformer BF16_TOL
    assert ok, worst
    perm = torch.randperm(B, generator=torch.Generator().manual_seed(4))[:5000].to(DEV)
    assert torch.equal(ff.score(hist[perm], mask[perm], cand[perm], packed), s[perm])


def test_config5_bench_step_fp32():
    """2,048 users (L=200, K=64) against a 200,000-news table with the fused top-100, fp32: the top
    lists of a user sample against the oracle's full scores (same ids, scores within the fp32 bar),
    and each user's list unchanged when ranked alone."""
    from miner_amd import corpus
    from oracle import corpus_oracle as co
    U, L, K, N, d, topk = 2048, 200, 64, 200_000, 768, 100
    g = torch.Generator(device=DEV).manual_seed(5)
    table = torch.randn((N, d), generator=g, device=DEV) / d ** 0.5
    W1, Q, W2 = synthetic.init_weights(5, d, 200, K, device=DEV)
    pk = corpus.pack_encoder(W1, Q, W2, dtype=torch.float32)
    hid = torch.randint(0, N, (U, L), generator=g, device=DEV, dtype=torch.int32)
    lens = torch.randint(1, L + 1, (U,), generator=g, device=DEV)
    mask = torch.arange(L, device=DEV)[None, :] >= (L - lens)[:, None]
    mui, proj = corpus.encode_users(table, mask, pk, his_ids=hid)
    top_s, top_i = corpus.rank_topk(mui, proj, table, topk)
    torch.cuda.synchronize()
    assert torch.isfinite(top_s).all() and bool((top_i >= 0).all())
    users = [0, 777, 2047]
    T = table.cpu()
    with torch.no_grad():
        for u in users:
            m_u, p_u = co.encode(T[hid[u].cpu().long()][None], mask[u].cpu()[None], W1.cpu(), Q.cpu(), W2.cpu())
            full = co.corpus_scores(m_u, p_u, T)[0]                  # [N] fp32 oracle
            got_i = top_i[u].cpu().long()
            ok, worst = orc.parity_ok(top_s[u].cpu().numpy(), full[got_i].numpy())
            assert ok, (u, worst)
            kth = float(full[got_i].min())
            # no news outside the list scores clearly above the list's last entry
            outside = torch.ones(N, dtype=torch.bool)
            outside[got_i] = False
            assert float(full[outside].max()) <= kth + 1e-5 * float(full.abs().max()), u
    sub = torch.tensor(users, device=DEV)
    s2, i2 = corpus.rank_topk(mui[sub], proj[sub], table, topk)
    assert torch.equal(s2, top_s[sub]) and torch.equal(i2, top_i[sub])


def test_config5_bench_step_fp16():
    """The bench's config-5 step in its BASELINE dtype (fp16): 2,048 users (L=200, K=64) against a
    200,000-news fp16 table with the fused top-100. Sampled users' lists against the oracle's full
    200k scores computed from the kernel's own 16-bit user vectors and the fp16 table (the ranker's
    arithmetic: fp16 operands, fp32 accumulation; RANK16_TOL of tests/test_gpu_corpus.py), no news
    outside a list above its last entry, and batch independence (users ranked alone: same lists)."""
    from miner_amd import corpus
    from oracle import corpus_oracle as co
    U, L, K, N, d, topk = 2048, 200, 64, 200_000, 768, 100
    rtol = rms_floor = 2e-4
    g = torch.Generator(device=DEV).manual_seed(5)
    table = (torch.randn((N, d), generator=g, device=DEV) / d ** 0.5).to(torch.float16)
    W1, Q, W2 = synthetic.init_weights(5, d, 200, K, device=DEV)
    pk = corpus.pack_encoder(W1, Q, W2, dtype=torch.float16)
    hid = torch.randint(0, N, (U, L), generator=g, device=DEV, dtype=torch.int32)
    lens = torch.randint(1, L + 1, (U,), generator=g, device=DEV)
    mask = torch.arange(L, device=DEV)[None, :] >= (L - lens)[:, None]
    mui, proj = corpus.encode_users(table, mask, pk, his_ids=hid)
    top_s, top_i = corpus.rank_topk(mui, proj, table, topk)
    torch.cuda.synchronize()
    assert mui.dtype == torch.float16 and torch.isfinite(top_s).all() and bool((top_i >= 0).all())
    users = [0, 1, 777, 1500, 2047]
    T = table.float().cpu()
    with torch.no_grad():
        full = co.corpus_scores(mui[users].float().cpu(), proj[users].float().cpu(), T)   # [5, N] fp32
    rms = float(full.pow(2).mean().sqrt())
    for r, u in enumerate(users):
        got_i = top_i[u].cpu().long()
        assert len(set(got_i.tolist())) == topk
        true = full[r, got_i].double()
        err = (top_s[u].cpu().double() - true).abs()
        assert bool((err <= rtol * true.abs() + rms_floor * rms).all()), (u, float(err.max()))
        kth = float(true.min())
        outside = torch.ones(N, dtype=torch.bool)
        outside[got_i] = False
        assert float(full[r, outside].max()) <= kth + rms_floor * rms + rtol * abs(kth), u
    sub = torch.tensor(users, device=DEV)
    s2, i2 = corpus.rank_topk(mui[sub], proj[sub], table, topk)
    assert torch.equal(s2, top_s[sub]) and torch.equal(i2, top_i[sub])


def test_config5_per_gpu_share_fp16():
    """BASELINE config 5 at one GPU's share of its 1M users (8 GPUs: 125,000 users each) against the
    200,000-news fp16 table, history 200, K = 64, top-100, in one host loop (corpus.rank_corpus,
    16,384 users per encode + rank pair). Sampled users — batch boundaries included — against the
    oracle's full 200k scores from their own 16-bit user vectors (RANK16_TOL as above), no news
    outside a list above its last entry; and the first 20,000 users ranked in batches of 7,000 give
    the same lists bit for bit (batch independence)."""
    from miner_amd import corpus
    from oracle import corpus_oracle as co
    U, L, K, N, d, topk = 125_000, 200, 64, 200_000, 768, 100
    rtol = rms_floor = 2e-4
    g = torch.Generator(device=DEV).manual_seed(55)
    table = (torch.randn((N, d), generator=g, device=DEV) / d ** 0.5).to(torch.float16)
    W1, Q, W2 = synthetic.init_weights(55, d, 200, K, device=DEV)
    pk = corpus.pack_encoder(W1, Q, W2, dtype=torch.float16)
    hid = torch.randint(0, N, (U, L), generator=g, device=DEV, dtype=torch.int32)
    lens = torch.randint(1, L + 1, (U,), generator=g, device=DEV)
    mask = torch.arange(L, device=DEV)[None, :] >= (L - lens)[:, None]
    top_s, top_i = corpus.rank_corpus(table, hid, mask, pk, topk)
    torch.cuda.synchronize()
    assert torch.isfinite(top_s).all() and bool((top_i >= 0).all())
    users = [0, 16383, 16384, 77777, 124999]
    sub = torch.tensor(users, device=DEV)
    mui, proj = corpus.encode_users(table, mask[sub], pk, his_ids=hid[sub])
    T = table.float().cpu()
    with torch.no_grad():
        full = co.corpus_scores(mui.float().cpu(), proj.float().cpu(), T)      # [5, N] fp32
    rms = float(full.pow(2).mean().sqrt())
    for r, u in enumerate(users):
        got_i = top_i[u].cpu().long()
        assert len(set(got_i.tolist())) == topk
        true = full[r, got_i].double()
        err = (top_s[u].cpu().double() - true).abs()
        assert bool((err <= rtol * true.abs() + rms_floor * rms).all()), (u, float(err.max()))
        kth = float(true.min())
        outside = torch.ones(N, dtype=torch.bool)
        outside[got_i] = False
        assert float(full[r, outside].max()) <= kth + rms_floor * rms + rtol * abs(kth), u
    s2, i2 = corpus.rank_corpus(table, hid[:20000], mask[:20000], pk, topk, batch=7000)
    assert torch.equal(s2, top_s[:20000]) and torch.equal(i2, top_i[:20000])
