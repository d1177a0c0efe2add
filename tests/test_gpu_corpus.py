"""Full-corpus ranking (BASELINE config 5; miner_encode_users + miner_rank_topk) — needs an MI355X.

* fp32 parity mode vs the reference's own Miner scoring the whole table (tests/golden/corpus_*.npz):
  mui within 1e-5·|ref| + 1e-5·rms; the returned top-k checked entry by entry against the
  reference's score of that news id, best first, and no news outside the list beating the k-th;
* 16-bit modes (bf16, fp16): the encoder vs the oracle on the same rounded inputs/weights
  (1e-2·|ref| + 2e-2·rms), and the ranker vs the oracle evaluated on the kernel's own 16-bit user
  vectors (only fp32 summation order differs: 2e-4·|ref| + 2e-4·rms);
* gather == dense bit-exactly; odd U, N not a multiple of 256, topk > N, K = 32 and 64, L = 200.
"""
import os

import numpy as np
import pytest
import torch

from miner_amd import corpus
from oracle import corpus_oracle as co
from oracle import miner_oracle as orc

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
HERE = os.path.dirname(os.path.abspath(__file__))
F32_TOL = dict(rtol=1e-5, rms_floor=1e-5)
ENC16_TOL = dict(rtol=1e-2, rms_floor=2e-2)
RANK16_TOL = dict(rtol=2e-4, rms_floor=2e-4)


def load_corpus(name):
    z = np.load(os.path.join(HERE, "golden", name + ".npz"), allow_pickle=False)
    g = {k: z[k] for k in z.files}
    g["score_type"] = str(g["score_type"])
    return g


def check_topk(ts, ti, ref_scores, k, tol):
    """ts/ti: kernel top-k [U,k]; ref_scores [U,N] (float64 numpy)."""
    ts, ti = ts.cpu().numpy().astype(np.float64), ti.cpu().numpy().astype(np.int64)
    U, N = ref_scores.shape
    rms = float(np.sqrt(np.mean(ref_scores ** 2)))
    bound = lambda x: tol["rtol"] * np.abs(x) + tol["rms_floor"] * rms
    for u in range(U):
        n_ok = min(k, N)
        assert (ti[u, n_ok:] == -1).all() and np.isneginf(ts[u, n_ok:]).all()
        ids = ti[u, :n_ok]
        assert len(set(ids.tolist())) == n_ok and (ids >= 0).all() and (ids < N).all()
        true = ref_scores[u, ids]
        assert (np.abs(ts[u, :n_ok] - true) <= bound(true)).all(), f"user {u}: returned scores off"
        assert (np.diff(ts[u, :n_ok]) <= 0).all(), f"user {u}: not sorted"
        kth = true.min()
        rest = np.delete(ref_scores[u], ids)
        assert (rest <= kth + 2 * bound(kth)).all(), f"user {u}: a news outside the top-k beats it"


@pytest.mark.parametrize("name", ["corpus_c5_weighted", "corpus_c5_max", "corpus_k32_mean"])
def test_fp32_matches_reference(name):
    g = load_corpus(name)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)
    table, hid, mask = t(g["table"]), t(g["his_ids"]), t(g["his_mask"])
    w2 = t(g["W2"]) if "W2" in g else None
    pk = corpus.pack_encoder(t(g["W1"]), t(g["Q"]), w2, dtype=torch.float32)
    mui, proj, m32 = corpus.encode_users(table[hid], mask, pk, with_proj=w2 is not None, return_f32=True)
    assert orc.parity_ok(m32.cpu().numpy(), g["mui"], **F32_TOL)[0]
    assert torch.equal(mui, m32)
    mui_g, proj_g = corpus.encode_users(table, mask, pk, his_ids=hid, with_proj=w2 is not None)
    assert torch.equal(mui_g, mui) and (proj is None or torch.equal(proj_g, proj))
    N = table.shape[0]
    for k in (17, 256):
        ts, ti = corpus.rank_topk(mui, proj, table, k, score_type=g["score_type"])
        check_topk(ts, ti, g["scores"].astype(np.float64), k, F32_TOL)


def _round(x, dt):
    return x.to(dt).to(torch.float32)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("score_type", ["weighted", "max"])
def test_16bit_config5_dims(dtype, score_type):
    """config-5 dimensions (L=200, K=64, d=768, Dc=200) on 33 users x 3000 news."""
    gen = torch.Generator().manual_seed(5)
    U, L, K, d, Dc, N = 33, 200, 64, 768, 200, 3000
    table = torch.randn(N, d, generator=gen) / d ** 0.5
    hl = torch.randint(0, L + 1, (U,), generator=gen)
    mask = torch.arange(L)[None, :] >= (L - hl)[:, None]
    hid = torch.where(mask, torch.randint(1, N, (U, L), generator=gen), torch.zeros(U, L, dtype=torch.long))
    W1 = (torch.rand(Dc, d, generator=gen) * 2 - 1) / d ** 0.5
    Q = (torch.rand(K, Dc, generator=gen) * 2 - 1) * 0.3
    W2 = (torch.rand(d, d, generator=gen) * 2 - 1) / d ** 0.5
    pk = corpus.pack_encoder(W1.to(DEV), Q.to(DEV), W2.to(DEV), dtype=dtype)
    tab16 = table.to(DEV, dtype)
    mui, proj = corpus.encode_users(tab16, mask.to(DEV), pk, his_ids=hid.to(DEV).int())
    ref_mui, ref_proj = co.encode(_round(table, dtype)[hid], mask, _round(W1, dtype), _round(Q, dtype),
                                  _round(W2, dtype))
    assert orc.parity_ok(mui.float().cpu().numpy(), ref_mui.numpy(), **ENC16_TOL)[0]
    assert orc.parity_ok(proj.float().cpu().numpy(), ref_proj.numpy(), **ENC16_TOL)[0]
    ts, ti = corpus.rank_topk(mui, proj, tab16, 100, score_type=score_type)
    ref = co.corpus_scores(mui.float().cpu(), proj.float().cpu(), _round(table, dtype), score_type)
    check_topk(ts, ti, ref.double().numpy(), 100, RANK16_TOL)


def test_topk_larger_than_table_and_k32():
    gen = torch.Generator().manual_seed(9)
    U, L, K, d, Dc, N = 5, 40, 32, 64, 96, 100
    table = torch.randn(N, d, generator=gen) / d ** 0.5
    mask = torch.ones(U, L, dtype=torch.bool)
    hid = torch.randint(0, N, (U, L), generator=gen)
    W1 = torch.randn(Dc, d, generator=gen) / d ** 0.5
    Q = torch.randn(K, Dc, generator=gen) * 0.3
    W2 = torch.randn(d, d, generator=gen) / d ** 0.5
    pk = corpus.pack_encoder(W1.to(DEV), Q.to(DEV), W2.to(DEV), dtype=torch.float32)
    mui, proj = corpus.encode_users(table.to(DEV)[hid.to(DEV)], mask.to(DEV), pk)
    ref_mui, ref_proj = co.encode(table[hid], mask, W1, Q, W2)
    assert orc.parity_ok(mui.cpu().numpy(), ref_mui.numpy(), **F32_TOL)[0]
    for st in ("weighted", "max", "mean"):
        ts, ti = corpus.rank_topk(mui, proj, table.to(DEV), 128, score_type=st)
        ref = co.corpus_scores(ref_mui, ref_proj, table, st)
        check_topk(ts, ti, ref.double().numpy(), 128, F32_TOL)


def test_argument_errors():
    z = torch.zeros(2, 64, 128, device=DEV)
    with pytest.raises(ValueError):
        corpus.rank_topk(z, z, torch.zeros(10, 128, device=DEV), 300)
    with pytest.raises(ValueError):
        corpus.rank_topk(z, z, torch.zeros(10, 128, device=DEV), 5, score_type="sum")
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        corpus.rank_topk(z.cpu(), z.cpu(), torch.zeros(10, 128), 5)


@pytest.mark.parametrize("dtype", [torch.float16, torch.float32])
@pytest.mark.parametrize("U,N,topk", [(2048 // 16, 20000, 100), (3, 200, 256), (37, 5000, 7)])
def test_split_equals_unsplit(dtype, U, N, topk, monkeypatch):
    """miner_rank_topk_ws (news slices per XCD-shared user group + rk_merge) returns exactly the
    unsplit kernel's top-k: the same per-pair arithmetic, a total order (score desc, id asc) and
    disjoint slices. Duplicated news rows force exact score ties across slices."""
    gen = torch.Generator().manual_seed(U + N)
    K, d = 64, 768
    table = torch.randn(N, d, generator=gen) / d ** 0.5
    table[N // 2:N // 2 + 50] = table[:50]            # exact ties, ids in different slices
    mui = (torch.randn(U, K, d, generator=gen) / 4).to(DEV, dtype)
    proj = (torch.randn(U, K, d, generator=gen) / 4).to(DEV, dtype)
    tab = table.to(DEV, dtype)
    for st in ("weighted", "max"):
        monkeypatch.setenv("MINER_RK_SPLIT", "1")
        a = corpus.rank_topk(mui, proj, tab, topk, score_type=st)
        monkeypatch.setenv("MINER_RK_SPLIT", "0")
        b = corpus.rank_topk(mui, proj, tab, topk, score_type=st)
        torch.cuda.synchronize()
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]), st
        if N < topk:
            assert (a[1][:, N:] == -1).all()


def test_split_needs_its_workspace(monkeypatch):
    """The launch takes the split form only on a workspace whose stated size covers it: a buffer
    sized under another MINER_RK_SPLIT setting (here one 8-byte pair short) runs the unsplit form
    and is left untouched (the size query and the launch may see different settings)."""
    import ctypes
    from miner_amd import _lib
    gen = torch.Generator().manual_seed(11)
    U, N, K, d, topk = 37, 3000, 64, 768, 20
    mui = (torch.randn(U, K, d, generator=gen) / 4).to(DEV, torch.float16)
    proj = (torch.randn(U, K, d, generator=gen) / 4).to(DEV, torch.float16)
    tab = (torch.randn(N, d, generator=gen) / d ** 0.5).to(DEV, torch.float16)
    monkeypatch.setenv("MINER_RK_SPLIT", "0")
    ref_s, ref_i = corpus.rank_topk(mui, proj, tab, topk)
    monkeypatch.setenv("MINER_RK_SPLIT", "1")
    lib = _lib.lib()
    need = int(lib.miner_rank_topk_workspace_bytes(U, topk))
    assert need > 0
    ws = torch.full((need,), 0x5A, dtype=torch.uint8, device=DEV)
    ts = torch.empty(U, topk, device=DEV)
    ti = torch.empty(U, topk, dtype=torch.int32, device=DEV)
    rc = lib.miner_rank_topk_ws(torch.cuda.current_stream().cuda_stream, 2, 0, mui.data_ptr(), proj.data_ptr(),
                                tab.data_ptr(), U, N, d, K, topk, ts.data_ptr(), ti.data_ptr(), ws.data_ptr(),
                                ctypes.c_size_t(need - 8))
    assert rc == 0
    torch.cuda.synchronize()
    assert bool((ws == 0x5A).all()), "undersized workspace was written"
    assert torch.equal(ts, ref_s) and torch.equal(ti, ref_i)


@pytest.mark.parametrize("K", [64, 32])
@pytest.mark.parametrize("score_type", ["weighted", "max", "mean"])
def test_16bit_one_chunk_rows(K, score_type):
    """d = 64 in 16-bit: one d-chunk per news step, so the deferred top-k merge of a step meets the
    next step's epilogue with no chunk barrier in between (corpus.hip adds one) — against the oracle."""
    gen = torch.Generator().manual_seed(K + len(score_type))
    U, d, N = 9, 64, 700
    mui = torch.randn(U, K, d, generator=gen) / 2
    proj = torch.randn(U, K, d, generator=gen) / 2
    table = torch.randn(N, d, generator=gen) / d ** 0.5
    m16, p16, t16 = (x.to(DEV, torch.float16) for x in (mui, proj, table))
    ts, ti = corpus.rank_topk(m16, p16, t16, 50, score_type=score_type)
    ref = co.corpus_scores(m16.float().cpu(), p16.float().cpu(), t16.float().cpu(), score_type)
    check_topk(ts, ti, ref.double().numpy(), 50, RANK16_TOL)
