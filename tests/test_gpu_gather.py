"""News-table gather mode (miner_score_gather) against the dense path on the same
rows — needs an MI355X. Both paths feed the kernel identical rows: bf16 results are bit-identical;
the fp32 parity path sums its S6 partials with LDS atomics (order not fixed), so fp32 is compared
within 1e-6 relative."""
import numpy as np
import pytest
import torch

from miner_amd import ops, synthetic
from oracle import miner_oracle as orc

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _same(a, b, dtype):
    if dtype == torch.bfloat16:
        assert torch.equal(a, b), float((a - b).abs().max())
    else:
        ok, worst = orc.parity_ok(a.cpu().numpy(), b.cpu().numpy(), rtol=1e-6, rms_floor=1e-6)
        assert ok, worst


def _setup(seed, B, L, d, C, n_news, dtype, ragged=None, Dc=200, K=32):
    g = torch.Generator(device="cpu").manual_seed(seed)
    table = (torch.randn((n_news, d), generator=g) / d ** 0.5).to(DEV, dtype)
    his_ids = torch.randint(0, n_news, (B, L), generator=g).to(DEV)
    lens = torch.randint(0, L + 1, (B,), generator=g)
    mask = (torch.arange(L)[None, :] >= (L - lens)[:, None]).to(DEV)
    his_ids[~mask] = 0                      # left padding = the pad news (row 0), as reader.py
    if ragged:
        sizes = torch.randint(ragged[0], ragged[1] + 1, (B,), generator=g)
        offs = torch.zeros(B + 1, dtype=torch.int32)
        offs[1:] = torch.cumsum(sizes, 0)
        cand_ids = torch.randint(0, n_news, (int(offs[-1]),), generator=g).to(DEV)
        offs = offs.to(DEV)
    else:
        cand_ids = torch.randint(0, n_news, (B, C), generator=g).to(DEV)
        offs = None
    W1, Q, W2 = synthetic.init_weights(seed, d, Dc, K, device=DEV)
    return table, his_ids, mask, cand_ids, offs, W1.to(dtype), Q.to(dtype), W2.to(dtype)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("d", [256, 768])
def test_gather_equals_dense(dtype, d):
    table, hid, mask, cid, offs, W1, Q, W2 = _setup(1, 97, 50, d, 40, 5000, dtype)
    pw = ops.pack_weights(W1, Q, W2, dtype=dtype)
    a, mui_a = ops.score_gather(table, hid, mask, cid, pw, return_user=True)
    b, mui_b = ops.score(table[hid], mask, table[cid], pw, return_user=True)
    torch.cuda.synchronize()
    _same(a, b, dtype)
    _same(mui_a, mui_b, dtype)


@pytest.mark.parametrize("score_type", ["weighted", "max", "mean"])
def test_gather_ragged_chunks_bias(score_type):
    dtype = torch.bfloat16
    table, hid, mask, cid, offs, W1, Q, W2 = _setup(2, 131, 50, 768, 0, 3000, dtype, ragged=(0, 150))
    bias = torch.rand(hid.shape, device=DEV) - 0.5
    w2 = W2 if score_type == "weighted" else None
    a = ops.score_gather(table, hid, mask, cid, W1, Q, w2, score_type=score_type, cand_offsets=offs, his_bias=bias)
    b = ops.score(table[hid], mask, table[cid], W1, Q, w2, score_type=score_type, cand_offsets=offs, his_bias=bias)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


def test_gather_fp32_ragged():
    table, hid, mask, cid, offs, W1, Q, W2 = _setup(3, 45, 20, 128, 0, 700, torch.float32, ragged=(1, 70), Dc=64, K=8)
    a = ops.score_gather(table, hid, mask, cid, W1, Q, W2, cand_offsets=offs)
    b = ops.score(table[hid], mask, table[cid], W1, Q, W2, cand_offsets=offs)
    torch.cuda.synchronize()
    _same(a, b, torch.float32)


def test_bad_ids_raise():
    table, hid, mask, cid, offs, W1, Q, W2 = _setup(4, 8, 10, 256, 5, 100, torch.bfloat16)
    bad = hid.clone()
    bad[3, 4] = 100
    with pytest.raises(ValueError, match="his_ids"):
        ops.score_gather(table, bad, mask, cid, W1, Q, W2)
    badc = cid.clone()
    badc[0, 0] = -1
    with pytest.raises(ValueError, match="cand_ids"):
        ops.score_gather(table, hid, mask, badc, W1, Q, W2)
