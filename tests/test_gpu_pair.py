"""The bf16 impression-pair kernel (miner_score with a workspace) against the single-impression
kernel (no workspace) — needs an MI355X.

Both kernels do the same per-impression arithmetic in the same order (the pair kernel only shares
the W2 stream of S5 between two impressions and parks the first impression's mui in a bf16
scratch, which is lossless for bf16 operands), so the results must be bit-identical. Edge cases:
odd impression counts (the last pair holds one impression), ragged candidates including empty
impressions and more than one 64-candidate chunk, the category bias, max/mean aggregation and the
mui output.
"""
import numpy as np
import pytest
import torch

from miner_amd import _lib, ops, synthetic

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
BF = torch.bfloat16


def _weights(d, Dc=200, K=32, seed=36):
    W1, Q, W2 = synthetic.init_weights(seed, d, Dc, K, device=DEV)
    return W1.to(BF), Q.to(BF), W2.to(BF)


def _both(*args, **kw):
    a = ops.score(*args, use_workspace=True, **kw)
    b = ops.score(*args, use_workspace=False, **kw)
    torch.cuda.synchronize()
    return a, b


def _same(a, b):
    if isinstance(a, tuple):
        for x, y in zip(a, b):
            _same(x, y)
        return
    assert a.shape == b.shape
    assert torch.isfinite(a).all()
    assert torch.equal(a, b), float((a - b).abs().max())


def test_workspace_query():
    lib = _lib.lib()
    n = lib.miner_score_workspace_bytes(_lib.DTYPE_BF16, _lib.SCORE_WEIGHTED, 50, 768, 200, 32)
    assert n > 0
    assert lib.miner_score_workspace_bytes(_lib.DTYPE_F32, _lib.SCORE_WEIGHTED, 50, 768, 200, 32) == 0
    assert lib.miner_score_workspace_bytes(_lib.DTYPE_BF16, _lib.SCORE_NONE, 50, 768, 200, 32) == 0


@pytest.mark.parametrize("d", [256, 512, 768])
@pytest.mark.parametrize("B", [1, 2, 3, 257, 1001])
def test_pair_equals_single_dense(d, B):
    imp = synthetic.impressions(7, 0, B, L=50, d=d, C=40, device=DEV, dtype=BF)
    W1, Q, W2 = _weights(d)
    _same(*_both(imp.history, imp.his_mask, imp.candidates, W1, Q, W2))


@pytest.mark.parametrize("score_type", ["weighted", "max", "mean"])
def test_pair_equals_single_ragged(score_type):
    """Ragged C_b in [0, 150]: empty impressions, one chunk, several 64-candidate chunks, and
    impressions too large to stage in LDS."""
    rng = np.random.default_rng(3)
    B, L, d = 301, 50, 768
    imp = synthetic.impressions(11, 0, B, L=L, d=d, C=40, device=DEV, dtype=BF)
    sizes = rng.integers(0, 151, B)
    sizes[:5] = [0, 1, 64, 65, 150]
    N = int(sizes.sum())
    cand = (torch.randn((N, d), device=DEV) / d ** 0.5).to(BF)
    offs = torch.zeros(B + 1, dtype=torch.int32, device=DEV)
    offs[1:] = torch.from_numpy(np.cumsum(sizes)).to(DEV)
    W1, Q, W2 = _weights(d)
    _same(*_both(imp.history, imp.his_mask, cand, W1, Q, W2 if score_type == "weighted" else None,
                 score_type=score_type, cand_offsets=offs))


def test_pair_equals_single_bias_and_user():
    B, L, d = 77, 50, 256
    imp = synthetic.impressions(5, 0, B, L=L, d=d, C=40, device=DEV, dtype=BF)
    bias = torch.rand((B, L), device=DEV) * 2 - 1
    W1, Q, W2 = _weights(d, Dc=200, K=32)
    _same(*_both(imp.history, imp.his_mask, imp.candidates, W1, Q, W2, his_bias=bias, return_user=True))


def test_pair_equals_single_short_history_small_K():
    """L <= 32 (one position tile) and K < 32 (padded interest rows)."""
    B, L, d = 64, 20, 512
    imp = synthetic.impressions(9, 0, B, L=L, d=d, C=5, device=DEV, dtype=BF)
    W1, Q, W2 = _weights(d, Dc=96, K=4)
    _same(*_both(imp.history, imp.his_mask, imp.candidates, W1, Q, W2, return_user=True))


def test_pair_mask_pointer_offsets():
    """A his_mask view at an odd byte offset: the mask words the DMA reads are realigned."""
    B, L, d = 33, 50, 768
    imp = synthetic.impressions(13, 0, B + 1, L=L, d=d, C=40, device=DEV, dtype=BF)
    mask = imp.his_mask[1:]            # storage offset L = 50 bytes: not 4-byte aligned
    assert mask.data_ptr() % 4 != 0
    W1, Q, W2 = _weights(d)
    _same(*_both(imp.history[1:], mask, imp.candidates[1:], W1, Q, W2))
