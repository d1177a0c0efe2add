"""Synthetic MIND-shaped impressions: impression i depends only on (seed, i), so any
sharding over ranks sees the same data; reader-faithful padding and labels. CPU only."""
import pytest
import torch

from miner_amd import distributed as mdist
from miner_amd import synthetic


@pytest.mark.parametrize("ragged", [None, (2, 78)])
def test_shards_concatenate_to_the_whole(ragged):
    kw = dict(L=12, d=32, C=6, ragged=ragged)
    whole = synthetic.impressions(36, 0, 700, **kw)
    for ws in (2, 3, 8):
        parts = [synthetic.impressions(36, *mdist.shard_range(700, r, ws), **kw) for r in range(ws)]
        assert torch.equal(torch.cat([p.history for p in parts]), whole.history)
        assert torch.equal(torch.cat([p.his_mask for p in parts]), whole.his_mask)
        assert torch.equal(torch.cat([p.labels.reshape(-1) for p in parts]), whole.labels.reshape(-1))
        assert torch.equal(torch.cat([p.candidates.reshape(-1, 32) for p in parts]), whole.candidates.reshape(-1, 32))
        assert torch.equal(torch.cat([p.impression_ids for p in parts]), whole.impression_ids)


def test_reader_faithful_layout():
    imp = synthetic.impressions(7, 100, 300, L=20, d=16, C=5, ragged=(2, 9))
    pad = synthetic.pad_news(7, 16, "cpu")
    m = imp.his_mask
    # left padding: once a row turns real it stays real (reader.py:369, entities.py:395)
    assert torch.all(m[:, 1:] >= m[:, :-1])
    assert torch.equal(imp.history[~m], pad.expand(int((~m).sum()), 16))
    offs = imp.cand_offsets.long()
    assert int(offs[-1]) == imp.candidates.shape[0]
    for b in range(imp.n):
        lab = imp.labels[offs[b]:offs[b + 1]]
        assert 2 <= lab.numel() <= 9
        assert lab.max() == 1 and lab.min() == 0      # reader.py:374 keeps only mixed impressions


def test_init_weights_follow_reference_initialisers():
    W1, Q, W2 = synthetic.init_weights(36, 768, 200, 32)
    assert W1.shape == (200, 768) and Q.shape == (32, 200) and W2.shape == (768, 768)
    assert W1.abs().max() <= 768 ** -0.5 and W2.abs().max() <= 768 ** -0.5
    bound = 5 / 3 * (6 / (200 + 32)) ** 0.5
    assert Q.abs().max() <= bound and Q.abs().max() > 0.9 * bound
