"""MIND tsv reader / artifacts against the reference's own reader on a tiny dataset
(tests/golden/reader_mind.npz, made by tests/golden/make_reader_golden.py). CPU only."""
import os
import pickle

import numpy as np
import pytest
import torch

from miner_amd import formats, model

HERE = os.path.dirname(os.path.abspath(__file__))
TINY = os.path.join(HERE, "golden", "mind_tiny")


def _read():
    cat = formats.read_category2id(os.path.join(TINY, "category2id.json"))
    news = formats.read_news_tsv(os.path.join(TINY, "news.tsv"), cat)
    g = np.load(os.path.join(HERE, "golden", "reader_mind.npz"))
    beh = formats.read_behaviors_tsv(os.path.join(TINY, "behaviors.tsv"), news, int(g["his_length"]))
    return news, beh, g


def test_reader_matches_reference_reader():
    news, beh, g = _read()
    # the reference yields one sample per (impression, candidate), impression-major
    offs = beh.cand_offsets.numpy()
    sizes = np.diff(offs)
    imp = np.repeat(beh.impression_ids.numpy(), sizes)
    np.testing.assert_array_equal(imp, g["impression_id"])
    np.testing.assert_array_equal(np.repeat(beh.his_ids.numpy(), sizes, axis=0), g["his_rows"])
    np.testing.assert_array_equal(np.repeat(beh.his_mask.numpy(), sizes, axis=0), g["his_mask"])
    np.testing.assert_array_equal(beh.cand_ids.numpy(), g["cand_row"])
    np.testing.assert_array_equal(beh.labels.numpy(), g["label"])


def test_reader_edge_cases():
    news, beh, _ = _read()
    assert news.n_rows == 13 and news.row["N1"] == 1
    assert news.category[news.row["N6"]] == 1          # unseen category -> 'unk'
    assert beh.impression_ids.tolist() == [0, 1, 2, 5, 6]   # lines 3 and 4 lack a click / non-click
    assert beh.his_ids[1].tolist() == [0] * 6               # empty history: all pad
    assert not beh.his_mask[1].any()
    assert beh.his_ids[2].tolist() == [1, 2, 3, 4, 5, 6]    # the OLDEST his_length clicks


def test_preds_pkl_matches_slow_evaluator_format(tmp_path):
    news, beh, _ = _read()
    probs = torch.rand(beh.cand_ids.numel())
    out = formats.save_predictions(str(tmp_path), probs, beh.impression_ids, beh.cand_offsets)
    with open(out, "rb") as f:
        d = pickle.load(f)   # our own file
    assert set(d) == {"pred", "impression_id"}
    assert len(d["pred"]) == len(d["impression_id"]) == beh.cand_ids.numel()
    assert all(isinstance(p, list) and len(p) == 1 for p in d["pred"])
    assert d["impression_id"][:3] == [0, 0, 0]


def test_news_table_loaders(tmp_path):
    t = torch.randn(13, 8)
    np.save(tmp_path / "t.npy", t.numpy())
    torch.save({"news": t}, tmp_path / "t.pt")
    from safetensors.torch import save_file
    save_file({"news": t}, str(tmp_path / "t.safetensors"))
    for p in ("t.npy", "t.pt", "t.safetensors"):
        assert torch.equal(formats.load_news_table(str(tmp_path / p), key="news" if p != "t.npy" else None), t)


def test_state_dict_round_trip(tmp_path):
    class Enc(torch.nn.Module):
        embed_dim = 64

    a = model.Miner(Enc(), False, 4, 32, "weighted", 0.0)
    b = model.Miner(Enc(), False, 4, 32, "weighted", 0.0)
    torch.save(a.state_dict(), tmp_path / "sd.pt")
    formats.load_miner_state_dict(b, str(tmp_path / "sd.pt"))
    for (ka, va), (kb, vb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert ka == kb and torch.equal(va, vb)
    assert set(a.state_dict()) == {"poly_attn.linear.weight", "poly_attn.context_codes", "target_aware_attn.linear.weight"}


def test_preds_pickle_stream_equals_pickle_dump():
    """The numpy-built preds.pkl stream loads to exactly what pickle.dump of the reference's structure
    (SlowEvaluator.save_predictions, evaluation.py:173-175) loads to, including empty input."""
    import pickle
    rng = np.random.default_rng(0)
    for n in (0, 1, 7, 1000):
        p = rng.random(n).astype(np.float32)
        p[: min(n, 2)] = [np.float32(0.5), np.float32(1e-38)][: min(n, 2)]
        ids = rng.integers(0, 2 ** 31 - 1, n).astype(np.int64)
        got = pickle.loads(formats.preds_pickle(p, ids))
        want = {"pred": [[float(x)] for x in p.tolist()], "impression_id": ids.tolist()}
        assert got == want
        assert all(type(v[0]) is float for v in got["pred"])
