"""Pin the full-corpus oracle (oracle/corpus_oracle.py) to the reference's own Miner scoring a
whole news table (tests/golden/corpus_*.npz, made by tests/golden/make_corpus_golden.py). CPU."""
import glob
import os

import numpy as np
import pytest
import torch

from oracle import corpus_oracle as co
from oracle import miner_oracle as orc

HERE = os.path.dirname(os.path.abspath(__file__))
NAMES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(HERE, "golden", "corpus_*.npz")))


def load_corpus(name):
    z = np.load(os.path.join(HERE, "golden", name + ".npz"), allow_pickle=False)
    g = {k: z[k] for k in z.files}
    g["score_type"] = str(g["score_type"])
    for k in ("U", "L", "K", "Dc", "d", "N"):
        g[k] = int(g[k])
    return g


@pytest.mark.parametrize("name", NAMES)
def test_oracle_matches_reference(name):
    g = load_corpus(name)
    t = torch.from_numpy
    E = t(g["table"])[t(g["his_ids"])]
    mui, proj = co.encode(E, t(g["his_mask"]), t(g["W1"]), t(g["Q"]), t(g["W2"]) if "W2" in g else None)
    assert orc.parity_ok(mui.numpy(), g["mui"])[0]
    s = co.corpus_scores(mui, proj, t(g["table"]), g["score_type"])
    ok, worst = orc.parity_ok(s.numpy(), g["scores"])
    assert ok, worst


def test_topk_order_and_ties():
    s = np.array([[0.5, 0.9, 0.5, -1.0, 0.9]])
    ts, ti = co.topk(s, 4)
    assert ti.tolist() == [[1, 4, 0, 2]]
    ts, ti = co.topk(s, 7)
    assert ti[0, 5:].tolist() == [-1, -1] and np.isinf(ts[0, 6])
