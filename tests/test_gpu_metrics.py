"""GPU per-impression metrics (miner_impression_metrics) against the reference's golden metric
files and the metrics oracle — needs an MI355X."""
import numpy as np
import pytest
import torch

from miner_amd import metrics as gm
from oracle import metrics_oracle as mo
from tests.conftest import golden_names, load_golden

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
METRICS = ["auc", "group_auc", "mrr", "ndcg@5", "ndcg@10", "hit@5", "hit@10"]
PER_IMP = {"group_auc": "per_imp_group_auc", "mrr": "per_imp_mrr", "ndcg@5": "per_imp_ndcg5",
           "ndcg@10": "per_imp_ndcg10", "hit@5": "per_imp_hit5", "hit@10": "per_imp_hit10"}


def _csr(targets, probs):
    sizes = [len(t) for t in targets]
    offs = np.zeros(len(sizes) + 1, np.int32)
    offs[1:] = np.cumsum(sizes)
    p = torch.tensor(np.concatenate([np.asarray(x, np.float32) for x in probs]), device=DEV)
    y = torch.tensor(np.concatenate([np.asarray(x, np.uint8) for x in targets]), device=DEV)
    return p, y, torch.tensor(offs, device=DEV)


@pytest.mark.parametrize("name", golden_names())
def test_matches_reference_golden(name):
    g = load_golden(name)
    # the reference ranks fp32 sigmoid values (stored as float64): exactly representable in fp32
    probs = g["probs_grouped"].astype(np.float32)
    assert np.array_equal(probs.astype(np.float64), g["probs_grouped"])
    p, y, o = _csr(list(g["labels"]), list(probs))
    per = gm.per_impression(p, y, o, METRICS[1:])
    for m, key in PER_IMP.items():
        np.testing.assert_allclose(per[m], g[key], atol=1e-12, equal_nan=True, err_msg=m)
    got = gm.compute_metrics(p, y, o, METRICS)
    for k, v in g["metrics"].items():
        assert got[k] == pytest.approx(v, abs=1e-12), k


@pytest.mark.parametrize("seed", range(5))
def test_ragged_ties_vs_oracle(seed):
    """Heavy ties (including mixed-label ties: host fix path), sizes 1..300, single-class impressions."""
    rng = np.random.default_rng(seed)
    G = 500
    sizes = rng.integers(1, 301, G)
    sizes[:3] = [1, 2, 300]
    targets, probs = [], []
    for n in sizes:
        targets.append(list((rng.random(n) < 0.25).astype(np.int64)))
        q = 4 if seed % 2 == 0 else 1000
        probs.append(list((np.round(rng.random(n) * q) / q).astype(np.float32).astype(np.float64)))
    targets[0][0] = 1
    targets[1][0] = 0
    metrics = ["group_auc", "mrr", "ndcg@3", "ndcg@10", "hit@1", "hit@5"]
    p, y, o = _csr(targets, probs)
    per = gm.per_impression(p, y, o, metrics)
    with np.errstate(all="ignore"):
        for m in metrics:
            np.testing.assert_allclose(per[m], mo.per_impression(targets, probs, m), atol=1e-12,
                                       equal_nan=True, err_msg=m)


def test_device_evaluator_matches_reference(tmp_path):
    g = load_golden("cfg1_demo")
    ev = gm.DeviceEvaluator()
    logits = torch.tensor(g["scores_per_candidate"], device=DEV)
    lab = torch.tensor(g["labels"], device=DEV)
    ids = torch.arange(g["B"], device=DEV)
    perm = torch.randperm(g["B"], device=DEV)
    for chunk in torch.chunk(perm, 3):
        ev.add(logits[chunk], lab[chunk], ids[chunk])
    got = ev.compute_scores(METRICS, True, str(tmp_path))
    for k, v in g["metrics"].items():
        assert got[k] == pytest.approx(v, abs=1e-9), k
    np.testing.assert_allclose(np.loadtxt(tmp_path / "mrr.txt", ndmin=1), g["per_imp_mrr"], atol=1e-9)


def test_throughput_many_impressions():
    """100k impressions x 40 candidates: one launch, no host loop."""
    G, C = 100_000, 40
    p = torch.rand(G * C, device=DEV)
    y = (torch.rand(G * C, device=DEV) < 0.1).to(torch.uint8)
    o = torch.arange(0, G * C + 1, C, device=DEV, dtype=torch.int32)
    per = gm.per_impression(p, y, o, ["group_auc", "mrr", "ndcg@10", "hit@5"])
    assert per["mrr"].shape == (G,)
