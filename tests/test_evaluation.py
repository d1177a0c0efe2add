"""miner_amd.evaluation (the drop-in evaluator) against the reference's golden metrics and the
metrics oracle. CPU only."""
import os
import tempfile
import types

import numpy as np
import pytest
import torch

from miner_amd import evaluation as ev
from oracle import metrics_oracle as mo

from test_oracle_golden import METRICS, PER_IMP


def _dataset(labels):
    """Minimal stand-in for src.entities.Dataset in the reference's per-candidate eval layout:
    one sample per (impression, candidate), impression-major (reader.py:376-379)."""
    samples = []
    for i, row in enumerate(labels):
        for lab in row:
            imp = types.SimpleNamespace(impression_id=i, label=[int(lab)])
            samples.append(types.SimpleNamespace(impression=imp))
    return types.SimpleNamespace(samples=samples)


def test_grouped_pairs_match_reference_metrics(golden):
    g = golden
    offs = np.arange(g["B"] + 1) * g["C"]
    pairs = ev.GroupedPairs(g["labels"].reshape(-1), g["probs_grouped"].reshape(-1), offs)
    with tempfile.TemporaryDirectory() as td:
        got = ev.compute_metrics(pairs, METRICS, True, td)
        for m, key in PER_IMP.items():
            np.testing.assert_allclose(np.loadtxt(os.path.join(td, ev.metric_file(m)), ndmin=1), g[key],
                                       atol=1e-12, equal_nan=True)
    for k, v in g["metrics"].items():
        assert got[k] == pytest.approx(v, abs=1e-12), k


def test_slow_evaluator_contract(golden):
    """eval_batch(logits [32,1], impression_ids) in eval_batch_size batches, then compute_scores."""
    g = golden
    ds = _dataset(g["labels"])
    e = ev.SlowEvaluator(ds)
    logits = torch.from_numpy(g["scores_per_candidate"]).reshape(-1, 1)
    ids = torch.arange(g["B"]).repeat_interleave(g["C"])
    for i in range(0, logits.shape[0], 32):
        e.eval_batch(logits[i:i + 32], ids[i:i + 32])
    with tempfile.TemporaryDirectory() as td:
        e.save_predictions(td)
        assert os.path.getsize(os.path.join(td, "preds.pkl")) > 0
        got = e.compute_scores(METRICS, False, td)
    for k, v in g["metrics"].items():
        assert got[k] == pytest.approx(v, abs=1e-12), k


def test_array_evaluator_batched_layout_any_order(golden):
    """Batched [B,C] scores in shuffled batches: grouping by impression id restores the order."""
    g = golden
    rng = np.random.default_rng(0)
    perm = rng.permutation(g["B"])
    a = ev.ArrayEvaluator()
    s = torch.from_numpy(g["scores_per_candidate"])
    lab = torch.from_numpy(g["labels"])
    for chunk in np.array_split(perm, 3):
        idx = torch.from_numpy(chunk)
        a.add(s[idx], lab[idx], idx)
    got = a.compute_scores(METRICS)
    for k, v in g["metrics"].items():
        assert got[k] == pytest.approx(v, abs=1e-9), k


def test_eval_loss_batched_layout(golden):
    g = golden
    if g["use_bias"]:
        pytest.skip("with category bias the per-candidate mui differs from the batched one")
    mui = torch.from_numpy(g["mui"])
    got = ev.eval_loss(mui, torch.from_numpy(g["scores_per_candidate"]), torch.from_numpy(g["labels"]))
    assert got == pytest.approx(float(g["eval_loss"]), rel=1e-6)


def test_eval_loss_ragged_equals_dense(golden):
    g = golden
    B, C = g["B"], g["C"]
    mui = torch.from_numpy(g["mui"])
    s = torch.from_numpy(g["scores_per_candidate"])
    lab = torch.from_numpy(g["labels"])
    offs = torch.arange(B + 1, dtype=torch.int32) * C
    a = ev.eval_loss(mui, s, lab)
    b = ev.eval_loss(mui, s.reshape(-1), lab.reshape(-1), cand_offsets=offs)
    assert a == pytest.approx(b, rel=1e-12)


@pytest.mark.parametrize("seed", range(6))
def test_random_ties_and_ragged_vs_oracle(seed):
    """Heavy ties (quantised scores), ragged impressions, single-label impressions (NaN AUC)."""
    rng = np.random.default_rng(seed)
    G = 300
    sizes = rng.integers(1, 12, G)
    targets, probs = [], []
    for n in sizes:
        t = (rng.random(n) < 0.3).astype(np.int64)
        p = np.round(rng.random(n) * 4) / 4           # 5 distinct values: many ties
        targets.append(list(t))
        probs.append(list(p))
    # the global auc needs both classes
    targets[0][0] = 1
    targets[1][0] = 0
    metrics = ["auc", "group_auc", "mrr", "ndcg@3", "ndcg@10", "hit@1", "hit@5"]
    with np.errstate(all="ignore"):
        want = mo.compute_scores(targets, probs, metrics)
        got = ev.compute_metrics(ev.GroupedPairs.from_lists(targets, probs), metrics)
        for m in metrics[1:]:
            np.testing.assert_allclose(ev.GroupedPairs.from_lists(targets, probs).per_impression(m),
                                       mo.per_impression(targets, probs, m), atol=1e-12, equal_nan=True)
    for k in want:
        if np.isnan(want[k]):
            assert np.isnan(got[k]), k
        else:
            assert got[k] == pytest.approx(want[k], abs=1e-12), k


def test_reference_metric_functions():
    y = np.array([0, 1, 0, 1, 0])
    s = np.array([0.1, 0.9, 0.3, 0.2, 0.8])
    assert ev.compute_mrr_score(y, s) == pytest.approx(mo.mrr(y, s))
    assert ev.compute_ndcg_score(y, s, 3) == pytest.approx(mo.ndcg(y, s, 3))
    assert ev.is_hit(y, s, 1) == mo.hit(y, s, 1) == 1
    assert ev.auc_score(y, s) == pytest.approx(4 / 6)


def test_row_batched_tie_order_equals_reference_calls():
    """miner_amd.metrics recomputes mixed-label ties for many impressions at once (np.argsort along
    rows); every row must equal the reference formulas called one impression at a time."""
    from miner_amd import metrics as gm
    rng = np.random.default_rng(3)
    for c in (2, 5, 16, 17, 40, 97):
        S = rng.integers(0, 4, size=(300, c)).astype(np.float64) / 4     # heavy ties
        Y = rng.integers(0, 2, size=(300, c)).astype(np.int64)
        Y[:, 0], Y[:, 1] = 1, 0
        mrr = gm.mrr_rows(Y, S)
        for k in (5, 10):
            nd = gm.ndcg_rows(Y, S, k)
            for r in range(S.shape[0]):
                assert nd[r] == ev.compute_ndcg_score(Y[r], S[r], k)
        for r in range(S.shape[0]):
            assert mrr[r] == ev.compute_mrr_score(Y[r], S[r])
