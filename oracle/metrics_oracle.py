"""ORACLE — test infrastructure only.

Restatement of the reference evaluator's metric arithmetic (src/evaluation.py) used as the checker
for ``miner_amd.evaluation``. Only ``tests/`` and ``bench.py``'s ``cpu_baseline`` leg import it.

The reference's global/per-impression AUC is scikit-learn's ``roc_auc_score``
(pinned scikit-learn 1.4.1.post1 in environment.yml:308; 1.7.2 is installed here). It is a
third-party dependency that is not vendored in the reference; its published algorithm (area under
the ROC curve, ties counted as one half) is called directly here.

Citations:
* ``compute_scores``      src/evaluation.py:36-84 (auc = flattened pairs :53-55, group metrics
                          nanmean over impressions :56-82)
* ``compute_mrr_score``   src/evaluation.py:177-192 (np.argsort descending, unstable on ties)
* ``compute_dcg_score``   src/evaluation.py:195-213
* ``compute_ndcg_score``  src/evaluation.py:216-231
* ``is_hit``              src/evaluation.py:245-249 (stable ``sorted``)
* ``_convert_targets/_convert_pred`` group by impression id, sorted by id: :118-149
"""
from __future__ import annotations

import functools
import operator

import numpy as np
from sklearn.metrics import roc_auc_score


def mrr(y_true: np.ndarray, y_score: np.ndarray) -> float:
    rank = np.argsort(y_score)[::-1]
    y_true = np.take(y_true, rank)
    rr = y_true / (np.arange(len(y_true)) + 1)
    return np.sum(rr) / np.sum(y_true)


def dcg(y_true: np.ndarray, y_score: np.ndarray, k: int) -> float:
    k = min(np.shape(y_true)[-1], k)
    order = np.argsort(y_score)[::-1]
    y_true = np.take(y_true, order[:k])
    gains = 2 ** y_true - 1
    discounts = np.log2(np.arange(len(y_true)) + 2)
    return np.sum(gains / discounts)


def ndcg(y_true: np.ndarray, y_score: np.ndarray, k: int) -> float:
    return dcg(y_true, y_score, k) / dcg(y_true, y_true, k)


def hit(y_true, y_score, k: int) -> int:
    ordered = sorted(zip(y_score, y_true), key=lambda x: x[0], reverse=True)
    return int(sum(label for _, label in ordered[:k]) > 0)


def group_by_impression(ids, values):
    """evaluation.py:135-149: concatenate per-id lists in arrival order, then sort by id."""
    groups: dict = {}
    for v, i in zip(values, ids):
        if not isinstance(v, list):
            v = [v]
        groups[i] = groups.get(i, []) + v
    return [g for _, g in sorted(groups.items())]


def compute_scores(targets, probs, metrics):
    """evaluation.py:36-84 on already-grouped per-impression lists."""
    assert len(targets) == len(probs)
    flat_t = functools.reduce(operator.iconcat, [list(t) for t in targets], [])
    flat_p = functools.reduce(operator.iconcat, [list(p) for p in probs], [])
    out = {}
    for metric in metrics:
        if metric == "auc":
            out["auc"] = roc_auc_score(y_true=flat_t, y_score=flat_p)
        elif metric == "group_auc":
            out["group_auc"] = np.nanmean([roc_auc_score(y_true=t, y_score=p)
                                           for t, p in zip(targets, probs)])
        elif metric == "mrr":
            out["mrr"] = np.nanmean([mrr(np.array(t), np.array(p)) for t, p in zip(targets, probs)])
        elif metric.startswith("ndcg"):
            k = int(metric.split("@")[1])
            out[f"ndcg@{k}"] = np.nanmean([ndcg(np.array(t), np.array(p), k)
                                           for t, p in zip(targets, probs)])
        elif metric.startswith("hit"):
            k = int(metric.split("@")[1])
            out[f"hit@{k}"] = np.nanmean([hit(np.array(t), np.array(p), k)
                                          for t, p in zip(targets, probs)])
    return out


def per_impression(targets, probs, metric):
    """The per-impression list the reference saves as <metric>.txt (evaluation.py:60-82)."""
    if metric == "group_auc":
        return [roc_auc_score(y_true=t, y_score=p) for t, p in zip(targets, probs)]
    if metric == "mrr":
        return [mrr(np.array(t), np.array(p)) for t, p in zip(targets, probs)]
    if metric.startswith("ndcg"):
        k = int(metric.split("@")[1])
        return [ndcg(np.array(t), np.array(p), k) for t, p in zip(targets, probs)]
    if metric.startswith("hit"):
        k = int(metric.split("@")[1])
        return [hit(np.array(t), np.array(p), k) for t, p in zip(targets, probs)]
    raise ValueError(metric)
