"""Drop-in mirror of the reference evaluator (src/evaluation.py) with vectorised metrics.

Same classes and contracts as the reference:

* ``SlowEvaluator(dataset)``: ``eval_batch(logits, impression_ids)`` appends
  ``sigmoid(logits)`` per sample (evaluation.py:151-170), ``compute_scores(metrics, save_result,
  path)`` groups the predictions by impression id, sorted by id (:118-149), and returns
  ``auc`` (global, flattened pairs :53-55), ``group_auc`` / ``mrr`` / ``ndcg@k`` / ``hit@k``
  (nanmean over impressions :56-82), writing the per-impression ``<metric>.txt`` files when asked;
  ``save_predictions(path)`` writes ``preds.pkl`` (:173-175).
* ``FastEvaluator`` (:87-110) and the metric functions ``compute_mrr_score`` (:177-192),
  ``compute_dcg_score`` (:195-213), ``compute_ndcg_score`` (:216-231) and ``is_hit`` (:245-249).

The metric arithmetic is vectorised over impressions (one lexsort of (impression, score) for the
whole set instead of a Python loop of sklearn calls: the reference's ~0.9 ms/impression metric step
is the bottleneck once scoring runs on the GPU). Ties follow the reference exactly: an impression
whose scores contain a tie between a clicked and a non-clicked candidate is re-ranked with the
reference's own ``np.argsort(...)[::-1]`` (mrr, ndcg) or stable ``sorted`` (hit@k) order.
AUC counts ties as one half, which is what scikit-learn's ``roc_auc_score`` computes.
"""
from __future__ import annotations

import os
import pickle
from typing import Optional, Dict, List, Sequence

import numpy as np
import torch
from torch import Tensor

# ---------------------------------------------------------------------------------------------
# reference metric functions (per impression)
# ---------------------------------------------------------------------------------------------


def compute_mrr_score(y_true: np.ndarray, y_score: np.ndarray):
    rank = np.argsort(y_score)[::-1]
    y_true = np.take(y_true, rank)
    rr_score = y_true / (np.arange(len(y_true)) + 1)
    return np.sum(rr_score) / np.sum(y_true)


def compute_dcg_score(y_true: np.ndarray, y_score: np.ndarray, k: int):
    k = min(np.shape(y_true)[-1], k)
    order = np.argsort(y_score)[::-1]
    y_true = np.take(y_true, order[:k])
    gains = 2 ** y_true - 1
    discounts = np.log2(np.arange(len(y_true)) + 2)
    return np.sum(gains / discounts)


def compute_ndcg_score(y_true: np.ndarray, y_score: np.ndarray, k: int):
    return compute_dcg_score(y_true, y_score, k) / compute_dcg_score(y_true, y_true, k)


def is_hit(y_true, y_score, k):
    ordered_pred = sorted(zip(y_score, y_true), key=lambda x: x[0], reverse=True)
    return int(sum(label for _, label in ordered_pred[:k]) > 0)


def auc_score(y_true, y_score) -> float:
    """Area under the ROC curve with ties counted one half (= sklearn roc_auc_score)."""
    y_true = np.asarray(y_true).astype(np.float64).ravel()
    y_score = np.asarray(y_score, dtype=np.float64).ravel()
    npos = y_true.sum()
    nneg = y_true.size - npos
    if npos == 0 or nneg == 0:
        return float("nan")
    order = np.argsort(y_score, kind="mergesort")
    s = y_score[order]
    # average rank of each tie group (1-based)
    starts = np.r_[0, np.flatnonzero(s[1:] != s[:-1]) + 1]
    ends = np.r_[starts[1:], s.size]
    avg = (starts + ends + 1) / 2.0
    ranks = np.repeat(avg, ends - starts)
    rank_pos = np.sum(ranks * y_true[order])
    return float((rank_pos - npos * (npos + 1) / 2.0) / (npos * nneg))


# ---------------------------------------------------------------------------------------------
# vectorised per-impression metrics
# ---------------------------------------------------------------------------------------------


class GroupedPairs:
    """Per-impression (label, score) lists flattened: group g owns rows [offs[g], offs[g+1])."""

    def __init__(self, labels: np.ndarray, scores: np.ndarray, offsets: np.ndarray):
        self.labels = np.asarray(labels, dtype=np.float64)
        self.scores = np.asarray(scores, dtype=np.float64)
        self.offsets = np.asarray(offsets, dtype=np.int64)
        self.G = self.offsets.size - 1
        self.sizes = np.diff(self.offsets)
        self.gid = np.repeat(np.arange(self.G), self.sizes)
        self._prepare()

    @classmethod
    def from_lists(cls, targets: Sequence[Sequence], probs: Sequence[Sequence]):
        sizes = np.fromiter((len(t) for t in targets), dtype=np.int64, count=len(targets))
        offs = np.zeros(len(targets) + 1, np.int64)
        offs[1:] = np.cumsum(sizes)
        lab = np.fromiter((x for t in targets for x in t), dtype=np.float64, count=int(offs[-1]))
        sc = np.fromiter((x for p in probs for x in p), dtype=np.float64, count=int(offs[-1]))
        return cls(lab, sc, offs)

    def _prepare(self):
        n = self.scores.size
        # descending score within group, ties by position (stable)
        pos = np.arange(n)
        order = np.lexsort((pos, -self.scores, self.gid))
        self.order = order
        s_sorted = self.scores[order]
        g_sorted = self.gid[order]
        same = np.zeros(n, bool)
        if n > 1:
            same[1:] = (s_sorted[1:] == s_sorted[:-1]) & (g_sorted[1:] == g_sorted[:-1])
        # rank (0-based) within group of each sorted element
        self.rank_sorted = pos - self.offsets[g_sorted]
        self.lab_sorted = self.labels[order]
        self.g_sorted = g_sorted
        # groups whose order among equal scores changes a label-dependent metric
        tie_groups = np.zeros(self.G, bool)
        if same.any():
            idx = np.flatnonzero(same)
            differing = self.lab_sorted[idx] != self.lab_sorted[idx - 1]
            # a tie run mixing labels: mark its group
            runs_start = np.flatnonzero(~same)
            run_id = np.cumsum(~same) - 1
            run_min = np.full(runs_start.size, np.inf)
            run_max = np.full(runs_start.size, -np.inf)
            np.minimum.at(run_min, run_id, self.lab_sorted)
            np.maximum.at(run_max, run_id, self.lab_sorted)
            mixed_run = run_min != run_max
            tie_groups[np.unique(g_sorted[runs_start[mixed_run]])] = True
            del differing
        self.tie_groups = tie_groups
        self.npos = np.bincount(self.gid, weights=self.labels, minlength=self.G)

    def _fix_ties(self, out: np.ndarray, fn) -> np.ndarray:
        for g in np.flatnonzero(self.tie_groups):
            lo, hi = self.offsets[g], self.offsets[g + 1]
            out[g] = fn(self.labels[lo:hi], self.scores[lo:hi])
        return out

    def group_auc(self) -> np.ndarray:
        n = self.scores.size
        # ascending by score within group for average ranks
        pos = np.arange(n)
        order = np.lexsort((self.scores, self.gid))
        s = self.scores[order]
        g = self.gid[order]
        lab = self.labels[order]
        newrun = np.ones(n, bool)
        if n > 1:
            newrun[1:] = (s[1:] != s[:-1]) | (g[1:] != g[:-1])
        starts = np.flatnonzero(newrun)
        ends = np.r_[starts[1:], n]
        rank0 = pos - self.offsets[g]
        avg = (rank0[starts] + (rank0[ends - 1]) + 2) / 2.0
        ranks = np.repeat(avg, ends - starts)
        rank_pos = np.bincount(g, weights=ranks * lab, minlength=self.G)
        npos = self.npos
        nneg = self.sizes - npos
        with np.errstate(invalid="ignore", divide="ignore"):
            auc = (rank_pos - npos * (npos + 1) / 2.0) / (npos * nneg)
        auc[(npos == 0) | (nneg == 0)] = np.nan
        return auc

    def mrr(self) -> np.ndarray:
        rr = self.lab_sorted / (self.rank_sorted + 1)
        with np.errstate(invalid="ignore", divide="ignore"):
            out = np.bincount(self.g_sorted, weights=rr, minlength=self.G) / self.npos
        return self._fix_ties(out, lambda t, p: compute_mrr_score(t, p))

    def ndcg(self, k: int) -> np.ndarray:
        disc = np.log2(self.rank_sorted + 2.0)
        top = self.rank_sorted < k
        gains = (2.0 ** self.lab_sorted - 1.0) / disc
        actual = np.bincount(self.g_sorted, weights=np.where(top, gains, 0.0), minlength=self.G)
        # ideal: labels sorted descending within group
        order = np.lexsort((-self.labels, self.gid))
        lab_ideal = self.labels[order]
        rank_ideal = np.arange(self.labels.size) - self.offsets[self.gid[order]]
        ideal = np.bincount(self.gid[order], weights=np.where(rank_ideal < k, (2.0 ** lab_ideal - 1.0) /
                                                                   np.log2(rank_ideal + 2.0), 0.0),
                            minlength=self.G)
        with np.errstate(invalid="ignore", divide="ignore"):
            out = actual / ideal
        return self._fix_ties(out, lambda t, p: compute_ndcg_score(t, p, k))

    def hit(self, k: int) -> np.ndarray:
        top = self.rank_sorted < k
        out = (np.bincount(self.g_sorted, weights=np.where(top, self.lab_sorted, 0.0), minlength=self.G) > 0)
        return out.astype(np.float64)   # stable order on ties == the reference's sorted(): no fix needed

    def per_impression(self, metric: str) -> np.ndarray:
        if metric == "group_auc":
            return self.group_auc()
        if metric == "mrr":
            return self.mrr()
        if metric.startswith("ndcg"):
            return self.ndcg(int(metric.split("@")[1]))
        if metric.startswith("hit"):
            return self.hit(int(metric.split("@")[1]))
        raise ValueError(f"unknown metric {metric}")


def metric_key(metric: str) -> str:
    if metric.startswith("ndcg") or metric.startswith("hit"):
        name, k = metric.split("@")
        return f"{name}@{int(k)}"
    return metric


def metric_file(metric: str) -> str:
    return {"group_auc": "group_auc.txt", "mrr": "mrr.txt"}.get(metric, metric.replace("@", "") + ".txt")


def save_scores(path, scores):
    with open(path, mode="w", encoding="utf-8") as f:
        for score in scores:
            f.write(str(score))
            f.write("\n")


def compute_metrics(pairs: GroupedPairs, metrics: List[str], save_result: bool = False,
                    path: str = None) -> Dict[str, float]:
    """evaluation.py:36-84 over GroupedPairs."""
    scores = {}
    for metric in metrics:
        if metric == "auc":
            scores["auc"] = auc_score(pairs.labels, pairs.scores)
            continue
        vals = pairs.per_impression(metric)
        scores[metric_key(metric)] = float(np.nanmean(vals))
        if save_result:
            out = vals.astype(int) if metric.startswith("hit") else vals
            save_scores(os.path.join(path, metric_file(metric)), out.tolist())
    return scores


# ---------------------------------------------------------------------------------------------
# evaluation loss on the batched layout
# ---------------------------------------------------------------------------------------------


def disagreement(mui: Tensor) -> Tensor:
    """Per-impression mean pairwise cosine of the K interests, diagonal zeroed -> [B] fp32
    (the ``pairwise_cosine_similarity(poly_attn, poly_attn, zero_diagonal=True)`` term of
    src/loss.py:81; src/utils.py:9-29)."""
    u = mui / torch.linalg.norm(mui, dim=2, keepdim=True)
    g = torch.matmul(u, u.transpose(1, 2))
    g.diagonal(dim1=1, dim2=2).zero_()
    return g.mean(dim=(1, 2))


def eval_loss_partials(mui: Optional[Tensor], scores: Tensor, labels: Tensor, *, first_sample: int,
                       total_samples: int, cand_offsets: Tensor = None, batch_size: int = 32,
                       dis: Optional[Tensor] = None) -> Tensor:
    """Numerator and positive count of the reference eval loss for a contiguous run of impressions.

    The reference evaluates one sample per (impression, candidate), impression-major, in batches
    of ``eval_batch_size`` (src/reader.py:376-379, config/eval_miner.txt:19) and sums
    ``Loss.compute_eval_loss`` per batch (src/loss.py:68-85, src/trainer.py:276-291), so the batch
    partition matters (a per-batch *mean* of the disagreement). Sample s (global index) lies in
    batch s // batch_size of size n_b = min(batch_size, total - batch_size·(s // batch_size)); the
    numerator is Σ_s D(imp(s)) / n_b(s) + Σ_s -logsigmoid(score_s)·label_s. Both sums decompose
    over impression ranges, so ranks add their partials (``first_sample`` = the global index of
    this run's first sample). Returns a float64 tensor [numerator, positives]; the loss is
    numerator / positives. ``dis`` [B]: the per-impression disagreement already formed (the news
    kernel's fused epilogue, news.score(disagreement=True)); else it is computed from ``mui``.
    """
    dev = scores.device
    if cand_offsets is None:
        B, C = scores.shape
        sizes = torch.full((B,), C, device=dev, dtype=torch.int64)
    else:
        sizes = torch.diff(cand_offsets.to(dev, torch.int64))
    s = scores.reshape(-1).double()
    lab = labels.reshape(-1).to(dev).double()
    D = torch.repeat_interleave((dis if dis is not None else disagreement(mui.float())).double(), sizes)
    idx = first_sample + torch.arange(s.numel(), device=dev, dtype=torch.int64)
    bstart = (idx // batch_size) * batch_size
    nb = torch.clamp(total_samples - bstart, max=batch_size).double()
    num = (D / nb).sum() + (-torch.nn.functional.logsigmoid(s) * lab).sum()
    return torch.stack([num, lab.sum()])


def eval_loss(mui: Tensor, scores: Tensor, labels: Tensor, cand_offsets: Tensor = None,
              batch_size: int = 32) -> float:
    """Single-process eval loss (src/trainer.py:291: total_loss / total_pos_example)."""
    n = scores.numel()
    p = eval_loss_partials(mui, scores, labels, first_sample=0, total_samples=n, cand_offsets=cand_offsets,
                           batch_size=batch_size)
    return float(p[0] / p[1])


# ---------------------------------------------------------------------------------------------
# evaluator classes (reference contract)
# ---------------------------------------------------------------------------------------------


class BaseEvaluator:
    def __init__(self, dataset):
        self.dataset = dataset
        self.prob_predictions = []
        self.targets = []
        self._convert_targets()

    def _convert_targets(self):
        raise NotImplementedError

    def _convert_pred(self):
        raise NotImplementedError

    def eval_batch(self, logits: Tensor, impression_ids: Tensor):
        raise NotImplementedError

    def compute_scores(self, metrics: List[str], save_result: bool, path: str = None):
        self._convert_pred()
        assert len(self.targets) == len(self.prob_predictions)
        pairs = GroupedPairs.from_lists(self.targets, self.prob_predictions)
        return compute_metrics(pairs, metrics, save_result, path)


class FastEvaluator(BaseEvaluator):
    """evaluation.py:87-110: softmax over the npratio+1 logits of each sample."""

    def _convert_targets(self):
        for sample in self.dataset.samples:
            self.targets.append(sample.impression.label)

    def _convert_pred(self):
        pass

    def eval_batch(self, logits: Tensor, impression_ids: Tensor):
        probs = torch.softmax(logits, dim=1)
        self.prob_predictions.extend(probs.tolist())


class SlowEvaluator(BaseEvaluator):
    """evaluation.py:113-175: per-candidate sigmoid probabilities grouped by impression id."""

    def __init__(self, dataset):
        super().__init__(dataset)
        self.impression_ids = []

    def _convert_targets(self):
        groups = {}
        for sample in self.dataset.samples:
            iid = sample.impression.impression_id
            groups.setdefault(iid, []).extend(sample.impression.label)
        self.targets = [v for _, v in sorted(groups.items())]

    def _convert_pred(self):
        groups = {}
        for prob, iid in zip(self.prob_predictions, self.impression_ids):
            if not isinstance(prob, list):
                prob = [prob]
            groups.setdefault(iid, []).extend(prob)
        self.prob_predictions = [v for _, v in sorted(groups.items())]

    def eval_batch(self, logits: Tensor, impression_ids: Tensor):
        probs = torch.sigmoid(logits)
        self.prob_predictions.extend(probs.tolist())
        self.impression_ids.extend(impression_ids.tolist())

    def save_predictions(self, path: str):
        pred_dict = {'pred': self.prob_predictions, 'impression_id': self.impression_ids}
        with open(os.path.join(path, 'preds.pkl'), 'wb') as f:
            pickle.dump(pred_dict, f)


class ArrayEvaluator:
    """Batched-layout evaluator: one row of C candidates per impression, no Python lists.

    ``add(scores, labels, impression_ids, cand_offsets=None)`` takes device or host tensors of a
    batch (dense [B,C] or ragged [N] + offsets); ``pairs()`` returns GroupedPairs sorted by id.
    Metrics equal SlowEvaluator's on the per-candidate layout of the same impressions.
    """

    def __init__(self):
        self._ids, self._probs, self._labels, self._sizes = [], [], [], []

    def add(self, scores: Tensor, labels: Tensor, impression_ids: Tensor, cand_offsets: Tensor = None):
        probs = torch.sigmoid(scores.float()).reshape(-1).cpu().numpy()
        lab = labels.reshape(-1).cpu().numpy()
        if cand_offsets is None:
            sizes = np.full(scores.shape[0], scores.shape[1], np.int64)
        else:
            sizes = np.diff(cand_offsets.cpu().numpy().astype(np.int64))
        self._ids.append(impression_ids.reshape(-1).cpu().numpy().astype(np.int64))
        self._probs.append(probs)
        self._labels.append(lab)
        self._sizes.append(sizes)

    def arrays(self):
        ids = np.concatenate(self._ids) if self._ids else np.zeros(0, np.int64)
        probs = np.concatenate(self._probs) if self._probs else np.zeros(0)
        lab = np.concatenate(self._labels) if self._labels else np.zeros(0)
        sizes = np.concatenate(self._sizes) if self._sizes else np.zeros(0, np.int64)
        return ids, probs, lab, sizes

    def pairs(self) -> GroupedPairs:
        ids, probs, lab, sizes = self.arrays()
        offs = np.zeros(sizes.size + 1, np.int64)
        offs[1:] = np.cumsum(sizes)
        order = np.argsort(ids, kind="stable")
        if np.any(order != np.arange(order.size)):
            idx = np.concatenate([np.arange(offs[i], offs[i + 1]) for i in order]) if order.size else order
            sizes = sizes[order]
            probs, lab = probs[idx], lab[idx]
            offs[1:] = np.cumsum(sizes)
        return GroupedPairs(lab, probs, offs)

    def compute_scores(self, metrics: List[str], save_result: bool = False, path: str = None):
        return compute_metrics(self.pairs(), metrics, save_result, path)
