"""GPU per-impression ranking metrics, behind the reference evaluator contract.

``per_impression`` runs ``miner_impression_metrics`` (include/miner_metrics.h) over impressions in
CSR layout: group AUC, MRR, nDCG@k and hit@k of every impression in one kernel. The reference's
only order-dependent case — MRR / nDCG of an impression where a tie mixes a click and a non-click,
ranked by numpy's ``argsort`` (src/evaluation.py:188, :208) — is flagged by the kernel and
recomputed here on the host with the reference functions, so results equal the reference's.

``compute_metrics`` returns the reference's metric dict (src/evaluation.py:36-84): the per-impression
metrics nan-averaged, and the flattened global ``auc`` (:53-55) over all pairs. ``DeviceEvaluator``
keeps (probability, label) on the device batch by batch; its ``compute_scores`` is the reference's
``compute_scores`` and, under torch.distributed, reduces over ranks (miner_amd.distributed).
"""
from __future__ import annotations

import os
from typing import Dict, List, Sequence

import numpy as np
import torch
from torch import Tensor

from . import _lib, evaluation


def _ks(metrics: Sequence[str]) -> List[int]:
    return sorted({int(m.split("@")[1]) for m in metrics if m.startswith(("ndcg@", "hit@"))})


def _dcg_rows(Y: np.ndarray, S: np.ndarray, k: int) -> np.ndarray:
    """compute_dcg_score (evaluation.py:195-231) of every row of S / Y at once: np.argsort along the
    rows sorts each row exactly as the 1-D call does (tests/test_evaluation.py pins this)."""
    kk = min(Y.shape[1], k)
    yt = np.take_along_axis(Y, np.argsort(S, axis=1)[:, ::-1][:, :kk], axis=1)
    gains = 2 ** yt - 1
    discounts = np.log2(np.arange(kk) + 2)
    return np.sum(gains / discounts, axis=1)


def ndcg_rows(Y: np.ndarray, S: np.ndarray, k: int) -> np.ndarray:
    return _dcg_rows(Y, S, k) / _dcg_rows(Y, Y, k)


def mrr_rows(Y: np.ndarray, S: np.ndarray) -> np.ndarray:
    """compute_mrr_score (evaluation.py:177-192) of every row at once."""
    yt = np.take_along_axis(Y, np.argsort(S, axis=1)[:, ::-1], axis=1)
    return np.sum(yt / (np.arange(Y.shape[1]) + 1), axis=1) / np.sum(yt, axis=1)


def per_impression_device(probs: Tensor, labels: Tensor, offsets: Tensor, metrics: Sequence[str]) -> Dict[str, Tensor]:
    """probs [N] (ranked values, fp32), labels [N] (0/1), offsets [G+1] int32 — device tensors.

    Returns {metric: float64 device tensor [G]} for every per-impression metric named in ``metrics``
    (group_auc, mrr, ndcg@k, hit@k); impression g owns [offsets[g], offsets[g+1]). Nothing but the
    count of mixed-label ties comes back to the host.
    """
    for t in (probs, labels, offsets):
        if t.device.type != "cuda":
            raise RuntimeError("miner_amd.metrics runs on the GPU only (no CPU fallback)")
    probs = probs.reshape(-1).to(torch.float32).contiguous()
    lab = labels.reshape(-1).to(torch.uint8).contiguous()
    offs = offsets.to(torch.int32).contiguous()
    G = offs.numel() - 1
    ks = _ks(metrics)
    if len(ks) > 8:
        raise ValueError("at most 8 distinct @k cut-offs per call")
    nk = len(ks)
    out = torch.empty((max(G, 0), 2 + 2 * nk), dtype=torch.float64, device=probs.device)
    mixed = torch.empty((max(G, 0),), dtype=torch.uint8, device=probs.device)
    karr = (np.ctypeslib.ctypes.c_int32 * max(nk, 1))(*ks)
    with torch.cuda.device(probs.device):
        rc = _lib.lib().miner_impression_metrics(torch.cuda.current_stream(probs.device).cuda_stream,
                                                 probs.data_ptr(), lab.data_ptr(), offs.data_ptr(), G,
                                                 karr, nk, out.data_ptr(), mixed.data_ptr())
    _lib.check(rc, "miner_impression_metrics")
    mix = torch.nonzero(mixed).reshape(-1) if G else None
    if mix is not None and mix.numel():
        # the reference's argsort order among mixed-label ties (np.argsort, evaluation.py:188, :208):
        # those rows are recomputed on the host by the reference formulas, batched per candidate count
        lo, hi = offs[mix].long(), offs[mix + 1].long()
        lens = (hi - lo).cpu().numpy()
        for c in np.unique(lens):
            sel = np.flatnonzero(lens == c)
            rows = mix[torch.from_numpy(sel).to(mix.device)]
            idx = lo[torch.from_numpy(sel).to(lo.device)][:, None] + torch.arange(int(c), device=lo.device)
            P = probs[idx].double().cpu().numpy()
            Y = lab[idx].cpu().numpy().astype(np.int64)
            fix = out[rows].cpu().numpy()
            fix[:, 1] = mrr_rows(Y, P)
            for t, k in enumerate(ks):
                fix[:, 2 + t] = ndcg_rows(Y, P, k)
            out[rows] = torch.from_numpy(fix).to(out.device)
    cols = {"group_auc": out[:, 0], "mrr": out[:, 1]}
    for t, k in enumerate(ks):
        cols[f"ndcg@{k}"] = out[:, 2 + t]
        cols[f"hit@{k}"] = out[:, 2 + nk + t]
    return {m: cols[evaluation.metric_key(m)] for m in metrics if m != "auc"}


def per_impression(probs: Tensor, labels: Tensor, offsets: Tensor, metrics: Sequence[str]) -> Dict[str, np.ndarray]:
    """``per_impression_device`` with the arrays on the host (float64 [G] per metric)."""
    return {m: v.cpu().numpy() for m, v in per_impression_device(probs, labels, offsets, metrics).items()}


def nan_sums(cols: Dict[str, Tensor]) -> Dict[str, tuple]:
    """{metric: (sum of the non-NaN values, their count)} reduced on the device, one copy back:
    the pieces of ``np.nanmean`` (evaluation.py:56-82) that add up across ranks."""
    if not cols:
        return {}
    names = list(cols)
    v = torch.stack([cols[m] for m in names])
    ok = ~torch.isnan(v)
    red = torch.stack([torch.where(ok, v, torch.zeros_like(v)).sum(1), ok.sum(1).to(torch.float64)]).cpu().numpy()
    return {m: (float(red[0, i]), float(red[1, i])) for i, m in enumerate(names)}


def global_auc(probs: Tensor, labels: Tensor) -> float:
    """The reference's flattened ``auc`` (src/evaluation.py:53-55, sklearn roc_auc_score over all
    pairs) computed exactly on the device (``miner_global_auc``: radix sort + integer rank sum, ties
    counted one half). NaN when a class is absent (where sklearn raises)."""
    for t in (probs, labels):
        if t.device.type != "cuda":
            raise RuntimeError("miner_amd.metrics runs on the GPU only (no CPU fallback)")
    p = probs.reshape(-1).to(torch.float32).contiguous()
    y = labels.reshape(-1).to(device=p.device, dtype=torch.uint8).contiguous()
    n = p.numel()
    if n != y.numel():
        raise ValueError(f"{n} scores but {y.numel()} labels")
    if n == 0:
        return float("nan")
    nbytes = _lib.lib().miner_auc_workspace_bytes(n)
    if nbytes == 0:
        raise ValueError(f"global AUC over {n} pairs is not supported (at most 2^31 - 1)")
    ws = torch.empty(nbytes, dtype=torch.uint8, device=p.device)
    out = torch.empty(1, dtype=torch.float64, device=p.device)
    with torch.cuda.device(p.device):
        rc = _lib.lib().miner_global_auc(torch.cuda.current_stream(p.device).cuda_stream, p.data_ptr(), y.data_ptr(),
                                         n, ws.data_ptr(), nbytes, out.data_ptr())
    _lib.check(rc, "miner_global_auc")
    return float(out.item())


def compute_metrics(probs: Tensor, labels: Tensor, offsets: Tensor, metrics: List[str], save_result: bool = False,
                    path: str = None) -> Dict[str, float]:
    """The reference's metric dict (src/evaluation.py:36-84) for impressions already sorted by id."""
    per = per_impression_device(probs, labels, offsets, metrics)
    sums = nan_sums(per)
    out = {}
    for m in metrics:
        if m == "auc":
            out["auc"] = global_auc(probs, labels)
            continue
        s, c = sums[m]
        out[evaluation.metric_key(m)] = s / c if c > 0 else float("nan")       # np.nanmean
        if save_result:
            vals = per[m].cpu().numpy()
            w = vals.astype(int) if m.startswith("hit") else vals
            evaluation.save_scores(os.path.join(path, evaluation.metric_file(m)), w.tolist())
    return out


class DeviceEvaluator:
    """Batched-layout evaluator with device-resident accumulation.

    ``add(scores, labels, impression_ids, cand_offsets=None)`` takes the kernel's logits (dense
    [B,C] or ragged [N] + offsets) on the device and keeps sigmoid(logits) (evaluation.py:165) and the
    labels there; ``compute_scores(metrics, save_result, path)`` orders impressions by id
    (evaluation.py:124, :143), runs the GPU metrics and, under torch.distributed, reduces over ranks
    (each rank holding a contiguous id range).
    """

    def __init__(self):
        self._probs, self._labels, self._sizes, self._ids = [], [], [], []

    def add(self, scores: Tensor, labels: Tensor, impression_ids: Tensor, cand_offsets: Tensor = None):
        self._probs.append(torch.sigmoid(scores.float()).reshape(-1))
        self._labels.append(labels.reshape(-1).to(device=scores.device, dtype=torch.uint8))
        if cand_offsets is None:
            self._sizes.append(torch.full((scores.shape[0],), scores.shape[1], device=scores.device, dtype=torch.int64))
        else:
            self._sizes.append(torch.diff(cand_offsets.to(device=scores.device, dtype=torch.int64)))
        self._ids.append(impression_ids.reshape(-1).to(device=scores.device, dtype=torch.int64))

    def arrays(self):
        if not self._probs:           # an empty shard (a rank with no impressions)
            dev = torch.device("cuda", torch.cuda.current_device())
            return (torch.zeros(0, device=dev), torch.zeros(0, dtype=torch.uint8, device=dev),
                    torch.zeros(1, dtype=torch.int32, device=dev))
        probs = torch.cat(self._probs)
        lab = torch.cat(self._labels)
        sizes = torch.cat(self._sizes)
        ids = torch.cat(self._ids)
        order = torch.argsort(ids, stable=True)
        offs = torch.zeros(sizes.numel() + 1, dtype=torch.int64, device=sizes.device)
        offs[1:] = torch.cumsum(sizes, 0)
        if not torch.equal(order, torch.arange(order.numel(), device=order.device)):
            # impressions re-laid out in id order (evaluation.py:124, :143), one gather on the device
            starts = offs[:-1][order]
            sizes = sizes[order]
            offs[1:] = torch.cumsum(sizes, 0)
            seg = torch.repeat_interleave(torch.arange(sizes.numel(), device=sizes.device), sizes)
            idx = starts[seg] + torch.arange(seg.numel(), device=seg.device) - offs[:-1][seg]
            probs, lab = probs[idx], lab[idx]
        return probs, lab, offs.to(torch.int32)

    def compute_scores(self, metrics: List[str], save_result: bool = False, path: str = None) -> Dict[str, float]:
        from . import distributed
        probs, lab, offs = self.arrays()
        if distributed.world()[1] == 1:
            if offs.numel() == 1:
                raise ValueError("no impressions to evaluate")
            return compute_metrics(probs, lab, offs, metrics, save_result, path)
        return distributed.reduce_device_metrics(probs, lab, offs, metrics, save_result, path)
