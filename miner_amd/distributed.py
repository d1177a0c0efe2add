"""Impression sharding and metric reduction across ranks.

Impressions are independent (no cross-impression term in src/model/model.py:113-216), so each rank
scores a contiguous impression range with replicated weights and no data-path collective. Only the
evaluation needs exchanges, and only small ones:

* group_auc / mrr / ndcg@k / hit@k are ``np.nanmean`` over impressions (src/evaluation.py:56-82):
  each rank all-reduces (Σ non-NaN values, count) — a few float64s per metric;
* the global ``auc`` (src/evaluation.py:53-55) is not decomposable: the (score, label) pairs are
  gathered once to rank 0 (c3: 120 M pairs ≈ 600 MB over xGMI), which computes the exact AUC on its
  device (miner_global_auc) and broadcasts it;
* the eval loss (src/loss.py:68-85, src/trainer.py:276-291) is a sum of per-sample terms once the
  batch partition is fixed: all-reduce (numerator, positives).

One process per GPU, ``torch.distributed`` with backend "nccl" (RCCL over xGMI) on the GPU box and
"gloo" for the CPU tests; collectives run on the device the backend needs.
"""
from __future__ import annotations

import os
from typing import Dict, List, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import evaluation


def world() -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def init_from_env(backend: str = None) -> Tuple[int, int, int]:
    """Initialise the default group from torchrun's env (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*).

    Returns (rank, world_size, local_rank); a single process without the env stays uninitialised.
    """
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, ws, local


def shard_range(n: int, rank: int, world_size: int) -> Tuple[int, int]:
    """Contiguous balanced shard of n impressions: (start, count); the first n % ws ranks get one more."""
    base, extra = divmod(n, world_size)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def _coll_device() -> torch.device:
    if dist.is_initialized() and dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def all_reduce_sum(x: np.ndarray) -> np.ndarray:
    """float64 all-reduce(SUM) of a small host array (identity on one process)."""
    if world()[1] == 1:
        return np.asarray(x, np.float64)
    t = torch.as_tensor(np.asarray(x, np.float64), device=_coll_device())
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy()


def all_gather_concat(x: torch.Tensor) -> torch.Tensor:
    """Concatenate every rank's 1-D tensor in rank order (variable lengths; identity on one process)."""
    if world()[1] == 1:
        return x
    dev = _coll_device()
    x = x.to(dev).contiguous()
    n = torch.tensor([x.numel()], device=dev, dtype=torch.int64)
    sizes = [torch.zeros_like(n) for _ in range(dist.get_world_size())]
    dist.all_gather(sizes, n)
    sizes = [int(s) for s in sizes]
    m = max(sizes)
    buf = torch.zeros(m, device=dev, dtype=x.dtype)
    buf[:x.numel()] = x
    out = [torch.empty_like(buf) for _ in sizes]
    dist.all_gather(out, buf)
    return torch.cat([o[:s] for o, s in zip(out, sizes)])


def gather_concat_to_root(x: torch.Tensor, root: int = 0):
    """Concatenate every rank's 1-D tensor in rank order on ``root`` only (None elsewhere; identity
    on one process). One gather of max-size padded buffers: the data crosses the links once."""
    if world()[1] == 1:
        return x
    dev = _coll_device()
    x = x.to(dev).contiguous()
    n = torch.tensor([x.numel()], device=dev, dtype=torch.int64)
    sizes = [torch.zeros_like(n) for _ in range(dist.get_world_size())]
    dist.all_gather(sizes, n)
    sizes = [int(s) for s in sizes]
    m = max(sizes)
    buf = torch.zeros(m, device=dev, dtype=x.dtype)
    buf[:x.numel()] = x
    if dist.get_rank() == root:
        out = [torch.empty_like(buf) for _ in sizes]
        dist.gather(buf, out, dst=root)
        return torch.cat([o[:s] for o, s in zip(out, sizes)])
    dist.gather(buf, None, dst=root)
    return None


def broadcast_float(v, root: int = 0) -> float:
    """One float64 from ``root`` to every rank."""
    if world()[1] == 1:
        return float(v)
    t = torch.tensor([float("nan") if v is None else float(v)], dtype=torch.float64, device=_coll_device())
    dist.broadcast(t, src=root)
    return float(t.item())


def reduce_metrics(pairs: "evaluation.GroupedPairs", metrics: List[str], save_result: bool = False,
                   path: str = None) -> Dict[str, float]:
    """The reference's compute_scores (src/evaluation.py:36-84) over all ranks' impressions.

    ``pairs`` holds this rank's impressions (a contiguous id range; ranks in id order). Every rank
    returns the same dict; with ``save_result`` rank 0 writes the per-impression <metric>.txt files
    in impression-id order, as the reference does for one process.
    """
    rank, ws = world()
    if ws == 1:
        return evaluation.compute_metrics(pairs, metrics, save_result, path)
    out = {}
    for metric in metrics:
        if metric == "auc":
            sc = gather_concat_to_root(torch.from_numpy(pairs.scores))
            lb = gather_concat_to_root(torch.from_numpy(pairs.labels.astype(np.uint8)))
            auc = evaluation.auc_score(lb.cpu().numpy(), sc.cpu().numpy()) if rank == 0 else None
            out["auc"] = broadcast_float(auc)
            continue
        vals = pairs.per_impression(metric)
        ok = ~np.isnan(vals)
        s, c = all_reduce_sum(np.array([vals[ok].sum(), ok.sum()], np.float64))
        out[evaluation.metric_key(metric)] = float(s / c) if c > 0 else float("nan")
        if save_result:
            full = gather_concat_to_root(torch.from_numpy(vals))
            if rank == 0:
                full = full.cpu().numpy()
                w = full.astype(int) if metric.startswith("hit") else full
                evaluation.save_scores(os.path.join(path, evaluation.metric_file(metric)), w.tolist())
    return out


def reduce_device_metrics(probs: torch.Tensor, labels: torch.Tensor, offsets: torch.Tensor, metrics: List[str],
                          save_result: bool = False, path: str = None) -> Dict[str, float]:
    """As ``reduce_metrics`` for device-resident (prob, label, offsets) of this rank's impressions,
    with the per-impression metrics computed by the GPU kernel (miner_amd.metrics)."""
    from . import metrics as gm
    rank, ws = world()
    per = gm.per_impression_device(probs, labels, offsets, [m for m in metrics if m != "auc"])
    sums = gm.nan_sums(per)
    out = {}
    for metric in metrics:
        if metric == "auc":
            # exact global AUC (evaluation.py:53-55): the pairs go to rank 0 once, the device rank
            # sum runs there (miner_global_auc), the value is broadcast
            sc = gather_concat_to_root(probs.float().reshape(-1))
            lb = gather_concat_to_root(labels.reshape(-1).to(torch.uint8))
            auc = gm.global_auc(sc.to(probs.device), lb.to(probs.device)) if rank == 0 else None
            out["auc"] = broadcast_float(auc)
            continue
        s, c = all_reduce_sum(np.array(sums[metric], np.float64))
        out[evaluation.metric_key(metric)] = float(s / c) if c > 0 else float("nan")
        if save_result:
            full = gather_concat_to_root(per[metric].cpu())
            if rank == 0:
                full = full.cpu().numpy()
                w = full.astype(int) if metric.startswith("hit") else full
                evaluation.save_scores(os.path.join(path, evaluation.metric_file(metric)), w.tolist())
    return out


def reduce_eval_loss(partials: torch.Tensor) -> float:
    """Sum (numerator, positives) from evaluation.eval_loss_partials over ranks -> the eval loss."""
    num, pos = all_reduce_sum(partials.detach().cpu().numpy())
    return float(num / pos)
