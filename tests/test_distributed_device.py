"""reduce_device_metrics (miner_amd/distributed.py) over 2 ranks with gloo: the eval loop's N > 1
metric path for device-resident (prob, label, offsets) — per-impression metrics from the GPU kernel,
(Σ, count) all-reduced per metric, the exact global AUC from pairs gathered once to rank 0 and
broadcast, the per-impression <metric>.txt files written by rank 0 in impression order. Checked
against the reference's golden metrics (tests/golden, made by the reference's SlowEvaluator).

* CPU: the three device steps (per_impression_device, nan_sums, global_auc) are replaced inside the
  test processes by the oracle's restatement of src/evaluation.py, so the reduction, gather and
  broadcast logic of reduce_device_metrics runs on the CPU suite (the product path never routes
  through the oracle: these stand-ins exist only in the spawned test workers).
* GPU: both ranks on cuda:0 with the real kernels (miner_metrics.hip, miner_auc.hip), gloo for the
  collectives (the tensors cross through the host as the backend needs).
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import load_golden
from test_oracle_golden import METRICS, PER_IMP


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _install_cpu_standins():
    """Test-only CPU replacements of the device metric steps, from the oracle (evaluation.py:36-84)."""
    from miner_amd import evaluation, metrics
    from oracle import metrics_oracle as mo

    def per_impression_device(probs, labels, offsets, mets):
        o = offsets.cpu().numpy().astype(np.int64)
        p, y = probs.cpu().double().numpy().reshape(-1), labels.cpu().numpy().reshape(-1)
        tg = [y[o[i]:o[i + 1]].tolist() for i in range(len(o) - 1)]
        pr = [p[o[i]:o[i + 1]].tolist() for i in range(len(o) - 1)]
        return {m: torch.tensor(np.asarray(mo.per_impression(tg, pr, m), np.float64)) for m in mets}

    def nan_sums(cols):
        out = {}
        for m, v in cols.items():
            v = v.double()
            ok = ~torch.isnan(v)
            out[m] = (float(v[ok].sum()), float(ok.sum()))
        return out

    def global_auc(probs, labels):
        from sklearn.metrics import roc_auc_score
        return float(roc_auc_score(labels.cpu().numpy(), probs.cpu().double().numpy()))

    metrics.per_impression_device = per_impression_device
    metrics.nan_sums = nan_sums
    metrics.global_auc = global_auc
    assert evaluation is not None


def _worker(rank, ws, port, name, outdir, on_gpu):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws),
                      LOCAL_RANK=str(rank))
    from miner_amd import distributed as mdist
    if not on_gpu:
        _install_cpu_standins()
    r, w, _ = mdist.init_from_env("gloo")
    assert (r, w) == (rank, ws)
    dev = "cuda:0" if on_gpu else "cpu"
    g = load_golden(name)
    B, C = g["B"], g["C"]
    start, cnt = mdist.shard_range(B, rank, ws)
    sl = slice(start, start + cnt)
    probs = torch.from_numpy(np.ascontiguousarray(g["probs_grouped"][sl])).float().reshape(-1).to(dev)
    labels = torch.from_numpy(np.ascontiguousarray(g["labels"][sl])).reshape(-1).to(torch.uint8).to(dev)
    offs = torch.from_numpy((np.arange(cnt + 1) * C).astype(np.int32)).to(dev)
    got = mdist.reduce_device_metrics(probs, labels, offs, METRICS, save_result=True, path=outdir)
    torch.save({k: float(v) for k, v in got.items()}, os.path.join(outdir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _run(name, ws, on_gpu):
    g = load_golden(name)
    with tempfile.TemporaryDirectory() as td:
        mp.start_processes(_worker, args=(ws, _free_port(), name, td, on_gpu), nprocs=ws, join=True,
                           start_method="spawn")
        per_rank = [torch.load(os.path.join(td, f"rank{r}.pt"), weights_only=True) for r in range(ws)]
        from miner_amd import evaluation as ev
        for m, key in PER_IMP.items():
            np.testing.assert_allclose(np.loadtxt(os.path.join(td, ev.metric_file(m)), ndmin=1), g[key],
                                       atol=1e-6 if on_gpu else 1e-12, equal_nan=True)
    for res in per_rank:
        assert res == per_rank[0]           # every rank holds the same answer
        for k, v in g["metrics"].items():
            assert res[k] == pytest.approx(v, abs=1e-6 if on_gpu else 1e-12), k


@pytest.mark.parametrize("name,ws", [("cfg1_demo", 2), ("edge_ties", 2)])
def test_reduce_device_metrics_gloo_cpu(name, ws):
    _run(name, ws, on_gpu=False)


@pytest.mark.gpu
@pytest.mark.parametrize("name,ws", [("cfg1_demo", 2), ("edge_ties", 2)])
def test_reduce_device_metrics_gloo_gpu(name, ws):
    _run(name, ws, on_gpu=True)
