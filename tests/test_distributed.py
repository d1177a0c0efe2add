"""Impression sharding + metric/loss reduction over 2 ranks (gloo on CPU), against the reference's
golden metrics computed by one process. Rehearses the N>1 path bench.py / the eval driver take."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from miner_amd import distributed as mdist
from miner_amd import evaluation as ev

from conftest import load_golden
from test_oracle_golden import METRICS, PER_IMP


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_range_partitions():
    for n in (0, 1, 7, 200, 3_000_000):
        for ws in (1, 2, 3, 8):
            spans = [mdist.shard_range(n, r, ws) for r in range(ws)]
            assert spans[0][0] == 0
            for (s0, c0), (s1, _) in zip(spans, spans[1:]):
                assert s0 + c0 == s1
            assert sum(c for _, c in spans) == n
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def _worker(rank, ws, port, name, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws),
                      LOCAL_RANK=str(rank))
    r, w, _ = mdist.init_from_env("gloo")
    assert (r, w) == (rank, ws)
    g = load_golden(name)
    B, C = g["B"], g["C"]
    start, cnt = mdist.shard_range(B, rank, ws)
    sl = slice(start, start + cnt)
    offs = np.arange(cnt + 1) * C
    pairs = ev.GroupedPairs(g["labels"][sl].reshape(-1), g["probs_grouped"][sl].reshape(-1), offs)
    got = mdist.reduce_metrics(pairs, METRICS, save_result=True, path=outdir)
    part = ev.eval_loss_partials(torch.from_numpy(g["mui"][sl]), torch.from_numpy(g["scores_per_candidate"][sl]),
                                 torch.from_numpy(g["labels"][sl]), first_sample=start * C, total_samples=B * C)
    loss = mdist.reduce_eval_loss(part)
    # preds.pkl through the multi-rank gather of the eval driver (rank 0 writes it)
    from miner_amd import eval_loop
    chunks = [(torch.from_numpy(g["probs_grouped"][sl]).float(), torch.arange(start, start + cnt),
               torch.from_numpy(offs.astype(np.int32)))]
    os.makedirs(os.path.join(outdir, "ranks"), exist_ok=True)
    eval_loop._write_predictions(os.path.join(outdir, "ranks"), chunks, rank)
    res = dict(got, eval_loss=loss)
    torch.save({k: float(v) for k, v in res.items()}, os.path.join(outdir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("name,ws", [("cfg1_demo", 2), ("edge_ties", 2), ("cfg1_demo", 3)])
def test_reduce_metrics_over_ranks_equals_single_process(name, ws):
    g = load_golden(name)
    with tempfile.TemporaryDirectory() as td:
        mp.start_processes(_worker, args=(ws, _free_port(), name, td), nprocs=ws, join=True, start_method="spawn")
        per_rank = [torch.load(os.path.join(td, f"rank{r}.pt"), weights_only=True) for r in range(ws)]
        for m, key in PER_IMP.items():
            np.testing.assert_allclose(np.loadtxt(os.path.join(td, ev.metric_file(m)), ndmin=1), g[key],
                                       atol=1e-12, equal_nan=True)
        # preds.pkl from the ranks is byte-identical to the one-process file
        from miner_amd import eval_loop
        B, C = g["B"], g["C"]
        one = [(torch.from_numpy(g["probs_grouped"]).float(), torch.arange(B),
                torch.from_numpy((np.arange(B + 1) * C).astype(np.int32)))]
        os.makedirs(os.path.join(td, "one"))
        eval_loop._write_predictions(os.path.join(td, "one"), one, 0)
        with open(os.path.join(td, "ranks", "preds.pkl"), "rb") as a, open(os.path.join(td, "one", "preds.pkl"), "rb") as b:
            assert a.read() == b.read()
    for res in per_rank:
        assert res == per_rank[0]           # every rank holds the same answer
        for k, v in g["metrics"].items():
            assert res[k] == pytest.approx(v, abs=1e-12), k
        assert res["eval_loss"] == pytest.approx(float(g["eval_loss"]), rel=1e-6)
