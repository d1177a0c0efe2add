"""The eval loop (Trainer._eval semantics on the MI355X kernels) against the CPU oracle, and its
multi-rank reduction (2 ranks, gloo, sharing cuda:0) against one process — needs an MI355X."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from miner_amd import eval_loop, ops, synthetic
from oracle import metrics_oracle as mo
from oracle import miner_oracle as orc

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
METRICS = ["auc", "group_auc", "mrr", "ndcg@5", "ndcg@10", "hit@5", "hit@10"]
CFG = dict(n=600, L=30, n_news=2000, d=256, Dc=64, K=8, ragged=(2, 30))


def _setup(device):
    table = synthetic.news_table(5, CFG["n_news"], CFG["d"], device=device)
    W1, Q, W2 = synthetic.init_weights(5, CFG["d"], CFG["Dc"], CFG["K"], device=device)
    return table, W1, Q, W2


@pytest.mark.parametrize("scorer", ["news", "gather"])
def test_eval_loop_matches_oracle(scorer):
    table, W1, Q, W2 = _setup(DEV)
    beh = synthetic.behaviors(5, 0, CFG["n"], L=CFG["L"], n_news=CFG["n_news"], ragged=CFG["ragged"], device=DEV)
    loss, scores = eval_loop.evaluate(ops.pack_weights(W1, Q, W2), table, beh, METRICS, chunk=256, scorer=scorer)
    # oracle: reference op order on the gathered rows, one impression at a time (ragged)
    t, w1, q, w2 = table.cpu(), W1.cpu(), Q.cpu(), W2.cpu()
    offs = beh.cand_offsets.cpu().numpy()
    hid, msk, cid, lab = beh.his_ids.cpu(), beh.his_mask.cpu(), beh.cand_ids.cpu(), beh.labels.cpu().numpy()
    targets, probs, mui_s, logits = [], [], [], []
    for b in range(beh.n):
        c = cid[offs[b]:offs[b + 1]]
        mui, s = orc.score_torch(t[hid[b]][None], msk[b][None], t[c][None], w1, q, w2)
        targets.append(list(lab[offs[b]:offs[b + 1]]))
        probs.append(list(torch.sigmoid(s[0]).double().numpy()))
        mui_s.append(mui.repeat(len(c), 1, 1))
        logits.append(s[0])
    want = mo.compute_scores(targets, probs, METRICS)
    for k, v in want.items():
        assert scores[k] == pytest.approx(v, abs=2e-4), k   # fp32 1e-5 score parity; rank flips only at near-ties
    ref_loss = orc.eval_loss_torch(torch.cat(mui_s), torch.cat(logits)[:, None],
                                   torch.from_numpy(np.concatenate([np.asarray(x) for x in targets]))[:, None].double())
    assert loss == pytest.approx(ref_loss, rel=1e-5)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, ws, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws),
                      LOCAL_RANK="0")
    from miner_amd import distributed
    distributed.init_from_env("gloo")
    table, W1, Q, W2 = _setup(DEV)
    table = table.to(torch.bfloat16)   # bf16: a deterministic reduction order, runs compare bit for bit
    start, count = distributed.shard_range(CFG["n"], rank, ws)
    beh = synthetic.behaviors(5, start, count, L=CFG["L"], n_news=CFG["n_news"], ragged=CFG["ragged"], device=DEV)
    whole = synthetic.behaviors(5, 0, CFG["n"], L=CFG["L"], n_news=CFG["n_news"], ragged=CFG["ragged"])
    first = int(whole.cand_offsets[start])
    loss, scores = eval_loop.evaluate(ops.pack_weights(W1, Q, W2, dtype=torch.bfloat16), table, beh, METRICS,
                                      first_sample=first, total_samples=int(whole.cand_offsets[-1]), chunk=128)
    torch.save(dict(scores, loss=loss), os.path.join(out, f"r{rank}.pt"))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def test_two_ranks_equal_one():
    table, W1, Q, W2 = _setup(DEV)
    table = table.to(torch.bfloat16)
    beh = synthetic.behaviors(5, 0, CFG["n"], L=CFG["L"], n_news=CFG["n_news"], ragged=CFG["ragged"], device=DEV)
    loss1, s1 = eval_loop.evaluate(ops.pack_weights(W1, Q, W2, dtype=torch.bfloat16), table, beh, METRICS, chunk=128)
    with tempfile.TemporaryDirectory() as td:
        mp.start_processes(_rank, args=(2, _free_port(), td), nprocs=2, join=True, start_method="spawn")
        res = [torch.load(os.path.join(td, f"r{r}.pt"), weights_only=True) for r in range(2)]
    for r in res:
        assert r["loss"] == pytest.approx(loss1, rel=1e-9)
        for k, v in s1.items():
            assert r[k] == pytest.approx(v, abs=1e-9), k


def test_driver_on_mind_files(tmp_path):
    """The eval driver end to end on the tiny MIND dataset: tsv reader + news table + state_dict."""
    from miner_amd import formats, model
    here = os.path.dirname(os.path.abspath(__file__))
    tiny = os.path.join(here, "golden", "mind_tiny")
    news = formats.read_news_tsv(os.path.join(tiny, "news.tsv"), formats.read_category2id(os.path.join(tiny, "category2id.json")))
    d = 256
    np.save(tmp_path / "t.npy", synthetic.news_table(3, news.n_rows, d).numpy())

    class Enc(torch.nn.Module):
        embed_dim = d

    m = model.Miner(Enc(), False, 32, 200, "weighted", 0.0)
    torch.save(m.state_dict(), tmp_path / "sd.pt")
    loss, scores = eval_loop.main(["--eval_behaviors_path", os.path.join(tiny, "behaviors.tsv"),
                                   "--eval_news_path", os.path.join(tiny, "news.tsv"),
                                   "--category2id_path", os.path.join(tiny, "category2id.json"),
                                   "--news_table", str(tmp_path / "t.npy"), "--state_dict", str(tmp_path / "sd.pt"),
                                   "--his_length", "6", "--precision", "fp32"])
    assert np.isfinite(loss) and 0.0 <= scores["auc"] <= 1.0
