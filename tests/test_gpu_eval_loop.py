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


WIDE = dict(CFG, n=300, L=100, K=64, ragged=(2, 100))


@pytest.mark.parametrize("scorer,cfg", [("news", CFG), ("gather", CFG), ("news", WIDE)],
                         ids=["news", "gather", "news-wide"])
def test_eval_loop_matches_oracle(scorer, cfg):
    """'news-wide' (K = 64 interests, 100-click histories) goes through news_score_x2w."""
    from miner_amd import news
    if cfg is WIDE:
        assert news.wide_supported(torch.float32, cfg["L"], cfg["d"], cfg["Dc"], cfg["K"])
    table = synthetic.news_table(5, cfg["n_news"], cfg["d"], device=DEV)
    W1, Q, W2 = synthetic.init_weights(5, cfg["d"], cfg["Dc"], cfg["K"], device=DEV)
    beh = synthetic.behaviors(5, 0, cfg["n"], L=cfg["L"], n_news=cfg["n_news"], ragged=cfg["ragged"], device=DEV)
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


def _tiny_setup(tmp_path, d):
    from miner_amd import formats
    here = os.path.dirname(os.path.abspath(__file__))
    tiny = os.path.join(here, "golden", "mind_tiny")
    news = formats.read_news_tsv(os.path.join(tiny, "news.tsv"), formats.read_category2id(os.path.join(tiny, "category2id.json")))
    np.save(tmp_path / "t.npy", synthetic.news_table(3, news.n_rows, d).numpy())
    files = ["--eval_behaviors_path", os.path.join(tiny, "behaviors.tsv"),
             "--eval_news_path", os.path.join(tiny, "news.tsv"),
             "--category2id_path", os.path.join(tiny, "category2id.json"),
             "--news_table", str(tmp_path / "t.npy"), "--eval_path", str(tmp_path / "eval")]
    return tiny, news, files


class _Enc(torch.nn.Module):
    embed_dim = 256


def _check_outputs(tmp_path, metric_files=("group_auc.txt", "mrr.txt", "ndcg5.txt", "ndcg10.txt", "hit5.txt", "hit10.txt")):
    import json
    import pickle
    runs = os.listdir(tmp_path / "eval")
    assert len(runs) == 1
    out = tmp_path / "eval" / runs[0]
    for f in ("all.log", "args.json", "preds.pkl") + tuple(metric_files):
        assert (out / f).exists(), f
    with open(out / "preds.pkl", "rb") as f:        # written by this test's own process
        pred = pickle.load(f)
    assert len(pred["pred"]) == len(pred["impression_id"]) and all(len(p) == 1 for p in pred["pred"])
    assert pred["impression_id"] == sorted(pred["impression_id"])
    with open(out / "args.json") as f:
        assert "saved_model_path" in json.load(f)
    return out, pred


def test_driver_on_mind_files(tmp_path):
    """`main.py eval` end to end on the tiny MIND dataset: tsv reader + news table + state_dict ->
    loss, metrics, and the reference's output files under <eval_path>/<timestamp>/."""
    from miner_amd import model
    tiny, news, files = _tiny_setup(tmp_path, 256)
    m = model.Miner(_Enc(), False, 32, 200, "weighted", 0.0)
    torch.save(m.state_dict(), tmp_path / "sd.pt")
    loss, scores = eval_loop.main(["eval", *files, "--saved_model_path", str(tmp_path / "sd.pt"),
                                   "--his_length", "6", "--save_eval_result"])
    assert np.isfinite(loss) and 0.0 <= scores["auc"] <= 1.0
    out, pred = _check_outputs(tmp_path)
    vals = np.loadtxt(out / "mrr.txt", ndmin=1)
    assert vals.size == len(set(pred["impression_id"]))


def test_driver_category_bias_checkpoint(tmp_path):
    """A use_category_bias checkpoint (state_dict with category_embedding.weight) is scored with the
    reference's per-candidate bias, not silently without it."""
    from miner_amd import formats, model
    tiny, news, files = _tiny_setup(tmp_path, 256)
    n_cat = int(news.category.max()) + 1
    m = model.Miner(_Enc(), True, 32, 200, "weighted", 0.0, num_category=n_cat, category_embed_dim=16,
                    category_pad_token_id=news.pad_category)
    torch.save(m.state_dict(), tmp_path / "sd.pt")
    loss_b, sc_b = eval_loop.main(["eval", *files, "--saved_model_path", str(tmp_path / "sd.pt"), "--his_length", "6"])
    sd = {k: v for k, v in m.state_dict().items() if not k.startswith("category_embedding")}
    torch.save(sd, tmp_path / "sd_nobias.pt")
    loss_n, sc_n = eval_loop.main(["eval", *files, "--saved_model_path", str(tmp_path / "sd_nobias.pt"),
                                   "--his_length", "6"])
    assert np.isfinite(loss_b) and loss_b != loss_n


def _bias_golden():
    from tests.conftest import load_golden
    g = load_golden("edge_bias")
    n_rows = g["table"].shape[0]
    row_cat = np.zeros(n_rows, np.int64)
    row_cat[g["his_ids"].reshape(-1)] = g["his_cat"].reshape(-1)
    row_cat[g["cand_ids"].reshape(-1)] = g["cand_cat"].reshape(-1)
    row_cat[0] = 0                                   # the pad news: the pad category
    B, C = g["B"], g["C"]
    beh = synthetic.Behaviors(torch.from_numpy(g["his_ids"]).to(DEV, torch.int32), torch.from_numpy(g["his_mask"]).to(DEV),
                              torch.from_numpy(g["cand_ids"].reshape(-1)).to(DEV, torch.int32),
                              torch.arange(0, (B + 1) * C, C, dtype=torch.int32, device=DEV),
                              torch.from_numpy(g["labels"].reshape(-1)).to(DEV, torch.uint8),
                              torch.arange(B, device=DEV))
    return g, beh, row_cat


@pytest.mark.parametrize("scorer", ["news", "gather"])
def test_category_bias_matches_reference_eval(scorer):
    """Per-(impression, candidate) category bias (model.py:113-122, :176 with reader.py:376-379's
    one-candidate samples) against the reference's own per-candidate eval in the edge_bias fixture:
    scores, metric dict and eval loss."""
    g, beh, row_cat = _bias_golden()
    table = torch.from_numpy(g["table"]).to(DEV)
    cat = eval_loop.CategoryBias.from_embedding(torch.from_numpy(g["category_embedding"]).to(DEV),
                                               torch.from_numpy(row_cat))
    preds = []
    loss, scores = eval_loop.evaluate(ops.pack_weights(*(torch.from_numpy(g[k]).to(DEV) for k in ("W1", "Q", "W2"))),
                                      table, beh, METRICS, scorer=scorer, category=cat, predictions=preds)
    probs = torch.cat([p[0] for p in preds]).cpu().double().numpy()
    ref = 1.0 / (1.0 + np.exp(-g["scores_per_candidate"].reshape(-1).astype(np.float64)))
    ok, worst = orc.parity_ok(probs, ref)
    assert ok, f"per-candidate bias probabilities off by {worst:.2f}x the tolerance"
    for k, v in g["metrics"].items():
        assert scores[k] == pytest.approx(v, abs=1e-6), k
    assert loss == pytest.approx(float(g["eval_loss"]), rel=1e-5)


def test_fastformer_eval_matches_reference():
    """trainer_fastformer._eval semantics: scores of the reference FastFormer (fixture), metrics as
    the reference evaluator computes them from those scores, vanilla eval loss (loss.py:47-65)."""
    from miner_amd import fastformer as ff
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fastformer_cfg4_slice.npz"))
    params = {k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("p.")}
    B, C = int(z["B"]), int(z["C"])
    rng = np.random.default_rng(0)
    lab = (rng.random((B, C)) < 0.25).astype(np.uint8)
    lab[:, 0], lab[:, 1] = 1, 0
    beh = synthetic.Behaviors(torch.from_numpy(z["his_ids"]).to(DEV, torch.int32), torch.from_numpy(z["his_mask"]).to(DEV),
                              torch.from_numpy(z["cand_ids"].reshape(-1)).to(DEV, torch.int32),
                              torch.arange(0, (B + 1) * C, C, dtype=torch.int32, device=DEV),
                              torch.from_numpy(lab.reshape(-1)).to(DEV), torch.arange(B, device=DEV))
    preds = []
    packed = ff.pack(ff.flatten_params({k: v.to(DEV) for k, v in params.items()}), torch.float32)
    loss, scores = eval_loop.evaluate_fastformer(packed, torch.from_numpy(z["table"]).to(DEV), beh, METRICS,
                                                 predictions=preds)
    ref_s = z["scores"].astype(np.float64)
    probs = torch.cat([p[0] for p in preds]).cpu().double().numpy()
    assert orc.parity_ok(probs, 1.0 / (1.0 + np.exp(-ref_s.reshape(-1))))[0]
    want = mo.compute_scores([list(r) for r in lab], [list(1.0 / (1.0 + np.exp(-r))) for r in ref_s], METRICS)
    for k, v in want.items():
        assert scores[k] == pytest.approx(v, abs=1e-6), k
    ref_loss = float(-(torch.nn.functional.logsigmoid(torch.from_numpy(ref_s)) * torch.from_numpy(lab)).sum() / lab.sum())
    assert loss == pytest.approx(ref_loss, rel=1e-5)


def test_driver_eval_fastformer(tmp_path):
    """`main.py eval_fastformer` end to end on the tiny MIND dataset with a FastFormer state_dict."""
    from miner_amd import fastformer as ff
    tiny, news, files = _tiny_setup(tmp_path, 256)
    enc = ff.FastFormer(_Enc(), "weighted", 0.0)
    torch.save(enc.state_dict(), tmp_path / "ff.pt")
    loss, scores = eval_loop.main(["eval_fastformer", *files, "--saved_model_path", str(tmp_path / "ff.pt"),
                                   "--his_length", "6", "--save_eval_result"])
    assert np.isfinite(loss) and 0.0 <= scores["auc"] <= 1.0
    _check_outputs(tmp_path)


def test_device_global_auc_matches_sklearn():
    """miner_global_auc (exact rank sum on the device) vs scikit-learn's roc_auc_score
    (evaluation.py:53-55), with heavy ties, -0/+0, negative scores, and one class absent."""
    from sklearn.metrics import roc_auc_score
    from miner_amd import metrics
    g = torch.Generator().manual_seed(0)
    for n, levels in ((1, None), (7, 3), (1000, None), (100_000, 50), (300_000, None)):
        s = torch.randn(n, generator=g)
        if levels:
            s = torch.round(s * levels) / levels
        y = (torch.rand(n, generator=g) < 0.3).to(torch.uint8)
        if n > 1:
            y[0], y[1] = 1, 0
            s[:4] = torch.tensor([0.0, -0.0, 0.0, -0.0])[:min(4, n)]
        got = metrics.global_auc(s.to(DEV), y.to(DEV))
        if y.min() == y.max():
            assert np.isnan(got)
        else:
            assert got == pytest.approx(roc_auc_score(y.numpy(), s.double().numpy()), abs=1e-12)
