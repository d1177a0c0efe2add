"""Generate the golden fixtures in tests/golden/*.npz by running the REFERENCE itself.

Run in the build container (the only place /root/reference exists):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [case ...]

It imports the reference's own ``src.model.model.Miner`` (src/model/model.py:13-138) with a stub
news encoder (an embedding-table lookup: the north_star path starts from precomputed news
embeddings), its ``SlowEvaluator`` (src/evaluation.py:113-175) and ``Loss.compute_eval_loss``
(src/loss.py:68-85), and records inputs, weights and outputs as plain arrays. The fixtures are data
only: no reference source or bytecode is stored. Skips cleanly when /root/reference is absent.

Layouts recorded per case:
* batched: one row per impression with all C candidates (the layout the HIP kernel uses);
* per-candidate: one sample per (impression, candidate), exactly as reader.py:376-379 builds the
  eval set, batched ``eval_batch_size``=32 (config/eval_miner.txt:19) through Miner.forward, fed to
  SlowEvaluator.eval_batch and compute_scores -> the reference's metric dict.
"""
from __future__ import annotations

import os
import sys
import tempfile

import numpy as np

REF = os.environ.get("MINER_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))
METRICS = ["auc", "group_auc", "mrr", "ndcg@5", "ndcg@10", "hit@5", "hit@10"]


def main():
    if not os.path.isdir(os.path.join(REF, "src")):
        print(f"reference not found at {REF}: skipping golden generation")
        return 0
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import torch
    import torch.nn as nn
    from src.model.model import Miner                      # noqa: E402  (reference)
    from src.evaluation import SlowEvaluator                # noqa: E402  (reference)
    from src.entities import Dataset                        # noqa: E402  (reference)
    from src.loss import Loss                               # noqa: E402  (reference)

    class StubNewsEncoder(nn.Module):
        """Stands in for NewsEncoder (news_encoder.py:60-106): token 0 of the title is a news id."""

        def __init__(self, table):
            super().__init__()
            self.embed_dim = table.shape[1]
            self.register_buffer("table", table)

        def forward(self, title_encoding, title_attn_mask, sapo_encoding=None, sapo_attn_mask=None):
            return self.table[title_encoding[:, 0]]

    only = set(sys.argv[1:])          # case names to (re)generate; all when empty

    def run_case(name, *, B, L, K, d, Dc, C, score_type="weighted", seed=0, use_bias=False,
                 hist_len=None, ties=False, n_cat=12, cat_dim=16):
        if only and name not in only:
            return
        rng = np.random.default_rng(seed)
        n_news = 1 + B * (L + C)
        table = (rng.standard_normal((n_news, d)) / np.sqrt(d)).astype(np.float32)
        # row 0 = the pad news: a real, nonzero embedding (reader.py:101-110)
        if hist_len is None:
            hist_len = rng.integers(0, L + 1, size=B)
        hist_len = np.asarray(hist_len)
        his_ids = np.zeros((B, L), np.int64)
        cand_ids = np.zeros((B, C), np.int64)
        nxt = 1
        for b in range(B):
            n = int(hist_len[b])
            his_ids[b, L - n:] = np.arange(nxt, nxt + n)    # left-padded (reader.py:369)
            nxt += n
            cand_ids[b] = np.arange(nxt, nxt + C)
            nxt += C
        his_mask = his_ids != 0                              # pad <=> masked (entities.py:395)
        labels = np.zeros((B, C), np.int64)
        for b in range(B):                                   # >=1 click and >=1 non-click (reader.py:374)
            npos = 1 if C == 1 else int(rng.integers(1, max(2, C // 4) + 1))
            labels[b, rng.choice(C, size=min(npos, C), replace=False)] = 1
            if C > 1 and labels[b].all():
                labels[b, 0] = 0
        his_cat = np.where(his_mask, rng.integers(1, n_cat, size=(B, L)), 0)
        cand_cat = rng.integers(1, n_cat, size=(B, C))

        torch.manual_seed(seed)
        enc = StubNewsEncoder(torch.from_numpy(table))
        if use_bias:
            model = Miner(enc, True, K, Dc, score_type, 0.2, num_category=n_cat,
                          category_embed_dim=cat_dim, category_pad_token_id=0)
        else:
            model = Miner(enc, False, K, Dc, score_type, 0.2)
        model.eval()
        if ties:  # collapse candidate embeddings so several candidates tie exactly
            tt = enc.table.clone()
            for b in range(B):
                tt[cand_ids[b, 1::2]] = tt[cand_ids[b, 0]].clone()
            enc.table.copy_(tt)
            table = tt.numpy()

        def fwd(hid, cid, hm, hc, cc):
            t = lambda x: torch.from_numpy(np.ascontiguousarray(x))
            title = t(cid)[..., None]
            his = t(hid)[..., None]
            return model(title=title, title_mask=torch.ones_like(title, dtype=torch.bool),
                         his_title=his, his_title_mask=torch.ones_like(his, dtype=torch.bool),
                         his_mask=t(hm), sapo=title, sapo_mask=torch.ones_like(title, dtype=torch.bool),
                         his_sapo=his, his_sapo_mask=torch.ones_like(his, dtype=torch.bool),
                         category=t(cc), his_category=t(hc))

        with torch.no_grad():
            mui, scores = fwd(his_ids, cand_ids, his_mask, his_cat, cand_cat)
            # reference eval layout: one sample per candidate, eval_batch_size 32
            s_his = np.repeat(his_ids, C, axis=0)
            s_mask = np.repeat(his_mask, C, axis=0)
            s_hcat = np.repeat(his_cat, C, axis=0)
            s_cand = cand_ids.reshape(-1, 1)
            s_ccat = cand_cat.reshape(-1, 1)
            s_lab = labels.reshape(-1, 1)
            s_imp = np.repeat(np.arange(B), C)
            ds = Dataset("golden", None, {"pad": 0})
            for i in range(B * C):
                imp = ds.create_impression(int(s_imp[i]), 0, [None], [int(s_lab[i, 0])])
                ds.add_sample(0, [], imp)
            ev = SlowEvaluator(ds)
            pc_scores = []
            total_loss, total_pos = 0.0, 0
            for i in range(0, B * C, 32):
                sl = slice(i, i + 32)
                pa, lg = fwd(s_his[sl], s_cand[sl], s_mask[sl], s_hcat[sl], s_ccat[sl])
                lab = torch.from_numpy(s_lab[sl])
                total_loss += Loss.compute_eval_loss(pa, lg, lab)
                total_pos += lab.sum().item()
                ev.eval_batch(lg, torch.from_numpy(s_imp[sl]))
                pc_scores.append(lg.numpy())
            eval_loss = total_loss / total_pos
            with tempfile.TemporaryDirectory() as td:
                m = ev.compute_scores(METRICS, True, td)
                per_imp = {k: np.loadtxt(os.path.join(td, f), ndmin=1) for k, f in
                           [("group_auc", "group_auc.txt"), ("mrr", "mrr.txt"), ("ndcg@5", "ndcg5.txt"),
                            ("ndcg@10", "ndcg10.txt"), ("hit@5", "hit5.txt"), ("hit@10", "hit10.txt")]}
            bias = None
            if use_bias:
                from src.utils import pairwise_cosine_similarity
                he = model.category_embedding(torch.from_numpy(his_cat))
                ce = model.category_embedding(torch.from_numpy(cand_cat))
                bias = pairwise_cosine_similarity(he, ce).mean(dim=2).numpy()

        arrs = dict(
            B=B, L=L, K=K, d=d, Dc=Dc, C=C, score_type=score_type, use_bias=int(use_bias),
            table=table, his_ids=his_ids, cand_ids=cand_ids, his_mask=his_mask, labels=labels,
            his_cat=his_cat, cand_cat=cand_cat,
            W1=model.poly_attn.linear.weight.detach().numpy(),
            Q=model.poly_attn.context_codes.detach().numpy(),
            mui=mui.numpy(), scores=scores.numpy(),
            scores_per_candidate=np.concatenate(pc_scores, 0).reshape(B, C),
            probs_grouped=np.asarray(ev.prob_predictions, np.float64).reshape(B, C),
            eval_loss=np.float64(eval_loss),
            metric_names=np.array(list(m.keys())), metric_values=np.array([m[k] for k in m], np.float64),
        )
        for k, v in per_imp.items():
            arrs["per_imp_" + k.replace("@", "")] = v
        if score_type == "weighted":
            arrs["W2"] = model.target_aware_attn.linear.weight.detach().numpy()
        if use_bias:
            arrs["category_embedding"] = model.category_embedding.weight.detach().numpy()
            arrs["bias"] = bias
        path = os.path.join(OUT, f"{name}.npz")
        np.savez_compressed(path, **arrs)
        print(f"{name}: B={B} L={L} K={K} d={d} Dc={Dc} C={C} {score_type} bias={use_bias} -> "
              f"{os.path.getsize(path) / 1e6:.2f} MB; metrics={ {k: round(float(v), 5) for k, v in m.items()} }")

    # config 1 (MIND-demo shape): 200 impressions, history 20, K 4, d 64, npratio 4
    run_case("cfg1_demo", B=200, L=20, K=4, d=64, Dc=32, C=5, seed=36)
    # config 3 slice (MIND-large shape)
    run_case("cfg3_slice", B=4, L=50, K=32, d=768, Dc=200, C=40, seed=1)
    # config 2 slice (MIND-small shape)
    run_case("cfg2_slice", B=6, L=50, K=32, d=256, Dc=200, C=40, seed=2)
    # aggregation variants
    run_case("edge_max", B=24, L=16, K=8, d=128, Dc=48, C=7, score_type="max", seed=3)
    run_case("edge_mean", B=24, L=16, K=8, d=128, Dc=48, C=7, score_type="mean", seed=4)
    # empty (all-pad) and full histories, mixed
    run_case("edge_hist", B=8, L=24, K=16, d=64, Dc=40, C=6, seed=5,
             hist_len=[0, 24, 0, 1, 23, 24, 12, 0])
    # L=1, C=2 and K=32 at odd L / C
    run_case("edge_L1", B=16, L=1, K=32, d=64, Dc=32, C=2, seed=6)
    run_case("edge_oddLC", B=10, L=37, K=32, d=192, Dc=72, C=33, seed=7)
    # category-aware bias on (model.py:113-122)
    run_case("edge_bias", B=12, L=20, K=8, d=64, Dc=32, C=5, seed=8, use_bias=True)
    # exact score ties (unstable argsort in mrr/ndcg, stable sort in hit@k)
    run_case("edge_ties", B=40, L=10, K=4, d=64, Dc=16, C=8, seed=9, ties=True)
    # reference-legal shapes past the fused kernels' K <= 32 / L <= 64 (the wide path): K = 64 with a
    # 120-long history, K = 40 (not a multiple of 16) with L = 80, and the bias path at L = 70
    run_case("wide_k64_l120", B=6, L=120, K=64, d=256, Dc=64, C=12, seed=10)
    run_case("wide_k40_l80_max", B=8, L=80, K=40, d=128, Dc=48, C=9, score_type="max", seed=11)
    run_case("wide_k36_l70_bias_mean", B=6, L=70, K=36, d=64, Dc=32, C=70, score_type="mean", seed=12,
             use_bias=True, hist_len=[0, 70, 69, 1, 35, 70])
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
