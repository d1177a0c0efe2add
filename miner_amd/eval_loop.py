"""``main.py eval`` / ``main.py eval_fastformer`` of the reference on the MI355X kernels.

The evaluation loops (src/trainer.py:218-300 ``Trainer.eval`` / ``_eval`` for Miner,
src/trainer_fastformer.py:250-348 for FastFormer) over impressions given as news ids.

The reference builds one sample per (impression, candidate) and runs the whole model per sample
(src/reader.py:376-379), then groups sigmoid predictions by impression id in Python. Here the news
encoder's output is a device table computed once, and each rank scores its contiguous shard of
impressions in large chunks:

* Miner: the per-news products are computed once (``news.precompute``: tanh(W1 e)·Qᵀ and W2 e,
  SURVEY §8 f2) and ``news.score`` scores the chunk (``ops.score_gather``, the fused kernel with the
  weights per impression, where the news path's limits do not hold). With a category embedding in
  the checkpoint (``use_category_bias``) the bias is per (impression, candidate) as in the
  reference's one-candidate samples (model.py:113-122, :176): every candidate is scored as its own
  sample with its own history softmax.
* FastFormer: ``fastformer.score_gather`` (the fused user encoder + dot products, model.py:318-322).

Metrics stay on the device (``metrics.DeviceEvaluator``; exact global AUC by ``miner_global_auc``),
the eval loss keeps the reference's semantics (Miner: ``Loss.compute_eval_loss`` per batch of
``eval_batch_size`` samples, src/loss.py:68-85; FastFormer: ``compute_vanilla_eval_loss``,
src/loss.py:47-65), and under torchrun every rank returns the same (loss, scores).

Outputs (src/base_trainer.py:80-82, src/trainer.py:288-289, src/evaluation.py:60-82, :173-175):
``<eval_path>/<timestamp>/`` holds ``all.log``, ``args.json``, ``preds.pkl`` and, with
``--save_eval_result``, the per-impression ``<metric>.txt`` files.

    python -m miner_amd.eval_loop eval @config/eval_miner.txt --news_table news_emb.npy
    python -m miner_amd.eval_loop eval_fastformer @config/eval_fastformer.txt --news_table emb256.npy
    python -m miner_amd.eval_loop eval --synthetic --num_impressions 20000           # no dataset here
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m miner_amd.eval_loop eval --synthetic ...

``--saved_model_path`` is a weights-only file holding the model's ``state_dict()`` (or
``{'model': state_dict}``): the reference's checkpoints are pickled whole modules
(src/base_trainer.py:204-235) and are never unpickled here — export ``model.state_dict()`` in the
reference environment. The news table is the news encoder's output, row 0 = the
pad news, row 1+i = news.tsv line i (miner_amd/formats.py).
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import logging
import os
import sys
import time
from datetime import datetime
from typing import Dict, List, Optional, Tuple

import torch

from . import distributed, evaluation, metrics, news, ops, synthetic

log = logging.getLogger("miner_amd.eval")


@dataclasses.dataclass
class CategoryBias:
    """The category bias of a ``use_category_bias`` Miner (model.py:113-122): the cosine of the
    clicked news' and the candidate's category embeddings (utils.py:9-29), as a table over category
    pairs. ``row_category`` maps news-table rows to category ids."""
    row_category: torch.Tensor    # [n_rows] int64
    cos: torch.Tensor             # [n_cat, n_cat] fp32

    @classmethod
    def from_embedding(cls, weight: torch.Tensor, row_category: torch.Tensor) -> "CategoryBias":
        """pairwise_cosine_similarity (utils.py:9-29) of every category pair: x/‖x‖ · (y/‖y‖)ᵀ.
        The pad category's zero embedding gives NaN rows, as in the reference, where they are
        overwritten by the history mask (pad ⇔ masked, entities.py:395)."""
        w = weight.float()
        u = torch.div(w, torch.linalg.norm(w, dim=1, keepdim=True))
        return cls(row_category.to(device=w.device, dtype=torch.int64), torch.matmul(u, u.t()))

    def per_sample(self, his_ids: torch.Tensor, his_mask: torch.Tensor, cand_ids: torch.Tensor) -> torch.Tensor:
        """his_ids / his_mask [N, L] of N one-candidate samples, cand_ids [N] -> his_bias [N, L]."""
        hc = self.row_category[his_ids.long()]
        cc = self.row_category[cand_ids.long()]
        b = self.cos[hc, cc[:, None]]
        return torch.where(his_mask, b, torch.zeros_like(b))     # masked slots: 1e-30 fill in-kernel


def _max_candidates(offs: torch.Tensor, n: int) -> int:
    return int((offs[1:] - offs[:-1]).max()) if n else 0


def evaluate(packed: "ops.PackedWeights", table: torch.Tensor, beh: "synthetic.Behaviors", metric_names: List[str],
             *, score_type: str = "weighted", evaluation_info=("metrics", "loss"), first_sample: int = 0,
             total_samples: Optional[int] = None, eval_batch_size: int = 32, chunk: int = 32768,
             save_result: bool = False, path: str = None, scorer: str = "auto",
             category: Optional[CategoryBias] = None,
             predictions: Optional[list] = None) -> Tuple[Optional[float], Optional[Dict[str, float]]]:
    """Trainer._eval (trainer.py:263-300) for this rank's impressions ``beh`` (a contiguous id range).

    ``first_sample`` / ``total_samples``: global index of this shard's first (impression,
    candidate) sample and the total over all ranks — the eval loss's batch partition
    (eval_batch_size, config/eval_miner.txt:19) is global. ``scorer``: "news" (per-news precompute +
    gather-stream kernel), "gather" (fused kernel, weights per impression) or "auto" (news where
    supported). ``category``: per-(impression, candidate) category bias (model.py:113-122).
    ``predictions``: a list that receives (probabilities, impression ids, offsets) per chunk, for
    preds.pkl.
    """
    ev = metrics.DeviceEvaluator()
    want_loss = "loss" in evaluation_info
    partial = torch.zeros(2, dtype=torch.float64, device=table.device)
    offs = beh.cand_offsets.to(torch.int64)
    total_samples = int(offs[-1]) if total_samples is None else total_samples
    L, d = beh.his_ids.shape[1], table.shape[1]
    max_c = 1 if category is not None else _max_candidates(offs, beh.n)
    news_ok = news.path_supported(table.dtype, L, d, packed.Dc, packed.K, n_news=table.shape[0])
    news_wide = news.wide_supported(table.dtype, L, d, packed.Dc, packed.K,
                                    n_news=table.shape[0])   # K > 32 or L > 64 (news_score_x2w)
    if scorer == "news":
        if not news_ok:
            raise ValueError(f"scorer='news': the news path does not support L={L} d={d} K={packed.K}")
        if max_c > news.MAX_CAND:
            raise ValueError(f"scorer='news': an impression has {max_c} candidates (at most {news.MAX_CAND})")
    use_news = scorer == "news" or (scorer == "auto" and news_ok and max_c <= news.MAX_CAND)
    nt = news.precompute(table, packed, with_proj=score_type == "weighted") if use_news else None
    # fp32 pair-plane tables: the eval loss's disagreement is formed inside the scoring kernel (no mui)
    fused_loss = want_loss and use_news and nt.x2 is not None and news.x2_enabled() and not news_wide
    # with the per-candidate bias every candidate is one sample: chunk by samples (mui is [N, K, d])
    mc = max(_max_candidates(offs, beh.n), 1)
    step = chunk if category is None else max(1, chunk // mc)
    # one mui buffer for every chunk of the eval loss (the news kernel writes it; 3.2 GB at 32k x 32 x 768);
    # with the per-candidate bias a chunk holds up to step x mc one-candidate samples
    rows = min(step, beh.n) if category is None else min(step * mc, int(offs[-1]))
    mui_buf = torch.empty((max(rows, 1), packed.K, d), device=table.device, dtype=torch.float32) \
        if (want_loss and use_news and not fused_loss) else None
    for s in range(0, beh.n, step):
        e = min(s + step, beh.n)
        o0, o1 = int(offs[s]), int(offs[e])
        c_off = (offs[s:e + 1] - o0).to(torch.int32)
        his, msk, cid = beh.his_ids[s:e], beh.his_mask[s:e], beh.cand_ids[o0:o1]
        bias, s_off = None, c_off
        if category is not None:          # one sample per (impression, candidate): reader.py:376-379
            sizes = torch.diff(c_off.to(torch.int64))
            his = torch.repeat_interleave(his, sizes, dim=0)
            msk = torch.repeat_interleave(msk, sizes, dim=0)
            bias = category.per_sample(his, msk, cid)
            s_off = torch.arange(o1 - o0 + 1, device=table.device, dtype=torch.int32)
        dis = None
        if use_news and fused_loss:
            scores, dis = news.score(nt, his, msk, cid, score_type=score_type, cand_offsets=s_off, his_bias=bias,
                                     validate=False, disagreement=True)
            mui = None
        elif use_news:
            out = news.score(nt, his, msk, cid, score_type=score_type, cand_offsets=s_off, his_bias=bias,
                             return_user=want_loss, validate=False, user_out=mui_buf)
            scores, mui = out if want_loss else (out, None)
        else:
            out = ops.score_gather(table, his, msk, cid, packed, score_type=score_type, cand_offsets=s_off,
                                   his_bias=bias, return_user=want_loss, validate=False)
            scores, mui = out if want_loss else (out, None)
        lab = beh.labels[o0:o1]
        if "metrics" in evaluation_info:
            ev.add(scores, lab, beh.impression_ids[s:e], c_off)
        if predictions is not None and "metrics" in evaluation_info:
            # SlowEvaluator.eval_batch runs only with 'metrics' (trainer.py:286-289): a loss-only eval
            # writes an empty preds.pkl, as the reference's
            predictions.append((torch.sigmoid(scores.float()), beh.impression_ids[s:e], c_off))
        if want_loss:
            partial += evaluation.eval_loss_partials(mui, scores, lab, first_sample=first_sample + o0,
                                                     total_samples=total_samples, cand_offsets=s_off,
                                                     batch_size=eval_batch_size, dis=dis)
    loss = distributed.reduce_eval_loss(partial) if want_loss else None
    scores = ev.compute_scores(metric_names, save_result, path) if "metrics" in evaluation_info else None
    return loss, scores


def vanilla_eval_loss_partials(scores: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """Loss.compute_vanilla_eval_loss (src/loss.py:47-65) summed over the eval batches
    (src/trainer_fastformer.py:320-341): per one-candidate sample -logsigmoid(score)·label, so the
    batch partition does not matter. Returns float64 [numerator, positives]."""
    s = scores.reshape(-1).double()
    lab = labels.reshape(-1).to(s.device).double()
    return torch.stack([(-torch.nn.functional.logsigmoid(s) * lab).sum(), lab.sum()])


def evaluate_fastformer(packed, table: torch.Tensor, beh: "synthetic.Behaviors", metric_names: List[str], *,
                        evaluation_info=("metrics", "loss"), chunk: int = 32768, save_result: bool = False,
                        path: str = None, predictions: Optional[list] = None
                        ) -> Tuple[Optional[float], Optional[Dict[str, float]]]:
    """trainer_fastformer.Trainer._eval (src/trainer_fastformer.py:299-348) for this rank's impressions:
    FastformerEncoder over the history rows, scores = candidates · user (model.py:318-322),
    eval loss = Loss.compute_vanilla_eval_loss (src/loss.py:47-65). The user vector does not depend
    on the candidate, so scoring each impression once equals the reference's one-candidate samples."""
    from . import fastformer as ff
    ev = metrics.DeviceEvaluator()
    want_loss = "loss" in evaluation_info
    partial = torch.zeros(2, dtype=torch.float64, device=table.device)
    offs = beh.cand_offsets.to(torch.int64)
    for s in range(0, beh.n, chunk):
        e = min(s + chunk, beh.n)
        o0, o1 = int(offs[s]), int(offs[e])
        c_off = (offs[s:e + 1] - o0).to(torch.int32)
        scores = ff.score_gather(table, beh.his_ids[s:e], beh.his_mask[s:e], beh.cand_ids[o0:o1], packed,
                                 cand_offsets=c_off, validate=False)
        lab = beh.labels[o0:o1]
        if "metrics" in evaluation_info:
            ev.add(scores, lab, beh.impression_ids[s:e], c_off)
        if predictions is not None and "metrics" in evaluation_info:     # trainer_fastformer.py:325-337
            predictions.append((torch.sigmoid(scores.float()), beh.impression_ids[s:e], c_off))
        if want_loss:
            partial += vanilla_eval_loss_partials(scores, lab)
    loss = distributed.reduce_eval_loss(partial) if want_loss else None
    scores = ev.compute_scores(metric_names, save_result, path) if "metrics" in evaluation_info else None
    return loss, scores


# ---------------------------------------------------------------------------------------------
# command line: main.py eval / eval_fastformer (arguments.py:11-43)
# ---------------------------------------------------------------------------------------------
MODES = ("eval", "eval_fastformer")


def convert_arg_line_to_args(arg_line):
    """Argument-file lines as src/utils.py:67-83 reads them: '#' comments and blank lines skipped,
    whitespace-separated tokens."""
    arg_line = arg_line.strip()
    if arg_line.startswith("#") or arg_line == "":
        return []
    return [a for a in arg_line.split() if a.strip()]


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description="MINER / FastFormer evaluation on MI355X (main.py eval)",
                                 fromfile_prefix_chars="@", allow_abbrev=False)
    ap.convert_arg_line_to_args = convert_arg_line_to_args
    # _add_common_arguments (arguments.py:28-45)
    ap.add_argument("--model_name", type=str, help="Name of the model")
    ap.add_argument("--pretrained_tokenizer", type=str, help="(news encoder side; unused: the table is given)")
    ap.add_argument("--user2id_path", type=str, help="(unused by the scoring path)")
    ap.add_argument("--category2id_path", type=str, help="Path to the category dictionary")
    ap.add_argument("--category_embed_path", type=str, default=None,
                    help="ignored, as in the reference (utils.load_embed returns None, utils.py:32-34)")
    ap.add_argument("--max_title_length", type=int, help="(news encoder side; unused)")
    ap.add_argument("--max_sapo_length", type=int, help="(news encoder side; unused)")
    ap.add_argument("--his_length", type=int, default=50, help="Max number of user click history")
    ap.add_argument("--seed", type=int, default=36, help="Seed value (synthetic data)")
    ap.add_argument("--save_eval_result", action="store_true", help="write the per-impression <metric>.txt files")
    ap.add_argument("--metrics", type=str, nargs="+",
                    default=["auc", "group_auc", "mrr", "ndcg@5", "ndcg@10", "hit@5", "hit@10"])
    ap.add_argument("--evaluation_info", type=str, nargs="+", choices=["loss", "metrics"], default=["metrics", "loss"])
    ap.add_argument("--device", type=str, default="cuda:0", help="device (torchrun: LOCAL_RANK wins)")
    # add_eval_arguments (arguments.py:11-25)
    ap.add_argument("--saved_model_path", type=str,
                    help="weights-only file with the model's state_dict() (or {'model': state_dict})")
    ap.add_argument("--data_name", type=str, help="Name of the eval dataset")
    ap.add_argument("--eval_behaviors_path", type=str, help="behaviors.tsv of the evaluation")
    ap.add_argument("--eval_news_path", type=str, help="news.tsv of the evaluation")
    ap.add_argument("--fast_eval", action="store_true",
                    help="refused: the reference's FastEvaluator has no save_predictions (trainer.py:288-289)")
    ap.add_argument("--eval_batch_size", type=int, default=32, help="samples per batch of the eval loss partition")
    ap.add_argument("--dataloader_num_workers", type=int, help="(no DataLoader: ids and table are on the device)")
    ap.add_argument("--dataloader_pin_memory", action="store_true", help="(no DataLoader)")
    ap.add_argument("--eval_path", type=str, default="eval", help="directory of the evaluation outputs")
    # this implementation
    ap.add_argument("--news_table", help="the news encoder's output [n_news+1, d] (.npy / .safetensors / "
                                         "weights-only .pt), row 0 = the pad news")
    ap.add_argument("--state_dict", help="alias of --saved_model_path")
    ap.add_argument("--score_type", default=None, choices=["weighted", "max", "mean"],
                    help="Miner aggregation (default: 'weighted' when the state_dict has target_aware_attn)")
    ap.add_argument("--precision", default="fp32", choices=["fp32", "bf16"],
                    help="fp32 = the reference's arithmetic (parity mode); bf16 = throughput mode")
    ap.add_argument("--synthetic", action="store_true",
                    help="synthetic impressions and random-init weights (no dataset or checkpoint here)")
    ap.add_argument("--num_impressions", type=int, default=20000)
    ap.add_argument("--num_news", type=int, default=104_151, help="MIND-large has ~104k news")
    ap.add_argument("--num_context_codes", type=int, default=32)
    ap.add_argument("--context_code_dim", type=int, default=200)
    ap.add_argument("--embed_dim", type=int, default=768)
    ap.add_argument("--candidates", type=int, default=40)
    ap.add_argument("--ragged", type=int, nargs=2, default=None, metavar=("LO", "HI"))
    ap.add_argument("--chunk", type=int, default=32768, help="impressions per kernel launch")
    return ap


def _load_state_dict(path: str) -> Dict[str, torch.Tensor]:
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(sd, dict) and "model" in sd and isinstance(sd["model"], dict):
        sd = sd["model"]
    if not isinstance(sd, dict):
        raise ValueError(f"{path}: expected a state_dict (weights-only); reference checkpoints are pickled "
                         "modules — export model.state_dict() first (INTEGRATION.md)")
    return sd


def _setup_output(args, rank: int) -> str:
    """<eval_path>/<timestamp>/ with all.log and args.json (src/base_trainer.py:41-82, :114-122)."""
    stamp = str(datetime.now()).replace(" ", "_").replace(":", "-")[:-7]
    path = os.path.join(args.eval_path, stamp)
    if rank == 0:
        os.makedirs(path, exist_ok=True)
        fh = logging.FileHandler(os.path.join(path, "all.log"))
        fh.setFormatter(logging.Formatter("%(asctime)s [%(levelname)-5.5s] %(message)s"))
        log.addHandler(fh)
        with open(os.path.join(path, "args.json"), mode="w", encoding="utf-8") as f:
            json.dump(vars(args), f, ensure_ascii=False, indent=4, sort_keys=True)
    return path


def _write_predictions(path: str, chunks: list, rank: int) -> Optional[str]:
    """preds.pkl (SlowEvaluator.save_predictions, evaluation.py:173-175) of every rank's samples,
    impression-major in id order, written by rank 0."""
    from . import formats
    if chunks:
        probs = torch.cat([c[0].reshape(-1) for c in chunks])
        ids = torch.cat([torch.repeat_interleave(c[1].to(torch.int64), torch.diff(c[2].to(torch.int64)))
                         for c in chunks])
    else:
        dev = torch.device("cuda", torch.cuda.current_device())
        probs, ids = torch.zeros(0, device=dev), torch.zeros(0, dtype=torch.int64, device=dev)
    probs = distributed.gather_concat_to_root(probs.float())
    ids = distributed.gather_concat_to_root(ids)
    if rank != 0:
        return None
    sizes = torch.ones(ids.numel() + 1, dtype=torch.int64)
    sizes[0] = 0
    return formats.save_predictions(path, probs, ids, torch.cumsum(sizes, 0))


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    mode = argv.pop(0) if argv and argv[0] in MODES else "eval"
    args = build_parser().parse_args(argv)
    args.mode = mode
    if args.fast_eval:
        raise SystemExit("--fast_eval: the reference's `main.py eval --fast_eval` fails at "
                         "evaluator.save_predictions (FastEvaluator has none, src/trainer.py:288-289, "
                         "src/evaluation.py:87-110); use the default SlowEvaluator semantics")
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(message)s")
    rank, world, local = distributed.init_from_env()
    dev = torch.device("cuda", local) if world > 1 or not args.device.startswith("cuda") else torch.device(args.device)
    torch.cuda.set_device(dev)
    dt = torch.bfloat16 if args.precision == "bf16" else torch.float32
    fast = mode == "eval_fastformer"
    path = _setup_output(args, rank)

    model_sd = None
    if not args.synthetic:
        args.saved_model_path = args.saved_model_path or args.state_dict
        for a in ("eval_behaviors_path", "eval_news_path", "category2id_path", "news_table", "saved_model_path"):
            if getattr(args, a) is None:
                raise SystemExit(f"--{a} is required without --synthetic")
        model_sd = _load_state_dict(args.saved_model_path)

    category = None
    if args.synthetic:
        d = 256 if fast else args.embed_dim
        table = synthetic.news_table(args.seed, args.num_news, d, device=dev, dtype=dt)
        start, count = distributed.shard_range(args.num_impressions, rank, world)
        beh = synthetic.behaviors(args.seed, start, count, L=args.his_length, n_news=args.num_news,
                                  C=args.candidates, ragged=args.ragged, device=dev)
    else:
        from . import formats
        nidx = formats.read_news_tsv(args.eval_news_path, formats.read_category2id(args.category2id_path))
        table = formats.load_news_table(args.news_table).to(dev, dt)
        if table.shape[0] != nidx.n_rows:
            raise ValueError(f"news table has {table.shape[0]} rows, news.tsv + pad needs {nidx.n_rows}")
        every = formats.read_behaviors_tsv(args.eval_behaviors_path, nidx, args.his_length)
        start, count = distributed.shard_range(every.n, rank, world)
        o = every.cand_offsets
        beh = synthetic.Behaviors(every.his_ids[start:start + count].to(dev), every.his_mask[start:start + count].to(dev),
                                  every.cand_ids[int(o[start]):int(o[start + count])].to(dev),
                                  (o[start:start + count + 1] - o[start]).to(dev),
                                  every.labels[int(o[start]):int(o[start + count])].to(dev),
                                  every.impression_ids[start:start + count].to(dev))
        if not fast and "category_embedding.weight" in model_sd:     # use_category_bias (model.py:113-122)
            category = CategoryBias.from_embedding(model_sd["category_embedding.weight"].to(dev),
                                                   torch.from_numpy(nidx.category))
    # global sample offset of this shard (the eval loss's batch partition spans ranks)
    n_mine = torch.tensor([int(beh.cand_offsets[-1])], dtype=torch.float64)
    counts = distributed.all_gather_concat(n_mine.to(distributed._coll_device())).cpu().long().tolist()
    first, total = sum(counts[:rank]), sum(counts)
    preds: list = []
    save = args.save_eval_result

    if fast:
        from . import fastformer as ff
        params = synthetic.fastformer_params(args.seed, device=dev) if args.synthetic else \
            ff.flatten_params(model_sd, device=dev)
        packed = ff.pack(params, dt)
        run = lambda: evaluate_fastformer(packed, table, beh, args.metrics, evaluation_info=args.evaluation_info,  # noqa: E731
                                          chunk=args.chunk, save_result=save, path=path, predictions=preds)
        name = args.model_name or "fastformer"
    else:
        if args.synthetic:
            W1, Q, W2 = synthetic.init_weights(args.seed, args.embed_dim, args.context_code_dim,
                                               args.num_context_codes, device=dev)
            score_type = args.score_type or "weighted"
        else:
            W1, Q = model_sd["poly_attn.linear.weight"].to(dev), model_sd["poly_attn.context_codes"].to(dev)
            W2 = model_sd.get("target_aware_attn.linear.weight")
            score_type = args.score_type or ("weighted" if W2 is not None else None)
            if score_type is None:
                raise SystemExit("--score_type max|mean is needed: the state_dict has no target_aware_attn")
            if score_type == "weighted":
                if W2 is None:
                    raise SystemExit("score_type 'weighted' needs target_aware_attn.linear.weight in the state_dict")
                W2 = W2.to(dev)
        packed = ops.pack_weights(W1, Q, W2 if score_type == "weighted" else None, dtype=dt)
        run = lambda: evaluate(packed, table, beh, args.metrics, score_type=score_type,  # noqa: E731
                               evaluation_info=args.evaluation_info, first_sample=first, total_samples=total,
                               eval_batch_size=args.eval_batch_size, chunk=args.chunk, save_result=save,
                               path=path, category=category, predictions=preds)
        name = args.model_name or "Miner"
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loss, scores = run()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    t1 = time.perf_counter()
    preds_path = _write_predictions(path, preds, rank)       # trainer.py:288-289 ("eval" in mode)
    el_w = time.perf_counter() - t1
    if rank == 0:
        log.info("Model: %s (MI355X, %s%s)", name, args.precision, ", per-candidate category bias" if category else "")
        log.info("Dataset: %s", "synthetic" if args.synthetic else (args.data_name or args.eval_behaviors_path))
        log.info("Test dataset: %d samples, %d rank(s)", total, world)
        log.info("----------------  Evaluation phrase  ----------------")
        if loss is not None:
            log.info("Loss %s", loss)
        for m in args.metrics:
            log.info("Metric %s: %s", m, scores[evaluation.metric_key(m)] if scores else None)
        log.info("Evaluation time %.3f s (%.1f M samples/s); outputs in %s (%s, written in %.2f s)", el,
                 total / el / 1e6, path, os.path.basename(preds_path) if preds_path else "-", el_w)
    if world > 1:
        torch.distributed.destroy_process_group()
    return loss, scores


if __name__ == "__main__":
    main()
