"""The evaluation loop of the reference's ``main.py eval`` (src/trainer.py:218-243 Trainer.eval and
:263-300 Trainer._eval), over impressions given as news ids, on the MI355X kernels.

The reference builds one sample per (impression, candidate) and runs the whole Miner per sample
(reader.py:376-379), then groups sigmoid predictions by impression id in Python. Here the news
encoder output is a device table computed once, its per-news products are computed once
(``news.precompute``: tanh(W1 e)·Qᵀ and W2 e), each rank scores its contiguous
shard of impressions with ``news.score`` in large chunks (``ops.score_gather``, the fused kernel
with the weights per impression, where the news path's limits do not hold), and the evaluation
stays on the device
(``metrics.DeviceEvaluator``); the eval loss keeps the reference's per-batch semantics
(``evaluation.eval_loss_partials``). Under torchrun every rank returns the same (loss, scores).

    python -m miner_amd.eval_loop --synthetic --num_impressions 20000            # 1 GPU
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m miner_amd.eval_loop --synthetic ...
    python -m miner_amd.eval_loop --eval_behaviors_path behaviors.tsv --eval_news_path news.tsv \
        --category2id_path category2id.json --news_table news_emb.npy --state_dict miner_state.pt

(files: MIND tsv as the reference reads them; the news table is the news encoder's output, row 0 =
the pad news, row 1+i = news.tsv line i; the state_dict is a reference Miner's, exported with
torch.save(model.state_dict()) — see miner_amd/formats.py).
"""
from __future__ import annotations

import argparse
import logging
import time
from typing import Dict, List, Optional, Tuple

import torch

from . import distributed, evaluation, metrics, news, ops, synthetic

log = logging.getLogger("miner_amd.eval")


def evaluate(packed: "ops.PackedWeights", table: torch.Tensor, beh: "synthetic.Behaviors", metric_names: List[str],
             *, score_type: str = "weighted", evaluation_info=("metrics", "loss"), first_sample: int = 0,
             total_samples: Optional[int] = None, eval_batch_size: int = 32, chunk: int = 32768,
             save_result: bool = False, path: str = None,
             scorer: str = "auto") -> Tuple[Optional[float], Optional[Dict[str, float]]]:
    """Trainer._eval (trainer.py:263-300) for this rank's impressions ``beh`` (a contiguous id range).

    ``first_sample`` / ``total_samples``: global index of this shard's first (impression,
    candidate) sample and the total over all ranks — the eval loss's batch partition
    (eval_batch_size, config/eval_miner.txt:19) is global. ``scorer``: "news" (per-news precompute +
    gather-stream kernel), "gather" (fused kernel, weights per impression) or "auto" (news where
    supported).
    """
    ev = metrics.DeviceEvaluator()
    want_loss = "loss" in evaluation_info
    partial = torch.zeros(2, dtype=torch.float64, device=table.device)
    offs = beh.cand_offsets.to(torch.int64)
    total_samples = int(offs[-1]) if total_samples is None else total_samples
    L, d = beh.his_ids.shape[1], table.shape[1]
    max_c = int((offs[1:] - offs[:-1]).max()) if beh.n else 0
    use_news = scorer == "news" or (scorer == "auto" and news.supported(table.dtype, L, d, packed.Dc, packed.K)
                                    and max_c <= news.MAX_CAND)
    nt = news.precompute(table, packed, with_proj=score_type == "weighted") if use_news else None
    for s in range(0, beh.n, chunk):
        e = min(s + chunk, beh.n)
        o0, o1 = int(offs[s]), int(offs[e])
        c_off = (offs[s:e + 1] - o0).to(torch.int32)
        if use_news:
            out = news.score(nt, beh.his_ids[s:e], beh.his_mask[s:e], beh.cand_ids[o0:o1], score_type=score_type,
                             cand_offsets=c_off, return_user=want_loss, validate=False)
        else:
            out = ops.score_gather(table, beh.his_ids[s:e], beh.his_mask[s:e], beh.cand_ids[o0:o1], packed,
                                   score_type=score_type, cand_offsets=c_off, return_user=want_loss, validate=False)
        scores, mui = out if want_loss else (out, None)
        lab = beh.labels[o0:o1]
        if "metrics" in evaluation_info:
            ev.add(scores, lab, beh.impression_ids[s:e], c_off)
        if want_loss:
            partial += evaluation.eval_loss_partials(mui, scores, lab, first_sample=first_sample + o0,
                                                     total_samples=total_samples, cand_offsets=c_off,
                                                     batch_size=eval_batch_size)
    loss = distributed.reduce_eval_loss(partial) if want_loss else None
    scores = ev.compute_scores(metric_names, save_result, path) if "metrics" in evaluation_info else None
    return loss, scores


def main(argv=None):
    ap = argparse.ArgumentParser(description="MINER evaluation on MI355X (synthetic MIND-shaped data)",
                                 fromfile_prefix_chars="@", allow_abbrev=False)
    ap.add_argument("--synthetic", action="store_true",
                    help="synthetic impressions and random-init weights (no dataset or checkpoint here)")
    ap.add_argument("--eval_behaviors_path")
    ap.add_argument("--eval_news_path")
    ap.add_argument("--category2id_path")
    ap.add_argument("--news_table", help=".npy / .safetensors / weights-only .pt [n_news+1, d]")
    ap.add_argument("--state_dict", help="reference Miner state_dict (torch.save(model.state_dict()))")
    ap.add_argument("--num_impressions", type=int, default=20000)
    ap.add_argument("--num_news", type=int, default=104_151, help="MIND-large has ~104k news")
    ap.add_argument("--his_length", type=int, default=50)
    ap.add_argument("--num_context_codes", type=int, default=32)
    ap.add_argument("--context_code_dim", type=int, default=200)
    ap.add_argument("--embed_dim", type=int, default=768)
    ap.add_argument("--candidates", type=int, default=40)
    ap.add_argument("--ragged", type=int, nargs=2, default=None, metavar=("LO", "HI"))
    ap.add_argument("--score_type", default="weighted", choices=["weighted", "max", "mean"])
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--metrics", nargs="+", default=["auc", "group_auc", "mrr", "ndcg@5", "ndcg@10", "hit@5", "hit@10"])
    ap.add_argument("--evaluation_info", nargs="+", default=["metrics", "loss"])
    ap.add_argument("--eval_batch_size", type=int, default=32)
    ap.add_argument("--seed", type=int, default=36)
    args = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(message)s")

    rank, world, local = distributed.init_from_env()
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    dt = torch.bfloat16 if args.precision == "bf16" else torch.float32
    if args.synthetic:
        table = synthetic.news_table(args.seed, args.num_news, args.embed_dim, device=dev, dtype=dt)
        W1, Q, W2 = synthetic.init_weights(args.seed, args.embed_dim, args.context_code_dim, args.num_context_codes,
                                           device=dev)
        start, count = distributed.shard_range(args.num_impressions, rank, world)
        beh = synthetic.behaviors(args.seed, start, count, L=args.his_length, n_news=args.num_news,
                                  C=args.candidates, ragged=args.ragged, device=dev)
    else:
        from . import formats
        for a in ("eval_behaviors_path", "eval_news_path", "category2id_path", "news_table", "state_dict"):
            if getattr(args, a) is None:
                ap.error(f"--{a} is required without --synthetic")
        news = formats.read_news_tsv(args.eval_news_path, formats.read_category2id(args.category2id_path))
        table = formats.load_news_table(args.news_table).to(dev, dt)
        if table.shape[0] != news.n_rows:
            raise ValueError(f"news table has {table.shape[0]} rows, news.tsv + pad needs {news.n_rows}")
        sd = torch.load(args.state_dict, map_location="cpu", weights_only=True)
        W1, Q = sd["poly_attn.linear.weight"].to(dev), sd["poly_attn.context_codes"].to(dev)
        W2 = sd["target_aware_attn.linear.weight"].to(dev) if args.score_type == "weighted" else None
        every = formats.read_behaviors_tsv(args.eval_behaviors_path, news, args.his_length)
        start, count = distributed.shard_range(every.n, rank, world)
        o = every.cand_offsets
        beh = synthetic.Behaviors(every.his_ids[start:start + count].to(dev), every.his_mask[start:start + count].to(dev),
                                  every.cand_ids[int(o[start]):int(o[start + count])].to(dev),
                                  (o[start:start + count + 1] - o[start]).to(dev),
                                  every.labels[int(o[start]):int(o[start + count])].to(dev),
                                  every.impression_ids[start:start + count].to(dev))
    packed = ops.pack_weights(W1, Q, W2 if args.score_type == "weighted" else None, dtype=dt)
    # global sample offset of this shard (the eval loss's batch partition spans ranks)
    n_mine = torch.tensor([int(beh.cand_offsets[-1])], dtype=torch.float64)
    counts = distributed.all_gather_concat(n_mine.to(distributed._coll_device())).cpu().long().tolist()
    first, total = sum(counts[:rank]), sum(counts)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loss, scores = evaluate(packed, table, beh, args.metrics, score_type=args.score_type,
                            evaluation_info=args.evaluation_info, first_sample=first, total_samples=total,
                            eval_batch_size=args.eval_batch_size)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if rank == 0:
        log.info("Model: Miner (MI355X fused scoring, %s); dataset: %s, %d samples, %d rank(s)",
                 args.precision, "synthetic" if args.synthetic else args.eval_behaviors_path, total, world)
        log.info("----------------  Evaluation phrase  ----------------")
        if loss is not None:
            log.info("Loss %s", loss)
        for m in args.metrics:
            log.info("Metric %s: %s", m, scores[evaluation.metric_key(m)] if scores else None)
        log.info("Evaluation time %.3f s (%.1f M samples/s)", el, total / el / 1e6)
    if world > 1:
        torch.distributed.destroy_process_group()
    return loss, scores


if __name__ == "__main__":
    main()
