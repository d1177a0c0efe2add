"""Benchmark: scored (user, candidate) pairs/s of the MINER scoring path on MI355X.

    python bench.py [--gpus N --steps K --warmup W]            # N=1 default
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json metric, config 3 "MIND-large shape"): history L=50, K=32 interests,
d=768, Dc=200, C=40 candidates per impression, bf16 operands / fp32 accumulation. Impressions
are given as news ids over a 104,000 x 768 news table (the reference's eval input: reader.py
feeds news ids, the news encoder's output is a per-news table), ids and table resident in HBM.
One step = the per-news precompute over the WHOLE table (news_pre: tanh(E·W1ᵀ)·Qᵀ and E·W2ᵀ,
SURVEY.md §8 f2) + one launch of the scoring kernel (news_score) over ``--batch`` impressions per
GPU; impressions are sharded across ranks with no collective on the data path (weak scaling);
``value`` = pairs scored by all ranks / max-over-ranks time.

Also reported (same JSON line): the HBM roofline of the scoring kernel (algorithmic bytes per
launch over its HIP-event launch time, on the stream it runs on), the precompute's time, the fp32
parity mode, the fused dense-row kernel (``--workload config3-dense``: weights per impression, rows
given as [B, L, d] tensors) for comparison, and the CPU baseline (the oracle — a restatement of
the reference's torch CPU path — timed on this host's cores over a bounded sample) at N=1.

``--workload corpus`` measures BASELINE config 5 (every user against a 200k-news table, history 200,
K=64, fp16, fused click score + top-k); ``--workload fastformer`` measures
BASELINE config 4 instead (the FastFormer user encoder,
SURVEY.md §8 f3): 50,000 impressions per GPU per step, history 50, 40 candidates, hidden 256,
bf16, same JSON contract.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

L, K, D, DC, C = 50, 32, 768, 200, 40
PEAK_BF16_TFLOPS = 2500.0      # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_F32_TFLOPS = 157.3        # fp32 MFMA / vector
PEAK_HBM_GBS = 8000.0          # HBM3E spec


def flops_per_impression(L, K, d, Dc, C):
    """Algorithmic FLOPs: 2LdDc + 2LDcK + 2KLd + 2Kd² + 4CdK + 2CK."""
    return 2 * L * d * Dc + 2 * L * Dc * K + 2 * K * L * d + 2 * K * d * d + 4 * C * d * K + 2 * C * K


def bytes_per_impression(L, d, C, elem):
    """Algorithmic HBM bytes: (L + C)·d·s + L (mask) + 4C (fp32 scores); weights excluded."""
    return (L + C) * d * elem + L + 4 * C


def cpu_baseline(seconds: float = 15.0):
    """Oracle (torch fp32 CPU restatement of model.py:159-216,127) on host cores."""
    from miner_amd import synthetic
    from oracle import miner_oracle as orc
    threads = torch.get_num_threads()
    imp = synthetic.impressions(36, 0, 512, L=L, d=D, C=C, device="cpu")
    W1, Q, W2 = synthetic.init_weights(36, D, DC, K)
    bs = 64
    # batched layout: 64 impressions x 40 candidates per call
    with torch.no_grad():
        orc.score_torch(imp.history[:bs], imp.his_mask[:bs], imp.candidates[:bs], W1, Q, W2)  # warmup
        pairs, t0, i = 0, time.perf_counter(), 0
        while True:
            lo = (i * bs) % 512
            orc.score_torch(imp.history[lo:lo + bs], imp.his_mask[lo:lo + bs], imp.candidates[lo:lo + bs], W1, Q, W2)
            pairs += bs * C
            i += 1
            el = time.perf_counter() - t0
            if el > seconds and i >= 2:
                break
        batched = pairs / el
        # reference-faithful layout: one candidate per sample, eval_batch_size 32
        n_imp = 0
        t0 = time.perf_counter()
        while True:
            lo = n_imp % 512
            orc.score_per_candidate_torch(imp.history[lo:lo + 2], imp.his_mask[lo:lo + 2],
                                          imp.candidates[lo:lo + 2], W1, Q, W2, batch_size=32)
            n_imp += 2
            el2 = time.perf_counter() - t0
            if el2 > seconds / 3 and n_imp >= 2:
                break
        per_cand = n_imp * C / el2
    return {"value": round(batched, 1), "unit": "pairs/s", "cores": threads, "kind": "port",
            "sample": f"{pairs // C} impressions x {C} candidates (L={L},K={K},d={D},Dc={DC}), fp32, "
                      f"batched 64 impressions/call, {el:.1f}s",
            "per_candidate_value": round(per_cand, 1),
            "per_candidate_sample": f"{n_imp} impressions, one candidate per sample, batch 32 "
                                    f"(reader.py:376-379 layout), {el2:.1f}s"}


FF_L, FF_C, FF_H, FF_B = 50, 40, 256, 50000


def ff_flops_per_impression(L=FF_L, C=FF_C, H=FF_H):
    """Algorithmic FLOPs of the FastFormer user encoder + click predictor (model.py:345-545, :322):
    per layer 6 H x H linears + 2 H -> 16 head projections + the 2 pooled attentions, then the
    pooler (att_fc1, att_fc2, weighted sum) and C dot products; the MFMA pad of L to 64 excluded."""
    layer = 6 * 2 * L * H * H + 2 * 2 * L * H * 16 + 2 * 2 * L * H
    return 2 * layer + 2 * L * H * H + 2 * L * H + 2 * L * H + 2 * C * H


def ff_bytes_per_impression(L=FF_L, C=FF_C, H=FF_H, elem=2):
    """Algorithmic HBM bytes: history + candidate rows, mask, fp32 scores (parameters excluded)."""
    return (L + C) * H * elem + L + 4 * C


def ff_cpu_baseline(seconds: float = 15.0):
    """FastFormer oracle (torch fp32 CPU restatement of model.py:345-545, :322) on host cores."""
    from miner_amd import fastformer as ff
    from miner_amd import synthetic
    from oracle import fastformer_oracle as ffo
    threads = torch.get_num_threads()
    blob = synthetic.fastformer_params(0)
    params = {n: t.reshape(shp) for (n, shp), t in
              zip(ff.PARAMS, torch.split(blob, [int(torch.Size(shp).numel()) for _, shp in ff.PARAMS]))}
    g = torch.Generator().manual_seed(1)
    bs = 64
    E = torch.randn(bs, FF_L, FF_H, generator=g) * 0.0625
    M = torch.rand(bs, FF_L, generator=g) > 0.3
    Cd = torch.randn(bs, FF_C, FF_H, generator=g) * 0.0625
    with torch.no_grad():
        ffo.scores(params, E, M, Cd)
        pairs, t0, i = 0, time.perf_counter(), 0
        while True:
            ffo.scores(params, E, M, Cd)
            pairs += bs * FF_C
            i += 1
            el = time.perf_counter() - t0
            if el > seconds and i >= 2:
                break
    return {"value": round(pairs / el, 1), "unit": "pairs/s", "cores": threads, "kind": "port",
            "sample": f"{pairs // FF_C} impressions x {FF_C} candidates (L={FF_L}, hidden {FF_H}), fp32, "
                      f"batched {bs} impressions/call, {el:.1f}s"}


def run_fastformer(args, rank, world, dev):
    """BASELINE config 4: the FastFormer kernel over FF_B resident impressions per GPU per step."""
    from miner_amd import fastformer as ff
    from miner_amd import synthetic
    B = args.batch if args.batch_set else FF_B
    bf = torch.bfloat16
    pool = []
    for p in range(args.pool):
        start = (rank * args.pool + p) * B
        g = torch.Generator().manual_seed(1000 + start)
        lens = torch.randint(0, FF_L + 1, (B,), generator=g)
        mask = (torch.arange(FF_L)[None, :] >= (FF_L - lens)[:, None]).to(dev)
        hist = (torch.randn(B, FF_L, FF_H, generator=g) * 0.0625).to(dev, bf)
        cand = (torch.randn(B, FF_C, FF_H, generator=g) * 0.0625).to(dev, bf)
        pool.append((hist, mask, cand))
    blob = synthetic.fastformer_params(0).to(dev)
    pk16 = ff.pack(blob, bf)
    pk32 = ff.pack(blob, torch.float32)
    torch.cuda.synchronize()

    def step(i):
        hist, mask, cand = pool[i % len(pool)]
        return ff.score(hist, mask, cand, pk16)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        out = step(i)
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    assert torch.isfinite(out).all()
    f32 = None
    if args.fp32_steps > 0:
        hist, mask, cand = pool[0]
        n32 = min(B, 5000)
        h32, c32, m32 = hist[:n32].float(), cand[:n32].float(), mask[:n32]
        ff.score(h32, m32, c32, pk32)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(args.fp32_steps):
            ff.score(h32, m32, c32, pk32)
        b.record(stream)
        torch.cuda.synchronize()
        ms32 = a.elapsed_time(b) / args.fp32_steps
        f32 = {"value": round(n32 * FF_C / (ms32 / 1e3), 1), "unit": "pairs/s", "ms_per_step": round(ms32, 3),
               "impressions": n32,
               "tflops": round(ff_flops_per_impression() * n32 / (ms32 / 1e3) / 1e12, 2)}
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    value = B * FF_C * args.steps * world / elapsed
    fl = ff_flops_per_impression() * B
    by = ff_bytes_per_impression() * B
    tflops = fl / (kern_ms / 1e3) / 1e12
    gbs = by / (kern_ms / 1e3) / 1e9
    roof = {"bound": "mfma", "achieved": round(tflops, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
            "frac": round(tflops / PEAK_BF16_TFLOPS, 4), "traffic": None, "kernel": "ff_fused<bf16>",
            "flops_per_launch": fl, "kernel_ms": round(kern_ms, 4)}
    roof_hbm = {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(gbs / PEAK_HBM_GBS, 4), "algorithmic_bytes_per_launch": by}
    cpu = ff_cpu_baseline(args.cpu_seconds) if (world == 1 and not args.no_cpu) else None
    line = {
        "metric": "(user,candidate) scores/sec, FastFormer user encoder (config 4)",
        "value": round(value, 1), "unit": "pairs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic (seeded config-4-shaped impressions, random-init weights)",
        "config": {"workload": "config 4 FastFormer user encoder", "history": FF_L, "hidden": FF_H,
                   "heads": 16, "layers": 2, "candidates": FF_C, "impressions_per_gpu_per_step": B,
                   "global_batch": B * world,
                   "parallelism": f"dp{world} (impression shards, no data-path collective)"},
        "roofline": roof, "roofline_hbm": roof_hbm, "fp32_parity_mode": f32, "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


N_NEWS = 104_000     # MIND-large-shaped news table (~104k news x 768)
NEWS_B = 131_072     # impressions per GPU per step (news-id input: 47 MB of ids per batch)


def news_bytes_per_impression(L, d, C, K, elem):
    """Algorithmic bytes of the news-path scoring kernel per impression: the gathered history rows
    of the table and of its projection, the candidate rows, the history logit rows (fp32), the ids,
    the mask and the fp32 scores (the per-news precompute is a separate launch)."""
    return 2 * L * d * elem + C * d * elem + L * K * 4 + 4 * L + L + 4 * C + 4 * C


def news_precompute_flops(n_news, d, Dc, K):
    """tanh(E·W1ᵀ)·Qᵀ and E·W2ᵀ over the table (model.py:171-174, :212)."""
    return n_news * (2 * d * Dc + 2 * Dc * K + 2 * d * d)


def load_news_traffic(path, B):
    try:
        with open(path) as f:
            t = json.load(f)
        if t.get("workload") == f"news_L{L}_K{K}_d{D}_C{C}_N{N_NEWS}_bf16" and t.get("batch") == B:
            return t
    except (OSError, ValueError):
        pass
    return None


def news_batch(seed, B, dev):
    """Impressions as news ids (the reference's eval input, reader.py:351-379): history length
    ~ U{0..L}, left-padded with the pad news (row 0, reader.py:101-110, :369); candidates uniform."""
    g = torch.Generator(device=dev).manual_seed(seed)
    lens = torch.randint(0, L + 1, (B,), generator=g, device=dev)
    mask = torch.arange(L, device=dev)[None, :] >= (L - lens)[:, None]
    hid = torch.randint(1, N_NEWS, (B, L), generator=g, device=dev, dtype=torch.int32)
    hid[~mask] = 0
    cid = torch.randint(1, N_NEWS, (B, C), generator=g, device=dev, dtype=torch.int32)
    return hid, mask, cid


def dense_kernel_line(dev, B=32768, steps=5):
    """The fused dense-row kernel (weights per impression, miner_score) on the same shape, for
    comparison: pairs/s and its MFMA fraction."""
    from miner_amd import ops, synthetic
    imp = synthetic.impressions(36, 0, B, L=L, d=D, C=C, device=dev, dtype=torch.bfloat16)
    W1, Q, W2 = synthetic.init_weights(36, D, DC, K, device=dev)
    pw = ops.pack_weights(W1, Q, W2, dtype=torch.bfloat16)
    ops.score(imp.history, imp.his_mask, imp.candidates, pw)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(steps):
        ops.score(imp.history, imp.his_mask, imp.candidates, pw)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / steps
    tf = flops_per_impression(L, K, D, DC, C) * B / (ms / 1e3) / 1e12
    del imp
    return {"kernel": "miner_fused<bf16,full>", "value": round(B * C / (ms / 1e3), 1), "unit": "pairs/s",
            "ms_per_launch": round(ms, 4), "impressions": B, "tflops": round(tf, 2),
            "frac_bf16_peak": round(tf / PEAK_BF16_TFLOPS, 4)}


def auc_parity(nt16, batch, table, W1, Q, W2, dev, n_imp=2048):
    """The metric's "AUC parity vs ref", on a bounded sample of the timed batch (part of the CPU
    baseline leg): scores of the reference CPU path (the oracle: model.py:113-216 as the same torch
    fp32 ops on the host) vs the GPU news path in its fp32 parity mode and in bf16, then the
    reference's metrics (evaluation.py:36-84, via the GPU metrics kernel) over one set of labels:
    Bernoulli(sigmoid(2·z)) of the reference's z-scored scores, with >= 1 click and >= 1 non-click per
    impression (reader.py:374)."""
    try:
        from miner_amd import metrics, news, ops
        from oracle import miner_oracle as orc
        hid, mask, cid = [x[:n_imp] for x in batch]
        t32 = table.float()
        nt32 = news.precompute(t32, ops.pack_weights(W1, Q, W2, dtype=torch.float32))
        s32 = news.score(nt32, hid, mask, cid, validate=False)
        s16 = news.score(nt16, hid, mask, cid, validate=False)
        T = t32.cpu()
        h, c = hid.cpu().long(), cid.cpu().long()
        with torch.no_grad():
            _, ref = orc.score_torch(T[h], mask.cpu(), T[c], W1.cpu(), Q.cpu(), W2.cpu())
        g = torch.Generator().manual_seed(36)
        z = (ref - ref.mean()) / ref.std()
        lab = (torch.rand(ref.shape, generator=g) < torch.sigmoid(2.0 * z)).to(torch.uint8)
        rows = torch.arange(ref.shape[0])
        lab[rows, ref.argmax(1)] = 1
        lab[rows, ref.argmin(1)] = 0
        labd = lab.reshape(-1).to(dev)
        offs = torch.arange(0, (ref.shape[0] + 1) * C, C, dtype=torch.int32, device=dev)
        names = ["auc", "group_auc", "mrr", "ndcg@5", "ndcg@10"]

        def mets(s):
            return metrics.compute_metrics(torch.sigmoid(s.float().reshape(-1).to(dev)), labd, offs, names)

        mr, m32, m16 = mets(ref), mets(s32), mets(s16)
        ok, worst = orc.parity_ok(s32.cpu().numpy(), ref.numpy())

        def r6(m):
            return {k: round(float(v), 6) for k, v in m.items()}

        return {"sample": f"{ref.shape[0]} impressions x {C} candidates of the timed batch (news ids); fp32 "
                          "reference CPU path (oracle) vs the GPU news path; labels ~ Bernoulli(sigmoid(2 z(ref)))",
                "reference_cpu": r6(mr), "gpu_fp32": r6(m32), "gpu_bf16": r6(m16),
                "max_abs_metric_delta_fp32": float(max(abs(m32[k] - mr[k]) for k in mr)),
                "max_abs_metric_delta_bf16": float(max(abs(m16[k] - mr[k]) for k in mr)),
                "fp32_scores_within_parity_tol": ok, "fp32_worst_frac_of_tol": round(worst, 4)}
    except Exception as e:  # a reporting leg: it never takes the bench line down
        return {"error": f"{type(e).__name__}: {e}"}


def run_news(args, rank, world, dev):
    """BASELINE config 3 on the news-id input: every step recomputes the per-news
    precompute over the whole table (news_pre) and scores a batch of impressions (news_score)."""
    from miner_amd import news, ops, synthetic
    B = args.batch if args.batch_set else NEWS_B
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(36)
    table = (torch.randn((N_NEWS, D), generator=g, device=dev) / D ** 0.5).to(bf)
    W1, Q, W2 = synthetic.init_weights(36, D, DC, K, device=dev)
    pw16 = ops.pack_weights(W1, Q, W2, dtype=bf)        # once per model, outside the timed region
    pool = [news_batch(36 + (rank * args.pool + p) * B, B, dev) for p in range(args.pool)]
    nt = news.precompute(table, pw16)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)

    def step(i, ev=None):
        nonlocal nt
        hid, mask, cid = pool[i % len(pool)]
        if ev is not None:
            ev[0].record(stream)
        nt = news.precompute(table, pw16, out=nt)
        if ev is not None:
            ev[1].record(stream)
        out = news.score(nt, hid, mask, cid, validate=False)
        if ev is not None:
            ev[2].record(stream)
        return out

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        out = step(i, ev[i])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    pre_ms = sum(e[0].elapsed_time(e[1]) for e in ev) / args.steps
    kern_ms = sum(e[1].elapsed_time(e[2]) for e in ev) / args.steps
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    assert torch.isfinite(out).all()

    # fp32 parity mode of the same path (fewer steps; 32k impressions)
    f32 = None
    if args.fp32_steps > 0:
        n32 = min(B, 32768)
        hid, mask, cid = [x[:n32] for x in pool[0]]
        t32 = table.float()
        pw32 = ops.pack_weights(W1, Q, W2, dtype=torch.float32)
        nt32 = news.precompute(t32, pw32)
        news.score(nt32, hid, mask, cid, validate=False)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(args.fp32_steps):
            nt32 = news.precompute(t32, pw32, out=nt32)
            news.score(nt32, hid, mask, cid, validate=False)
        b.record(stream)
        torch.cuda.synchronize()
        ms32 = a.elapsed_time(b) / args.fp32_steps
        f32 = {"value": round(n32 * C / (ms32 / 1e3), 1), "unit": "pairs/s", "ms_per_step": round(ms32, 3),
               "impressions": n32, "note": "news path, fp32 operands and arithmetic (the parity mode)"}
        del t32, nt32
    dense = None
    if world == 1 and not args.no_dense:
        dense = dense_kernel_line(dev)

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    value = B * C * args.steps * world / elapsed
    by = news_bytes_per_impression(L, D, C, K, 2) * B
    gbs = by / (kern_ms / 1e3) / 1e9
    traffic = load_news_traffic(args.news_traffic, B)
    roof = {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(gbs / PEAK_HBM_GBS, 4),
            "traffic": traffic.get("hbm_bytes_per_launch") if traffic else None,
            "kernel": "news_score<bf16,weighted>", "algorithmic_bytes_per_launch": by,
            "kernel_ms": round(kern_ms, 4),
            "note": "algorithmic bytes = gathered rows (history of the table and of its projection, "
                    "candidates) + logit rows + ids + mask + scores; traffic = PMC HBM bytes per launch "
                    "(rows re-read by other impressions hit L2 / the Infinity Cache)"}
    pre_fl = news_precompute_flops(N_NEWS, D, DC, K)
    pre = {"kernel": "news_pre2<bf16> (GEMM-shaped)", "ms": round(pre_ms, 4), "flops": pre_fl,
           "tflops": round(pre_fl / (pre_ms / 1e3) / 1e12, 2),
           "frac_bf16_peak": round(pre_fl / (pre_ms / 1e3) / 1e12 / PEAK_BF16_TFLOPS, 4)}
    cpu = cpu_baseline(args.cpu_seconds) if (world == 1 and not args.no_cpu) else None
    auc = auc_parity(nt, pool[0], table, W1, Q, W2, dev) if (world == 1 and not args.no_cpu) else None
    line = {
        "metric": "(user,candidate) scores/sec at history=50,K=32,d=768; AUC parity vs ref",
        "value": round(value, 1), "unit": "pairs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic (seeded MIND-large-shaped impressions as news ids over a random news table; "
                "random-init weights)",
        "config": {"workload": "config 3 MIND-large shape, news-id input (per step: per-news precompute "
                               "over the whole table + scoring)",
                   "history": L, "K": K, "d": D, "Dc": DC, "candidates": C, "news_table": N_NEWS,
                   "impressions_per_gpu_per_step": B, "global_batch": B * world,
                   "parallelism": f"dp{world} (impression shards, no data-path collective)"},
        "roofline": roof, "precompute": pre, "fp32_parity_mode": f32, "dense_rows_kernel": dense,
        "cpu_baseline": cpu, "auc_parity": auc,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


C5_L, C5_K, C5_N, C5_U, C5_TOPK = 200, 64, 200_000, 2048, 100


def corpus_cpu_baseline(seconds: float = 10.0):
    """Config-5 oracle (the reference's encoder + click score restated in torch fp32 on the CPU,
    oracle/corpus_oracle.py) on host cores: 8 users against news chunks of 4096 until `seconds`."""
    from miner_amd import synthetic
    from oracle import corpus_oracle as co
    threads = torch.get_num_threads()
    g = torch.Generator().manual_seed(5)
    U = 8
    news = torch.randn((16384, D), generator=g) / D ** 0.5
    E = news[torch.randint(0, 16384, (U, C5_L), generator=g)]
    mask = torch.rand((U, C5_L), generator=g) > 0.2
    W1, Q, W2 = synthetic.init_weights(5, D, DC, C5_K)
    with torch.no_grad():
        t0 = time.perf_counter()
        mui, proj = co.encode(E, mask, W1, Q, W2)
        pairs, i = 0, 0
        while True:
            lo = (i * 4096) % 16384
            co.corpus_scores(mui, proj, news[lo:lo + 4096])
            pairs += U * 4096
            i += 1
            el = time.perf_counter() - t0
            if el > seconds and i >= 2:
                break
    return {"value": round(pairs / el, 1), "unit": "(user,news) pairs/s", "cores": threads, "kind": "port",
            "sample": f"{U} users (history {C5_L}, K={C5_K}, d={D}) encoded and scored against {pairs // U} news "
                      f"rows in chunks of 4096, fp32, {el:.1f}s (top-k selection not included)"}


def run_corpus(args, rank, world, dev):
    """BASELINE config 5: every user against the whole 200k-news table (fp16), history 200, K=64,
    fused click score + running top-k (never materialising the U x N scores). One step = encode
    ``--batch`` users (default 2048) per GPU and rank them against the table; users shard over
    ranks (weak scaling, no data-path collective)."""
    from miner_amd import corpus, synthetic
    U = args.batch if args.batch_set else C5_U
    dt = torch.float16
    g = torch.Generator(device=dev).manual_seed(5)
    table = (torch.randn((C5_N, D), generator=g, device=dev) / D ** 0.5).to(dt)
    W1, Q, W2 = synthetic.init_weights(5, D, DC, C5_K, device=dev)
    pk = corpus.pack_encoder(W1, Q, W2, dtype=dt)
    pool = []
    for p in range(args.pool):
        gg = torch.Generator(device=dev).manual_seed(1000 + rank * args.pool + p)
        hid = torch.randint(0, C5_N, (U, C5_L), generator=gg, device=dev, dtype=torch.int32)
        lens = torch.randint(1, C5_L + 1, (U,), generator=gg, device=dev)
        mask = torch.arange(C5_L, device=dev)[None, :] >= (C5_L - lens)[:, None]
        pool.append((hid, mask))
    stream = torch.cuda.current_stream(dev)

    def step(i, ev=None):
        hid, mask = pool[i % len(pool)]
        if ev is not None:
            ev[0].record(stream)
        mui, proj = corpus.encode_users(table, mask, pk, his_ids=hid)
        if ev is not None:
            ev[1].record(stream)
        out = corpus.rank_topk(mui, proj, table, C5_TOPK)
        if ev is not None:
            ev[2].record(stream)
        return out

    steps = args.steps if args.steps_set else 5
    warm = args.warmup if args.warmup_set else 1
    for i in range(warm):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    t0 = time.perf_counter()
    for i in range(steps):
        out = step(i, ev[i])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    enc_ms = sum(e[0].elapsed_time(e[1]) for e in ev) / steps
    rank_ms = sum(e[1].elapsed_time(e[2]) for e in ev) / steps
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    assert torch.isfinite(out[0]).all()
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    pairs = U * C5_N
    fl = pairs * 4 * C5_K * D            # M = mui·e and Lg = proj·e per (user, news) pair (model.py:127, :213)
    tflops = fl / (rank_ms / 1e3) / 1e12
    enc_fl = U * (2 * C5_L * D * DC + 2 * C5_L * DC * C5_K + 2 * C5_K * C5_L * D + 2 * C5_K * D * D)
    line = {
        "metric": "(user,news) click scores/sec, full-corpus ranking with fused top-k (config 5)",
        "value": round(pairs * steps * world / elapsed, 1), "unit": "pairs/s", "n_gpus": world, "steps": steps,
        "warmup": warm, "ms_per_step": round(elapsed / steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "fp16",
        "data": "synthetic (random news table and user histories, random-init weights)",
        "config": {"workload": "config 5 full-corpus ranking stress", "news": C5_N, "history": C5_L, "K": C5_K,
                   "d": D, "Dc": DC, "topk": C5_TOPK, "users_per_gpu_per_step": U, "global_users_per_step": U * world,
                   "parallelism": f"dp{world} (user shards, news table replicated, no data-path collective)"},
        "roofline": {"bound": "mfma", "achieved": round(tflops, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(tflops / PEAK_BF16_TFLOPS, 4), "traffic": None, "kernel": "rk_fused<fp16>",
                     "flops_per_launch": fl, "kernel_ms": round(rank_ms, 3)},
        "encoder": {"kernel": "ue_fused<fp16>", "ms": round(enc_ms, 3),
                    "tflops": round(enc_fl / (enc_ms / 1e3) / 1e12, 2)},
        "cpu_baseline": corpus_cpu_baseline(min(args.cpu_seconds, 10.0)) if (world == 1 and not args.no_cpu) else None,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def load_traffic(path):
    try:
        with open(path) as f:
            t = json.load(f)
        if t.get("workload") == f"L{L}_K{K}_d{D}_Dc{DC}_C{C}_bf16":
            return t
    except (OSError, ValueError):
        pass
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="config3", choices=["config3", "config3-dense", "fastformer", "corpus"])
    ap.add_argument("--batch", type=int, default=None, help="impressions per GPU per step")
    ap.add_argument("--pool", type=int, default=2, help="distinct resident batches per GPU")
    ap.add_argument("--fp32-steps", type=int, default=2)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--news-traffic", default=os.path.join(ROOT, "profiles", "pmc_traffic_news.json"))
    ap.add_argument("--no-dense", action="store_true", help="skip the dense-row kernel comparison")
    args = ap.parse_args()
    args.batch_set = args.batch is not None
    args.steps_set = "--steps" in sys.argv
    args.warmup_set = "--warmup" in sys.argv
    if args.batch is None:
        args.batch = 32768

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    if args.workload == "fastformer":
        return run_fastformer(args, rank, world, dev)
    if args.workload == "config3":
        return run_news(args, rank, world, dev)
    if args.workload == "corpus":
        return run_corpus(args, rank, world, dev)

    from miner_amd import ops, synthetic

    B = args.batch
    bf = torch.bfloat16
    pool = []
    for p in range(args.pool):
        start = (rank * args.pool + p) * B      # each rank scores its own shard
        imp = synthetic.impressions(36, start, B, L=L, d=D, C=C, device=dev, dtype=bf)
        pool.append(imp)
    W1, Q, W2 = synthetic.init_weights(36, D, DC, K, device=dev)
    pw16 = ops.pack_weights(W1, Q, W2, dtype=bf)        # once per model, outside the timed region
    pw32 = ops.pack_weights(W1, Q, W2, dtype=torch.float32)
    out = torch.empty((B, C), device=dev, dtype=torch.float32)
    torch.cuda.synchronize()

    def step(i):
        imp = pool[i % len(pool)]
        return ops.score(imp.history, imp.his_mask, imp.candidates, pw16)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        out = step(i)
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    assert torch.isfinite(out).all()

    # fp32 parity mode on the same impressions (fewer steps: it runs at the fp32 MFMA rate)
    f32 = None
    if args.fp32_steps > 0:
        imp = pool[0]
        h32, c32 = imp.history.float(), imp.candidates.float()
        ops.score(h32, imp.his_mask, c32, pw32)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(args.fp32_steps):
            ops.score(h32, imp.his_mask, c32, pw32)
        b.record(stream)
        torch.cuda.synchronize()
        ms32 = a.elapsed_time(b) / args.fp32_steps
        f32 = {"value": round(B * C / (ms32 / 1e3), 1), "unit": "pairs/s", "ms_per_step": round(ms32, 3),
               "tflops": round(flops_per_impression(L, K, D, DC, C) * B / (ms32 / 1e3) / 1e12, 2),
               "frac_fp32_peak": round(flops_per_impression(L, K, D, DC, C) * B / (ms32 / 1e3) / 1e12 / PEAK_F32_TFLOPS, 4)}
        del h32, c32

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    pairs_total = B * C * args.steps * world
    value = pairs_total / elapsed
    fl = flops_per_impression(L, K, D, DC, C) * B
    by = bytes_per_impression(L, D, C, 2) * B
    tflops = fl / (kern_ms / 1e3) / 1e12
    gbs = by / (kern_ms / 1e3) / 1e9
    traffic = load_traffic(args.traffic)
    traffic_bytes, mfma_busy = None, None
    if traffic and traffic.get("batch") == B:
        traffic_bytes = traffic.get("hbm_bytes_per_launch")
        mfma_busy = traffic.get("mfma_busy_frac")
    roof = {"bound": "mfma", "achieved": round(tflops, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
            "frac": round(tflops / PEAK_BF16_TFLOPS, 4), "traffic": traffic_bytes,
            "kernel": "miner_fused<bf16,full>", "flops_per_launch": fl, "kernel_ms": round(kern_ms, 4),
            "mfma_busy_pmc": mfma_busy}
    roof_hbm = {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(gbs / PEAK_HBM_GBS, 4), "algorithmic_bytes_per_launch": by,
                "traffic": traffic_bytes}
    cpu = None
    if world == 1 and not args.no_cpu:
        cpu = cpu_baseline(args.cpu_seconds)
    line = {
        "metric": "(user,candidate) scores/sec at history=50,K=32,d=768; AUC parity vs ref",
        "value": round(value, 1), "unit": "pairs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic (seeded MIND-large-shaped impressions, random-init weights)",
        "config": {"workload": "config 3 MIND-large shape", "history": L, "K": K, "d": D, "Dc": DC,
                   "candidates": C, "impressions_per_gpu_per_step": B, "global_batch": B * world,
                   "parallelism": f"dp{world} (impression shards, no data-path collective)"},
        "roofline": roof, "roofline_hbm": roof_hbm, "fp32_parity_mode": f32, "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
