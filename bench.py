"""Benchmark: scored (user, candidate) pairs/s of the MINER scoring path on MI355X.

    python bench.py [--gpus N --steps K --warmup W]          # N=1 default; N>1 spawns N ranks itself
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Headline (BASELINE.json metric, config 3 "MIND-large shape": history L=50, K=32 interests, d=768,
Dc=200, C=40 candidates per impression), at the REFERENCE'S precision: fp32 operands and fp32
arithmetic (the reference evaluates in fp32, src/trainer.py:278-281; scores match its CPU path to
1e-5). Impressions are news ids over a 104,000 x 768 news table (the reference's eval input:
reader.py feeds news ids, the news encoder's output is a per-news table), resident in HBM.

One step = the per-news precompute over the WHOLE table (news_pre: tanh(E·W1ᵀ)·Qᵀ and E·W2ᵀ,
SURVEY.md §8 f2) + one launch of the scoring kernel (news_score) over ``--batch`` impressions per
GPU (default 3,000,000 = the whole MIND-large-shaped eval set per GPU); impressions are sharded
across ranks with no collective on the data path (weak scaling); ``value`` = pairs scored by all
ranks / max-over-ranks time.

Also on the line: ``roofline`` of the scoring kernel on SURVEY §8(d)'s algorithmic bytes
((L+C)·d·4 + L + 4C per impression) over its HIP-event launch time, with the MFMA fraction of its
contraction FLOPs beside it and the bytes it really gathers (``gathered_bytes``); the bf16
throughput mode of the same path (``bf16_mode``, with its AUC delta); config 2 (d=256, 50k
impressions); the metric step (per-impression metrics + exact global AUC on the device); the fused
dense-row kernel; the AUC parity of the GPU path against the reference CPU path on a sample; and
the CPU baseline (the oracle — the reference's torch CPU path restated — on this host's cores) at
N=1.

``--workload fastformer`` measures BASELINE config 4 (FastFormer user encoder), ``--workload corpus``
config 5 (full-corpus ranking), ``--workload config3-dense`` the fused kernel on [B, L, d] rows.
``--dry-run`` exercises the launcher and the timing protocol on the CPU (gloo), no kernel.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

L, K, D, DC, C = 50, 32, 768, 200, 40
PEAK_BF16_TFLOPS = 2500.0      # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_F32_TFLOPS = 157.3        # fp32 MFMA = fp32 vector (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0          # HBM3E spec
METRIC = "(user,candidate) scores/sec at history=50,K=32,d=768; AUC parity vs ref"


# ---------------------------------------------------------------------------------------------
# algorithmic work
# ---------------------------------------------------------------------------------------------
def flops_per_impression(L, K, d, Dc, C):
    """Algorithmic FLOPs of the whole path: 2LdDc + 2LDcK + 2KLd + 2Kd² + 4CdK + 2CK."""
    return 2 * L * d * Dc + 2 * L * Dc * K + 2 * K * L * d + 2 * K * d * d + 4 * C * d * K + 2 * C * K


def bytes_per_impression(L, d, C, elem):
    """SURVEY §8(d) algorithmic HBM bytes: (L + C)·d·s + L (mask) + 4C (fp32 scores); weights excluded."""
    return (L + C) * d * elem + L + 4 * C


def news_gathered_bytes(L, d, C, K, elem):
    """Bytes the news-path scoring kernel actually moves per impression: history rows of the table
    AND of its projection (the E·W2ᵀ reformulation's second gather), candidate rows, the history
    logit rows (fp32), ids, mask, fp32 scores. Not the roofline's numerator (that is §8(d))."""
    return 2 * L * d * elem + C * d * elem + L * K * 4 + 4 * L + L + 4 * C + 4 * C


def news_kernel_flops(L, K, d, C):
    """Contraction FLOPs of the news-path scoring kernel per impression (unpadded): mui = A·E[his]
    and X = A·proj[his] (2·2KLd), M = Cand·muiᵀ and Lg = Cand·Xᵀ (2·2CdK)."""
    return 4 * K * L * d + 4 * C * d * K


def news_precompute_flops(n_news, d, Dc, K):
    """tanh(E·W1ᵀ)·Qᵀ and E·W2ᵀ over the table (model.py:171-174, :212)."""
    return n_news * (2 * d * Dc + 2 * Dc * K + 2 * d * d)


# ---------------------------------------------------------------------------------------------
# timing protocol: W untimed steps, barrier + sync, K timed steps, barrier + sync, max over ranks
# ---------------------------------------------------------------------------------------------
def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def timed_steps(step, steps, warmup, world, dev):
    """Runs step(i, timed) W times untimed then K times timed; returns max-over-ranks seconds."""
    for i in range(warmup):
        step(i, False)
    _sync(dev)
    if world > 1:
        dist.barrier()
    _sync(dev)
    t0 = time.perf_counter()
    for i in range(steps):
        step(i, True)
    _sync(dev)
    if world > 1:
        dist.barrier()
    _sync(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if dev.type == "cuda" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


class EventTimer:
    """HIP events recorded on the stream the kernels run on (torch's current stream, where every
    miner_amd op enqueues): per-step segment times in ms."""

    def __init__(self, dev, n_seg):
        self.stream = torch.cuda.current_stream(dev)
        self.n = n_seg
        self.ev = []

    def step(self):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(self.n + 1)]
        self.ev.append(e)
        return e

    def mean_ms(self, seg):
        return sum(e[seg].elapsed_time(e[seg + 1]) for e in self.ev) / max(len(self.ev), 1)


def host_info():
    """Threads used by the CPU baseline, the host's CPUs and the CPU model (lscpu)."""
    model = None
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                model = line.split(":", 1)[1].strip()
                break
    except (OSError, subprocess.SubprocessError):
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = None
    return {"threads_used": torch.get_num_threads(), "host_cpus": os.cpu_count(), "affinity_cpus": aff,
            "quota_cpus": cgroup_cpu_quota(), "cpu_model": model}


def cgroup_cpu_quota():
    """CPUs the container may actually use: the cgroup CPU quota (v2 cpu.max "quota period", v1
    cfs_quota_us / cfs_period_us), rounded up; None when unlimited or unreadable. The affinity mask
    can list every CPU of the machine while the quota allows a few of them."""
    import math
    for qf, pf in (("/sys/fs/cgroup/cpu.max", None),
                   ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "/sys/fs/cgroup/cpu/cpu.cfs_period_us"),
                   ("/sys/fs/cgroup/cpu,cpuacct/cpu.cfs_quota_us", "/sys/fs/cgroup/cpu,cpuacct/cpu.cfs_period_us")):
        try:
            with open(qf) as f:
                parts = f.read().split()
            if pf is None:
                quota, period = parts[0], parts[1]
            else:
                quota = parts[0]
                with open(pf) as f:
                    period = f.read().split()[0]
            if quota in ("max", "-1") or int(quota) <= 0:
                return None
            return max(1, math.ceil(int(quota) / int(period)))
        except (OSError, ValueError, IndexError):
            continue
    return None


# ---------------------------------------------------------------------------------------------
# CPU baselines (the oracle = the reference's torch CPU path restated; oracle/ is the checker)
# ---------------------------------------------------------------------------------------------
def _batched_oracle_rate(imp, W1, Q, W2, seconds, bs=64):
    """pairs/s of the oracle's batched torch CPU path (bs impressions per call) over ~seconds."""
    from oracle import miner_oracle as orc
    n = imp.history.shape[0]
    orc.score_torch(imp.history[:bs], imp.his_mask[:bs], imp.candidates[:bs], W1, Q, W2)  # warmup
    pairs, t0, i = 0, time.perf_counter(), 0
    while True:
        lo = (i * bs) % n
        orc.score_torch(imp.history[lo:lo + bs], imp.his_mask[lo:lo + bs], imp.candidates[lo:lo + bs], W1, Q, W2)
        pairs += bs * C
        i += 1
        el = time.perf_counter() - t0
        if el > seconds and i >= 2:
            return pairs / el, pairs, el


def cpu_baseline(seconds: float = 15.0, d: int = D):
    """Oracle (torch fp32 CPU restatement of model.py:159-216,127) on host cores, config-3 shape, at
    the pool's per-GPU CPU share (torch's default here, OMP_NUM_THREADS = 16 on the GPU box) and, when
    it differs, at the CPUs the container may use: the cgroup CPU quota capped by the affinity mask
    (SURVEY §8(d) asks for torch.set_num_threads(os.cpu_count()); os.cpu_count() and the affinity
    list the whole machine — 256 there — and running that many threads on a quota of a few CPUs
    measured oversubscription, not the CPU: VERDICT r4 item 8). ``value`` / ``cores`` are the faster
    leg; both legs are on the line."""
    from miner_amd import synthetic
    from oracle import miner_oracle as orc
    hi = host_info()
    imp = synthetic.impressions(36, 0, 512, L=L, d=d, C=C, device="cpu")
    W1, Q, W2 = synthetic.init_weights(36, d, DC, K)
    share = torch.get_num_threads()
    aff = hi["affinity_cpus"] or hi["host_cpus"] or share
    usable = min(aff, hi["quota_cpus"]) if hi["quota_cpus"] else aff
    legs = {}
    with torch.no_grad():
        for n_thr in dict.fromkeys([share, usable]):       # one leg when both counts agree
            torch.set_num_threads(n_thr)
            rate, pairs, el = _batched_oracle_rate(imp, W1, Q, W2, seconds / 2 if n_thr != share else seconds)
            legs[n_thr] = {"value": round(rate, 1), "threads": n_thr, "seconds": round(el, 1),
                           "impressions": pairs // C}
        torch.set_num_threads(share)
        # reference-faithful layout: one candidate per sample, eval_batch_size 32 (pool share threads)
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
    best = max(legs.values(), key=lambda x: x["value"])
    return {"value": best["value"], "unit": "pairs/s", "cores": best["threads"], "kind": "port",
            "cores_note": f"torch threads of the faster leg; legs: the pool's per-GPU CPU share ({share} threads, "
                          f"OMP_NUM_THREADS on the GPU box) and the {usable} CPUs the container may use (cgroup "
                          f"quota {hi['quota_cpus']} capped by the {aff}-CPU affinity; one leg when equal). "
                          "host_cpus / affinity_cpus list the whole machine",
            "legs": list(legs.values()),
            "sample": f"{best['impressions']} impressions x {C} candidates (L={L},K={K},d={d},Dc={DC}), fp32, "
                      f"batched 64 impressions/call, {best['seconds']}s",
            "host_cpus": hi["host_cpus"], "affinity_cpus": hi["affinity_cpus"], "quota_cpus": hi["quota_cpus"],
            "cpu_model": hi["cpu_model"],
            "per_candidate_value": round(per_cand, 1),
            "per_candidate_sample": f"{n_imp} impressions, one candidate per sample, batch 32 "
                                    f"(reader.py:376-379 layout), {share} threads, {el2:.1f}s"}


def metric_step_cpu_baseline(n_imp: int = 2000):
    """The reference's metric step (evaluation.py:36-84: sklearn per impression + np.argsort per
    impression, restated in oracle/metrics_oracle.py) on the host, seconds per impression."""
    import numpy as np
    from oracle import metrics_oracle as mo
    rng = np.random.default_rng(0)
    targets, probs = [], []
    for _ in range(n_imp):
        y = (rng.random(C) < 0.2).astype(np.int64)
        y[0], y[1] = 1, 0
        targets.append(list(y))
        probs.append(list(rng.random(C)))
    t0 = time.perf_counter()
    mo.compute_scores(targets, probs, ["auc", "group_auc", "mrr", "ndcg@5", "ndcg@10", "hit@5", "hit@10"])
    el = time.perf_counter() - t0
    return {"ms_per_impression": round(el / n_imp * 1e3, 4), "sample": f"{n_imp} impressions x {C} candidates, "
            "7 metrics (auc, group_auc, mrr, ndcg@5/10, hit@5/10), one thread"}


# ---------------------------------------------------------------------------------------------
# config 3 headline: the news-id path
# ---------------------------------------------------------------------------------------------
N_NEWS = 104_000     # MIND-large-shaped news table (~104k news x 768)
NEWS_B = 3_000_000   # impressions per GPU per step: the whole MIND-large-shaped eval set (config 3)
C2_B, C2_D, C2_NEWS = 50_000, 256, 65_238   # config 2 (MIND-small shape: ~65k news)


def news_batch(seed, B, n_news, dev, chunk=1 << 20, full=False):
    """Impressions as news ids (the reference's eval input, reader.py:351-379): history length
    ~ U{0..L}, left-padded with the pad news (row 0, reader.py:101-110, :369); candidates uniform.
    ``full``: every history holds L clicks (no padding: the most rows gathered per impression)."""
    g = torch.Generator(device=dev).manual_seed(seed)
    hid = torch.empty((B, L), dtype=torch.int32, device=dev)
    mask = torch.empty((B, L), dtype=torch.bool, device=dev)
    cid = torch.empty((B, C), dtype=torch.int32, device=dev)
    pos = torch.arange(L, device=dev)
    for s in range(0, B, chunk):
        e = min(s + chunk, B)
        lens = torch.full((e - s,), L, device=dev) if full else torch.randint(0, L + 1, (e - s,), generator=g, device=dev)
        m = pos[None, :] >= (L - lens)[:, None]
        h = torch.randint(1, n_news, (e - s, L), generator=g, device=dev, dtype=torch.int32)
        hid[s:e] = torch.where(m, h, torch.zeros_like(h))
        mask[s:e] = m
        cid[s:e] = torch.randint(1, n_news, (e - s, C), generator=g, device=dev, dtype=torch.int32)
    return hid, mask, cid


PMC_STATUS = {}      # counter file -> "used" or why it was rejected (goes on the bench line)


def load_pmc(path, workload, B, family):
    """The PMC counter file of a kernel (tools/pmc_traffic.py) if it measured THIS workload, batch and
    kernel source: the file's source_sha16 must equal the sha of the kernel family's current sources
    (tools/srcsha.py) and its matched kernel symbols must be that family's; otherwise None (the line
    then reports traffic / busy as null) and the reason goes to the line's pmc_status."""
    from tools.srcsha import KERNEL_SOURCES, source_sha16
    key = os.path.relpath(path, ROOT)
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError) as e:
        PMC_STATUS[key] = f"unreadable: {type(e).__name__}"
        return None
    want = source_sha16(KERNEL_SOURCES[family])
    sym = {"news_x2": "news_score_x2", "news": "news_score", "miner_score": "miner_fused", "fastformer": "ff_fused",
           "corpus": "rk_fused"}[family]
    if t.get("workload") != workload or t.get("batch") != B:
        PMC_STATUS[key] = f"rejected: measured {t.get('workload')} x {t.get('batch')}, not {workload} x {B}"
    elif t.get("source_sha16") != want:
        PMC_STATUS[key] = f"rejected: source sha {t.get('source_sha16')} != current {want} (re-profile the kernel)"
    elif not t.get("kernel_symbols") or not all(sym in k for k in t["kernel_symbols"]):
        PMC_STATUS[key] = f"rejected: matched kernel symbols {t.get('kernel_symbols')} are not {sym}"
    else:
        PMC_STATUS[key] = "used"
        return t
    return None


def measure_news(table, W1, Q, W2, pool, steps, warmup, world, dev, x2=None):
    """One dtype of the news path: per step precompute + score over pool[i % len(pool)]. fp32 tables:
    ``x2`` True = the fp16-pair kernel (news_score_x2, default), False = the fp32-MFMA kernel.
    Returns (elapsed s, precompute ms, scoring ms, {pool index: scores of its last step}, NewsTable)."""
    from miner_amd import news, ops
    pw = ops.pack_weights(W1, Q, W2, dtype=table.dtype)      # once per model, outside the timed region
    nt = news.precompute(table, pw, x2=x2)
    tm = EventTimer(dev, 2)
    out = {}

    def step(i, timed):
        nonlocal nt
        hid, mask, cid = pool[i % len(pool)]
        e = tm.step() if timed else None
        if e:
            e[0].record(tm.stream)
        nt = news.precompute(table, pw, out=nt, x2=x2)
        if e:
            e[1].record(tm.stream)
        out[i % len(pool)] = news.score(nt, hid, mask, cid, validate=False, x2=x2)
        if e:
            e[2].record(tm.stream)

    elapsed = timed_steps(step, steps, warmup, world, dev)
    return elapsed, tm.mean_ms(0), tm.mean_ms(1), out, nt


NEWS_MODES = {   # mode -> (fp16/bf16/fp32 MFMA products per fp32-equivalent product, dense peak TFLOP/s)
    "x2": (3, PEAK_BF16_TFLOPS),        # fp32 operands as fp16 pairs: lo·hi + hi·lo + hi·hi on the fp16 MFMA
    "mfma32": (1, PEAK_F32_TFLOPS),     # exact fp32 fma chains on the fp32 MFMA
    "bf16": (1, PEAK_BF16_TFLOPS),      # bf16 operands on the bf16 MFMA
}


def roofline_news(B, kern_ms, elem, d=D, pmc=None, kernel="", mode="bf16"):
    """Roofline of one news-path scoring launch. Two ceilings: HBM (SURVEY §8(d) bytes at 8 TB/s)
    and MFMA (the kernel's contraction FLOPs x the MFMA products each costs, at the dtype's dense
    peak); ``bound`` is the lower of the two (the longer ceiling time) and ``frac`` is against it,
    the other fraction beside it."""
    by = bytes_per_impression(L, d, C, elem) * B
    fl = news_kernel_flops(L, K, d, C) * B
    cost, peak_tf = NEWS_MODES[mode]
    t = kern_ms / 1e3
    gbs = by / t / 1e9
    tf = fl * cost / t / 1e12
    hbm_ms = by / (PEAK_HBM_GBS * 1e9) * 1e3
    mfma_ms = fl * cost / (peak_tf * 1e12) * 1e3
    gathered = news_gathered_bytes(L, d, C, K, elem)
    hbm = {"achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(gbs / PEAK_HBM_GBS, 4)}
    mfma = {"flops_per_impression": news_kernel_flops(L, K, d, C), "mfma_products_per_flop": cost,
            "achieved_tflops": round(tf, 2), "peak_tflops": peak_tf, "frac": round(tf / peak_tf, 4),
            "busy_frac_pmc": pmc.get("mfma_busy_frac") if pmc else None}
    if hbm_ms >= mfma_ms:
        head = {"bound": "hbm", **hbm}
    else:
        head = {"bound": "mfma", "achieved": round(tf, 2), "peak": peak_tf, "unit": "TFLOP/s",
                "frac": round(tf / peak_tf, 4)}
    head.update({
        "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None,
        "kernel": kernel, "kernel_ms": round(kern_ms, 4), "impressions_per_launch": B,
        "ceiling_ms": {"hbm": round(hbm_ms, 3), "mfma": round(mfma_ms, 3)},
        "algorithmic_bytes_per_impression": bytes_per_impression(L, d, C, elem),
        "algorithmic_bytes_per_launch": by, "hbm": hbm, "mfma": mfma,
        "gathered_bytes": {"per_impression": gathered, "per_launch": gathered * B,
                           "achieved_gbs": round(gathered * B / t / 1e9, 1)},
        "note": "bound = the lower of the two ceilings (HBM: SURVEY §8(d) bytes (L+C)·d·s + L + 4C per impression "
                "at 8 TB/s, weights and the per-news precompute excluded; MFMA: contraction FLOPs 2·2KLd + 2·2CdK "
                "(unpadded) x MFMA products per FLOP at the dense peak of the MFMA dtype); achieved over the "
                "HIP-event launch time; gathered_bytes: what the kernel moves (history rows of the table and of "
                "its projection, candidates, logit rows, ids, scores; re-reads served by L2 / the Infinity Cache); "
                "traffic: PMC HBM bytes per launch (2·FETCH_SIZE + WRITE_SIZE, gfx950 correction)"})
    return head


def device_metrics(scores, dev):
    """The reference's metric step (evaluation.py:36-84) over every impression of the batch, on the
    device (per-impression kernel + exact global AUC); labels Bernoulli(sigmoid(2 z(scores))) with
    >= 1 click and >= 1 non-click per impression (reader.py:374). Returns (labels, offsets, metrics,
    (steady-state ms, first-call ms))."""
    from miner_amd import metrics
    s = scores.float()
    g = torch.Generator(device=dev).manual_seed(7)
    z = (s - s.mean()) / s.std()
    lab = (torch.rand(s.shape, generator=g, device=dev) < torch.sigmoid(2.0 * z)).to(torch.uint8)
    rows = torch.arange(s.shape[0], device=dev)
    lab[rows, s.argmax(1)] = 1
    lab[rows, s.argmin(1)] = 0
    offs = torch.arange(0, (s.shape[0] + 1) * C, C, dtype=torch.int32, device=dev)
    names = ["auc", "group_auc", "mrr", "ndcg@5", "ndcg@10", "hit@5", "hit@10"]
    n_w = min(1000, s.shape[0])         # warm call (library init, first launches) on a slice
    metrics.compute_metrics(torch.sigmoid(s[:n_w]).reshape(-1), lab[:n_w].reshape(-1), offs[:n_w + 1], names)
    # the first full-size call also grows the caching allocator (sort buffers over every pair);
    # reported apart from the steady-state step (median of the next 3 calls, identical results)
    times = []
    for _ in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m = metrics.compute_metrics(torch.sigmoid(s).reshape(-1), lab.reshape(-1), offs, names)
        torch.cuda.synchronize()
        times.append((time.perf_counter() - t0) * 1e3)
    return lab, offs, m, (sorted(times[1:])[1], times[0])


def host_tolist_line(scores, ms_per_step, n_sample=100_000):
    """SURVEY §8(d) "with and without host .tolist()": the reference's eval hands every batch's
    sigmoid(logits) to Python as a list (evaluation.py:165 SlowEvaluator.eval_batch). Timed here:
    sigmoid on the device + the copy of the whole step's scores into pinned host memory (HIP events
    around both), and list conversion on a bounded sample of them (scaled to the step; it is
    per-element host work). The build's own evaluator keeps the scores on the device instead."""
    B, Cc = scores.shape
    host = torch.empty((B, Cc), dtype=torch.float32, pin_memory=True)
    st = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for rep in range(2):                                  # first pass warms the copy path
        a.record(st)
        host.copy_(torch.sigmoid(scores), non_blocking=True)
        b.record(st)
        torch.cuda.synchronize()
    d2h_ms = a.elapsed_time(b)
    n = min(n_sample, B)
    t0 = time.perf_counter()
    lst = host[:n].reshape(-1).tolist()
    tolist_ms = (time.perf_counter() - t0) * 1e3 * (B / n)
    assert len(lst) == n * Cc
    per_step = ms_per_step + d2h_ms + tolist_ms
    return {"value": round(B * Cc / (per_step / 1e3), 1), "unit": "pairs/s",
            "ms_per_step": round(per_step, 2), "d2h_sigmoid_ms": round(d2h_ms, 2),
            "tolist_ms": round(tolist_ms, 1),
            "sample": f"sigmoid + pinned D2H copy of the whole step ({B} x {Cc}); .tolist() timed on "
                      f"{n} impressions and scaled to {B}"}


def auc_parity(s32_full, s16_full, batch, table32, W1, Q, W2, dev, n_imp=2048):
    """The metric's "AUC parity vs ref", on a bounded sample of the timed batch (part of the CPU
    baseline leg): scores of the reference CPU path (the oracle: model.py:113-216 as the same torch
    fp32 ops on the host) vs the GPU news path in fp32 (the headline mode) and in bf16, then the
    reference's metrics (evaluation.py:36-84, via the GPU metrics kernels) over one set of labels:
    Bernoulli(sigmoid(2·z)) of the reference's z-scored scores, with >= 1 click and >= 1 non-click per
    impression (reader.py:374). The GPU scores are the first n_imp rows of the timed steps' own output
    for this batch (impressions are independent), so this leg launches no scoring kernel and the
    rocprof average of the headline kernel is over the timed launches only."""
    try:
        from miner_amd import metrics
        from oracle import miner_oracle as orc
        hid, mask, cid = [x[:n_imp] for x in batch]
        s32, s16 = s32_full[:n_imp], s16_full[:n_imp]
        T = table32.cpu()
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


def config2_line(args, rank, world, dev):
    """BASELINE config 2 (MIND-small shape: 50k impressions, L=50, K=32, d=256, bf16) on the news
    path, plus its fp32 form; rooflines with both ceilings, PMC traffic when profiled."""
    from miner_amd import synthetic
    out = {"workload": "config 2 MIND-small shape, news-id input", "impressions_per_gpu_per_step": C2_B,
           "d": C2_D, "news_table": C2_NEWS}
    g = torch.Generator(device=dev).manual_seed(2)
    t32 = torch.randn((C2_NEWS, C2_D), generator=g, device=dev) / C2_D ** 0.5
    W1, Q, W2 = synthetic.init_weights(2, C2_D, DC, K, device=dev)
    pool = [news_batch(1000 + rank, C2_B, C2_NEWS, dev)]
    for name, tab in (("bf16", t32.to(torch.bfloat16)), ("fp32", t32)):
        el, pre_ms, kern_ms, _, _ = measure_news(tab, W1, Q, W2, pool, args.steps, args.warmup, world, dev)
        elem = 2 if name == "bf16" else 4
        pmc = load_pmc(args.news_traffic_c2 if name == "bf16" else args.news_traffic_c2_32,
                       f"news_L{L}_K{K}_d{C2_D}_C{C}_N{C2_NEWS}_{name}", C2_B, "news" if name == "bf16" else "news_x2")
        kern = "news_score<bf16,weighted,4 chunks>" if name == "bf16" else "news_score_x2<weighted,dense,4 chunks>"
        out[name] = {"value": round(C2_B * C * args.steps * world / el, 1), "unit": "pairs/s",
                     "ms_per_step": round(el / args.steps * 1e3, 4), "precompute_ms": round(pre_ms, 4),
                     "roofline": roofline_news(C2_B, kern_ms, elem, d=C2_D, pmc=pmc, kernel=kern,
                                               mode="bf16" if name == "bf16" else "x2")}
    out["value"] = out["bf16"]["value"]
    out["dtype"] = "bf16 (config 2's dtype); fp32 beside it"
    return out


def run_news(args, rank, world, dev):
    """BASELINE config 3 on the news-id input, fp32 headline: every step recomputes
    the per-news precompute over the whole table (news_pre + the fp16-pair split) and scores this
    rank's shard of the 3,000,000-impression eval set (news_score_x2). At N > 1 the one set is
    sharded (BASELINE config 3: "3M impressions ... sharded across 8xMI355X"; no data-path
    collective); the per-GPU 3M weak-scaling figure rides beside it."""
    from miner_amd import distributed, synthetic
    total = args.batch or NEWS_B
    _, B = distributed.shard_range(total, rank, world)
    g = torch.Generator(device=dev).manual_seed(36)
    table32 = torch.randn((N_NEWS, D), generator=g, device=dev) / D ** 0.5
    W1, Q, W2 = synthetic.init_weights(36, D, DC, K, device=dev)
    pool = [news_batch(36 + (rank * args.pool + p), B, N_NEWS, dev) for p in range(args.pool)]
    torch.cuda.synchronize()
    # the dense-row comparison line first: measured after the minute of fp32 / bf16 news launches
    # below it read 3.53-3.59 ms, in isolation every version of the kernel since round-1 v8 reads
    # 3.26-3.37 ms (tools/bisect_dense.py, profiles/r02_dense_bisect.txt)
    dense = dense_kernel_line(dev, pmc_paths={"bf16": args.traffic, "fp32": args.traffic_dense32}) \
        if (world == 1 and not args.no_dense) else None

    # headline: fp32 (the reference's precision) on the fp16 matrix cores (exact-sum fp16 pairs)
    el32, pre32, kern32, o32, nt32 = measure_news(table32, W1, Q, W2, pool, args.steps, args.warmup, world, dev,
                                                  x2=True)
    s32 = o32[0]
    assert torch.isfinite(s32).all()
    # the exact fp32-MFMA kernel (news_score32) on the same batch: the fp32-fma-chain reference form
    exact = None
    if world == 1 and not args.no_exact:
        n_ex = min(args.steps, 5)
        elx, prex, kernx, ox, _ = measure_news(table32, W1, Q, W2, pool, n_ex, 1, world, dev, x2=False)
        d_ex = (ox[0].double() - s32.double()).abs().max() / s32.double().pow(2).mean().sqrt()
        exact = {"kernel": "news_score32<weighted, dense, fp32 MFMA, 24 chunks>", "steps": n_ex,
                 "value": round(B * C * n_ex / elx, 1), "unit": "pairs/s", "ms_per_step": round(elx / n_ex * 1e3, 4),
                 "roofline": roofline_news(B, kernx, 4, pmc=load_pmc(args.news_traffic32x, f"news_L{L}_K{K}_d{D}_C{C}_"
                                                                                         f"N{N_NEWS}_fp32", B, "news"),
                                           kernel="news_score32<weighted, dense, fp32 MFMA, 24 chunks>", mode="mfma32"),
                 "max_abs_diff_vs_headline_x_rms": float(d_ex)}
        del ox
    # the reference's default eval (config/eval_miner.txt: --evaluation_info metrics loss): the same
    # kernel with the eval loss's disagreement formed in its epilogue (no mui written)
    loss_line = None
    if world == 1 and not args.no_exact:
        from miner_amd import news as _news
        hid0, mask0, cid0 = pool[0]
        res = [None]

        def loss_fn():
            res[0] = _news.score(nt32, hid0, mask0, cid0, validate=False, x2=True, disagreement=True)

        ms_l = _kernel_ms(loss_fn, 3, 1, dev)
        assert torch.isfinite(res[0][1]).all()
        pmcl = load_pmc(args.news_traffic32_loss, f"news_L{L}_K{K}_d{D}_C{C}_N{N_NEWS}_fp32_loss", B, "news_x2")
        loss_line = {"kernel": "news_score_x2<weighted, dense, 12 chunks, MIND shape, LOSS> (scores + per-impression "
                               "disagreement D, loss.py:81; the Gram spread over the four mui waves)",
                     "value": round(B * C / (ms_l / 1e3), 1),
                     "unit": "pairs/s", "ms_per_launch": round(ms_l, 4), "impressions": B,
                     "vs_plain_kernel": round(kern32 / ms_l, 4),
                     "traffic": pmcl.get("hbm_bytes_per_launch") if pmcl else None,
                     "mfma_busy_pmc": pmcl.get("mfma_busy_frac") if pmcl else None}
        del res
    # every history full (hist_len = L, no left padding): the masked-slot grouping saves nothing here
    full_hist = None
    if world == 1 and not args.no_exact:
        pool_f = [news_batch(4000, B, N_NEWS, dev, full=True)]
        n_f = min(args.steps, 5)
        elf, _, kernf, _, _ = measure_news(table32, W1, Q, W2, pool_f, n_f, 1, world, dev, x2=True)
        rf = roofline_news(B, kernf, 4, mode="x2",
                           pmc=load_pmc(args.news_traffic32_full, f"news_L{L}_K{K}_d{D}_C{C}_N{N_NEWS}_fp32_full", B,
                                        "news_x2"),
                           kernel="news_score_x2<weighted, dense, 12 chunks, MIND shape>, full histories")
        gathered = news_gathered_bytes(L, D, C, K, 4)
        full_hist = {"histories": f"all {L} slots clicked (no padding)", "steps": n_f,
                     "value": round(B * C * n_f / elf, 1), "unit": "pairs/s", "ms_per_step": round(elf / n_f * 1e3, 4),
                     "kernel_ms": round(kernf, 4), "roofline": rf,
                     "gathered_over_algorithmic_bytes": round(gathered / bytes_per_impression(L, D, C, 4), 4),
                     "vs_headline_kernel_ms": round(kernf / kern32, 4)}
        del pool_f
    # bf16 throughput mode, same batch and protocol
    table16 = table32.to(torch.bfloat16)
    el16, pre16, kern16, o16, nt16 = measure_news(table16, W1, Q, W2, pool, args.steps, args.warmup, world, dev)
    s16 = o16[0]
    assert torch.isfinite(s16).all()
    # N > 1: the per-GPU weak-scaling figure (NEWS_B impressions on every rank)
    weak = None
    if world > 1 and not args.no_weak:
        del o16
        pw_ = [news_batch(5000 + rank, NEWS_B, N_NEWS, dev)]
        n_w = min(args.steps, 5)
        elw, _, kernw, _, _ = measure_news(table32, W1, Q, W2, pw_, n_w, 1, world, dev, x2=True)
        weak = {"scaling": "weak", "impressions_per_gpu_per_step": NEWS_B, "global_batch": NEWS_B * world,
                "steps": n_w, "value": round(NEWS_B * C * n_w * world / elw, 1), "unit": "pairs/s",
                "ms_per_step": round(elw / n_w * 1e3, 4), "kernel_ms_rank0": round(kernw, 4)}
        del pw_
    c2 = config2_line(args, rank, world, dev) if not args.no_config2 else None
    c4 = config4_subline(dev, pmc_path=args.traffic_ff) if (world == 1 and not args.no_config2) else None
    c5 = config5_subline(dev, pmc_path=args.traffic_rk) if (world == 1 and not args.no_config2) else None
    wide = wide_news_subline(dev) if (world == 1 and not args.no_config2) else None

    if rank != 0:
        return
    value = total * C * args.steps / el32
    pmc32 = load_pmc(args.news_traffic32, f"news_L{L}_K{K}_d{D}_C{C}_N{N_NEWS}_fp32", B, "news_x2")
    pmc16 = load_pmc(args.news_traffic, f"news_L{L}_K{K}_d{D}_C{C}_N{N_NEWS}_bf16", B, "news")
    roof = roofline_news(B, kern32, 4, pmc=pmc32, mode="x2",
                         kernel="news_score_x2<weighted, dense, fp16-pair operands, 12 chunks, MIND shape>")
    pre_fl = news_precompute_flops(N_NEWS, D, DC, K)
    # metric step on the device over the whole fp32 batch, and the bf16 AUC delta at full size
    metric_step = None
    if not args.no_metrics:
        lab, offs, m32, (ms, ms_first) = device_metrics(s32, dev)
        from miner_amd import metrics
        m16 = metrics.compute_metrics(torch.sigmoid(s16.float()).reshape(-1), lab.reshape(-1), offs, list(m32))
        metric_step = {"ms": round(ms, 2), "ms_first_call": round(ms_first, 2), "pairs": B * C, "impressions": B,
                       "what": "per-impression group_auc/mrr/ndcg@5,10/hit@5,10 kernel + exact global AUC "
                               "(device radix sort + rank sum) over rank 0's fp32 batch",
                       "fp32": {k: round(float(v), 6) for k, v in m32.items()},
                       "bf16_delta": {k: float(m16[k] - m32[k]) for k in m32},
                       "cpu_reference": metric_step_cpu_baseline() if (world == 1 and not args.no_cpu) else None}
    bf16_mode = {"value": round(total * C * args.steps / el16, 1), "unit": "pairs/s",
                 "ms_per_step": round(el16 / args.steps * 1e3, 4), "precompute_ms": round(pre16, 4),
                 "roofline": roofline_news(B, kern16, 2, pmc=pmc16, kernel="news_score<bf16,weighted,6 chunks>",
                                           mode="bf16"),
                 "auc_delta_vs_fp32": metric_step["bf16_delta"]["auc"] if metric_step else None,
                 "note": "bf16 operands, fp32 accumulation: no reference counterpart (the reference evaluates "
                         "in fp32); its metric deltas vs the fp32 headline are in metric_step.bf16_delta"}
    with_host = host_tolist_line(s32, el32 / args.steps * 1e3) if world == 1 else None
    cpu = cpu_baseline(args.cpu_seconds) if (world == 1 and not args.no_cpu) else None
    auc = auc_parity(s32, s16, pool[0], table32, W1, Q, W2, dev) if (world == 1 and not args.no_cpu) else None
    line = {
        "metric": METRIC,
        "value": round(value, 1), "unit": "pairs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(el32 / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "strong" if world > 1 else "weak", "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (seeded MIND-large-shaped impressions as news ids over a random news table; "
                "random-init weights)",
        "config": {"workload": "config 3 MIND-large shape, news-id input, fp32 (per step: per-news precompute "
                               "over the whole table + scoring this rank's shard of the 3M-impression set)",
                   "history": L, "K": K, "d": D, "Dc": DC, "candidates": C, "news_table": N_NEWS,
                   "impressions_per_gpu_per_step": B, "global_batch": total,
                   "timed_seconds": round(el32, 3),
                   "parallelism": f"dp{world} (contiguous impression shards of one set, no data-path collective)"},
        "fp32_arithmetic": "fp32 operands carried as exact-sum fp16 pairs in a power-of-two scale (hi + lo, "
                           "|x - hi - lo| <= 2^-22 |x|); each fp32 product is lo·hi + hi·lo + hi·hi on the fp16 "
                           "MFMA with fp32 accumulation; scores within 1e-5 of the reference CPU path "
                           "(auc_parity; tests/test_gpu_news.py: error vs float64 <= the fp32-MFMA kernel's)",
        "roofline": roof,
        "precompute": {"kernels": "news_pre<fp32, fp16 pairs> + x2_absmax/x2_split of the table and of proj",
                       "ms": round(pre32, 4), "flops": pre_fl, "tflops": round(pre_fl / (pre32 / 1e3) / 1e12, 2),
                       # the W1 / W2 products run as three fp16 MFMAs each (MINER_DTYPE_F32): priced on
                       # the fp16 dense peak at 3 products per algorithmic FLOP
                       "frac_fp16_peak_pairs": round(3 * pre_fl / (pre32 / 1e3) / 1e12 / PEAK_BF16_TFLOPS, 4)},
        "fp32_mfma_exact": exact, "eval_with_loss": loss_line, "full_histories": full_hist, "weak_scaling": weak,
        "bf16_mode": bf16_mode, "config2": c2, "config4": c4, "config5": c5, "wide_news": wide,
        "metric_step": metric_step,
        "dense_rows_kernel": dense, "with_host_tolist": with_host,
        "cpu_baseline": cpu, "auc_parity": auc, "pmc_status": PMC_STATUS,
    }
    print(json.dumps(line), flush=True)


def dense_kernel_line(dev, B=32768, steps=10, pmc_paths=None):
    """The fused dense-row kernel (the drop-in Miner.score module path, model.py:61-138: weights per
    impression, miner_score) on the config-3 shape, bf16 and fp32 (the reference's precision), each
    with its roofline (FLOPs 2LdDc + 2LDcK + 2KLd + 2Kd² + 4CdK + 2CK per impression: MFMA-bound)."""
    from miner_amd import ops, synthetic
    W1, Q, W2 = synthetic.init_weights(36, D, DC, K, device=dev)
    out = {}
    prev = os.environ.get("MINER_DENSE_FP32")
    for name, dt, peak, n in (("bf16", torch.bfloat16, PEAK_BF16_TFLOPS, B), ("fp32", torch.float32, PEAK_F32_TFLOPS,
                                                                               B // 4),
                              ("fp32_mfma_exact", torch.float32, PEAK_F32_TFLOPS, B // 4)):
        # fp32: S1 / S5 on fp16 pairs (the default); fp32_mfma_exact: every product on the fp32 MFMA
        if name == "fp32_mfma_exact":
            os.environ["MINER_DENSE_FP32"] = "mfma32"
        elif prev is None:
            os.environ.pop("MINER_DENSE_FP32", None)
        imp = synthetic.impressions(36, 0, n, L=L, d=D, C=C, device=dev, dtype=dt)
        pw = ops.pack_weights(W1, Q, W2, dtype=dt)
        for _ in range(3):
            ops.score(imp.history, imp.his_mask, imp.candidates, pw)
        torch.cuda.synchronize()
        st = torch.cuda.current_stream(dev)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(steps):
            ops.score(imp.history, imp.his_mask, imp.candidates, pw)
        b.record(st)
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / steps
        fl = flops_per_impression(L, K, D, DC, C) * n
        tf = fl / (ms / 1e3) / 1e12
        by = bytes_per_impression(L, D, C, 2 if name == "bf16" else 4) * n
        del imp
        kname = {"bf16": "miner_fused<bf16,full>", "fp32": "miner_fused<fp32,full,fp16-pair S1/S5>",
                 "fp32_mfma_exact": "miner_fused<fp32,full>"}[name]
        # the counter files of the two default forms (tools/r06_pmc.sh), bound to miner_score.hip's sha
        pmc = None
        if pmc_paths and name in pmc_paths:
            pmc = load_pmc(pmc_paths[name], f"L{L}_K{K}_d{D}_Dc{DC}_C{C}_{'bf16' if name == 'bf16' else 'fp32'}",
                           n, "miner_score")
        out[name] = {"kernel": kname, "value": round(n * C / (ms / 1e3), 1), "unit": "pairs/s",
                     "ms_per_launch": round(ms, 4), "impressions": n,
                     "roofline": {"bound": "mfma", "achieved": round(tf, 2), "peak": peak, "unit": "TFLOP/s",
                                  "frac": round(tf / peak, 4), "flops_per_launch": fl,
                                  "hbm_frac": round(by / (ms / 1e3) / 1e9 / PEAK_HBM_GBS, 4),
                                  "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None,
                                  "traffic_over_algorithmic": round(pmc["hbm_bytes_per_launch"] / by, 4) if pmc else None,
                                  "mfma_busy_pmc": pmc.get("mfma_busy_frac") if pmc else None}}
        if name == "fp32":
            # the same run seen on the matrix cores it uses: S1 / S5 (2·L·d·Dc + 2·K·d² per impression)
            # as three fp16 products each at the fp16 dense peak, S2 / S4 / S6 on the fp32 MFMA
            f_pair = (2 * L * D * DC + 2 * K * D * D) * n
            t_s = ms / 1e3
            out[name]["roofline"]["matrix_cores"] = {
                "fp16_pair_tflops": round(3 * f_pair / t_s / 1e12, 2), "fp16_peak": PEAK_BF16_TFLOPS,
                "fp16_frac": round(3 * f_pair / t_s / 1e12 / PEAK_BF16_TFLOPS, 4),
                "fp32_mfma_tflops": round((fl - f_pair) / t_s / 1e12, 2), "fp32_peak": peak,
                "note": "frac above = algorithmic fp32 FLOPs over the fp32 peak; the S1 / S5 share runs on the "
                        "fp16 matrix cores as fp16 pairs (3 products per FLOP), the S2 / S4 / S6 share on the fp32 MFMA"}
    if prev is None:
        os.environ.pop("MINER_DENSE_FP32", None)
    else:
        os.environ["MINER_DENSE_FP32"] = prev
    out["note"] = ("Miner.score / Miner.forward's drop-in module path on dense [B, L, d] / [B, C, d] rows: every "
                   "impression re-reads W1 and W2 (the news-id path precomputes them per news row instead). fp32: "
                   "S1 (W1·Eᵀ) and S5 (W2·muiᵀ) on fp16 pairs (each fp32 operand of a row with a power-of-two unit u "
                   "carried as hi = f16(x/u), lo = f16(x/u - hi), lo·hi + hi·lo + hi·hi on the fp16 MFMA, the units "
                   "applied exactly; W1 / W2 pair copies packed once; error vs float64 within 1.5x the fp32 MFMA's, "
                   "tests/test_gpu_parity.py::test_x6_error_vs_fp32_mfma, ::test_fp32_pairs_heavy_tailed), S2 / S4 / "
                   "S6 on the fp32 MFMA; its frac is algorithmic FLOPs over the fp32 peak; traffic counts the history "
                   "rows about twice per impression (S1's cut and S4's gathers: beyond what an XCD's L2 holds for "
                   "32 CUs). fp32_mfma_exact: every product on the fp32 MFMA (MINER_DENSE_FP32=mfma32)")
    return out


# ---------------------------------------------------------------------------------------------
# config 4: FastFormer user encoder
# ---------------------------------------------------------------------------------------------
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
    hi = host_info()
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
    return {"value": round(pairs / el, 1), "unit": "pairs/s", "cores": hi["threads_used"], "kind": "port",
            "host_cpus": hi["host_cpus"], "cpu_model": hi["cpu_model"],
            "sample": f"{pairs // FF_C} impressions x {FF_C} candidates (L={FF_L}, hidden {FF_H}), fp32, "
                      f"batched {bs} impressions/call, {el:.1f}s"}


def run_fastformer(args, rank, world, dev):
    """BASELINE config 4: the FastFormer kernel over FF_B resident impressions per GPU per step."""
    from miner_amd import fastformer as ff
    from miner_amd import synthetic
    B = args.batch or FF_B
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
    tm = EventTimer(dev, 1)
    out = [None]

    def step(i, timed):
        hist, mask, cand = pool[i % len(pool)]
        e = tm.step() if timed else None
        if e:
            e[0].record(tm.stream)
        out[0] = ff.score(hist, mask, cand, pk16)
        if e:
            e[1].record(tm.stream)

    elapsed = timed_steps(step, args.steps, args.warmup, world, dev)
    kern_ms = tm.mean_ms(0)
    assert torch.isfinite(out[0]).all()
    f32 = None
    if args.fp32_steps > 0:
        hist, mask, cand = pool[0]
        n32 = min(B, 5000)
        h32, c32, m32 = hist[:n32].float(), cand[:n32].float(), mask[:n32]
        ff.score(h32, m32, c32, pk32)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(tm.stream)
        for _ in range(args.fp32_steps):
            ff.score(h32, m32, c32, pk32)
        b.record(tm.stream)
        torch.cuda.synchronize()
        ms32 = a.elapsed_time(b) / args.fp32_steps
        f32 = {"value": round(n32 * FF_C / (ms32 / 1e3), 1), "unit": "pairs/s", "ms_per_step": round(ms32, 3),
               "impressions": n32,
               "tflops": round(ff_flops_per_impression() * n32 / (ms32 / 1e3) / 1e12, 2)}
    if rank != 0:
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


# ---------------------------------------------------------------------------------------------
# config 5: full-corpus ranking
# ---------------------------------------------------------------------------------------------
C5_L, C5_K, C5_N, C5_U, C5_TOPK = 200, 64, 200_000, 2048, 100
C5_SHARE_U = 1_000_000 // 8          # config 5's users per GPU on 8 GPUs


def corpus_cpu_baseline(seconds: float = 10.0):
    """Config-5 oracle (the reference's encoder + click score restated in torch fp32 on the CPU,
    oracle/corpus_oracle.py) on host cores: 8 users against news chunks of 4096 until `seconds`."""
    from miner_amd import synthetic
    from oracle import corpus_oracle as co
    hi = host_info()
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
    return {"value": round(pairs / el, 1), "unit": "(user,news) pairs/s", "cores": hi["threads_used"],
            "kind": "port", "host_cpus": hi["host_cpus"], "cpu_model": hi["cpu_model"],
            "sample": f"{U} users (history {C5_L}, K={C5_K}, d={D}) encoded and scored against {pairs // U} news "
                      f"rows in chunks of 4096, fp32, {el:.1f}s (top-k selection not included)"}


def _kernel_ms(fn, steps, warmup, dev):
    """Mean HIP-event time of ``fn()`` on the current stream after ``warmup`` untimed calls."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize(dev)
    st = torch.cuda.current_stream(dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(steps):
        fn()
    b.record(st)
    torch.cuda.synchronize(dev)
    return a.elapsed_time(b) / steps


def config4_subline(dev, steps=5, warmup=2, pmc_path=None):
    """BASELINE config 4 (FastFormer, 50k impressions, bf16) measured inside the default run, so the
    driver's bench carries it; the full line is ``--workload fastformer``."""
    from miner_amd import fastformer as ff
    from miner_amd import synthetic
    g = torch.Generator().manual_seed(1000)
    lens = torch.randint(0, FF_L + 1, (FF_B,), generator=g)
    mask = (torch.arange(FF_L)[None, :] >= (FF_L - lens)[:, None]).to(dev)
    hist = (torch.randn(FF_B, FF_L, FF_H, generator=g) * 0.0625).to(dev, torch.bfloat16)
    cand = (torch.randn(FF_B, FF_C, FF_H, generator=g) * 0.0625).to(dev, torch.bfloat16)
    pk = ff.pack(synthetic.fastformer_params(0).to(dev), torch.bfloat16)
    out = [None]

    def fn():
        out[0] = ff.score(hist, mask, cand, pk)

    ms = _kernel_ms(fn, steps, warmup, dev)
    assert torch.isfinite(out[0]).all()
    tflops = ff_flops_per_impression() * FF_B / (ms / 1e3) / 1e12
    pmc = load_pmc(pmc_path, f"ff_L{FF_L}_H{FF_H}_C{FF_C}_bf16_dense", FF_B, "fastformer") if pmc_path else None
    return {"workload": "config 4 FastFormer user encoder (L=50, hidden 256, 16 heads, 2 layers, C=40)",
            "value": round(FF_B * FF_C / (ms / 1e3), 1), "unit": "pairs/s", "dtype": "bf16",
            "impressions_per_step": FF_B, "ms_per_step": round(ms, 4), "steps": steps,
            "roofline": {"bound": "mfma", "achieved": round(tflops, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(tflops / PEAK_BF16_TFLOPS, 4), "kernel": "ff_fused<bf16>",
                         "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None,
                         "mfma_busy_pmc": pmc.get("mfma_busy_frac") if pmc else None,
                         "valu_insts_per_impression": round(pmc["SQ_INSTS_VALU"] / FF_B, 1)
                         if pmc and "SQ_INSTS_VALU" in pmc else None}}


WN_B, WN_L, WN_K = 100_000, 100, 64      # the wide news-id line: K = 64, L = 100


def wide_news_subline(dev, steps=5, warmup=2):
    """A reference-legal model past the news kernels' K <= 32 / L <= 64 (model.py:18-21, :159-185):
    K = 64 interests, history 100, d = 768, 40 candidates, 100k impressions as news ids over the
    104k-news table (left padding = the pad news, as news_batch). The news-id path (per-news
    precompute, logits in 32-interest slices + news_score_x2w, fp32 on the fp16 matrix cores)
    against the wide path it replaces (miner_encode_users + miner_score_wide, exact fp32, recomputing
    gelu(mui·W2ᵀ) per user), the latter on the first 20k impressions."""
    from miner_amd import news, ops, synthetic
    g = torch.Generator(device=dev).manual_seed(64)
    table = torch.randn((N_NEWS, D), generator=g, device=dev) / D ** 0.5
    W1, Q, W2 = synthetic.init_weights(64, D, DC, WN_K, device=dev)
    pos = torch.arange(WN_L, device=dev)
    lens = torch.randint(0, WN_L + 1, (WN_B,), generator=g, device=dev)
    mask = pos[None, :] >= (WN_L - lens)[:, None]
    hid = torch.where(mask, torch.randint(1, N_NEWS, (WN_B, WN_L), generator=g, device=dev, dtype=torch.int32),
                      torch.zeros((), dtype=torch.int32, device=dev))
    cid = torch.randint(1, N_NEWS, (WN_B, C), generator=g, device=dev, dtype=torch.int32)
    nt = [news.precompute(table, W1, Q, W2, x2=True)]
    out = [None]

    def pre():
        nt[0] = news.precompute(table, W1, Q, W2, out=nt[0], x2=True)

    def fn():
        out[0] = news.score(nt[0], hid, mask, cid, validate=False, x2=True)

    pre_ms = _kernel_ms(pre, 2, 1, dev)
    ms = _kernel_ms(fn, steps, warmup, dev)
    assert torch.isfinite(out[0]).all()
    Bo = 20_000
    pw = ops.pack_weights(W1, Q, W2)
    old = [None]

    def fn_old():
        old[0] = ops.score_gather(table, hid[:Bo], mask[:Bo], cid[:Bo], pw, validate=False)

    ms_old = _kernel_ms(fn_old, 2, 1, dev)
    d_old = float((old[0].double() - out[0][:Bo].double()).abs().max() / old[0].double().pow(2).mean().sqrt())
    byt = bytes_per_impression(WN_L, D, C, 4) * WN_B
    gbs = byt / (ms / 1e3) / 1e9
    return {"workload": f"K={WN_K}, history {WN_L}, d={D}, {C} candidates, {WN_B} impressions as news ids "
                        f"({N_NEWS}-news table), fp32",
            "value": round(WN_B * C / (ms / 1e3), 1), "unit": "pairs/s", "dtype": "fp32",
            "kernel": "news_score_x2w<weighted, dense> (fp16-pair operands)", "ms_per_launch": round(ms, 4),
            "steps": steps, "precompute_ms": round(pre_ms, 3),
            "value_with_precompute": round(WN_B * C / ((ms + pre_ms) / 1e3), 1),
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(gbs / PEAK_HBM_GBS, 4),
                         "algorithmic_bytes_per_impression": bytes_per_impression(WN_L, D, C, 4)},
            "replaced_wide_path": {"kernels": "ue_fused<fp32> + wide_score<fp32> (miner_encode_users + "
                                              "miner_score_wide)", "impressions": Bo,
                                   "value": round(Bo * C / (ms_old / 1e3), 1), "unit": "pairs/s",
                                   "ms_per_launch": round(ms_old, 3),
                                   "max_abs_diff_x_rms": d_old}}


def config5_subline(dev, steps=2, warmup=1, share_users=C5_SHARE_U, pmc_path=None):
    """BASELINE config 5 (full-corpus ranking: 2048 users x 200k news, L=200, K=64, fp16, top-100) measured
    inside the default run; the full line is ``--workload corpus``."""
    from miner_amd import corpus, synthetic
    dt = torch.float16
    g = torch.Generator(device=dev).manual_seed(5)
    table = (torch.randn((C5_N, D), generator=g, device=dev) / D ** 0.5).to(dt)
    W1, Q, W2 = synthetic.init_weights(5, D, DC, C5_K, device=dev)
    pk = corpus.pack_encoder(W1, Q, W2, dtype=dt)
    hid = torch.randint(0, C5_N, (C5_U, C5_L), generator=g, device=dev, dtype=torch.int32)
    lens = torch.randint(1, C5_L + 1, (C5_U,), generator=g, device=dev)
    mask = torch.arange(C5_L, device=dev)[None, :] >= (C5_L - lens)[:, None]
    out = [None]

    def fn():
        mui, proj = corpus.encode_users(table, mask, pk, his_ids=hid)
        out[0] = corpus.rank_topk(mui, proj, table, C5_TOPK)

    ms = _kernel_ms(fn, steps, warmup, dev)
    assert torch.isfinite(out[0][0]).all()
    rk_pmc = load_pmc(pmc_path, f"rk_U{C5_U}_N{C5_N}_L{C5_L}_K{C5_K}_d{D}_top{C5_TOPK}_fp16", C5_U, "corpus") \
        if pmc_path else None
    fl = C5_U * C5_N * 4 * C5_K * D
    tflops = fl / (ms / 1e3) / 1e12
    # one GPU's share of config 5's 1M users on 8 GPUs (125,000), ranked in one host loop
    # (corpus.rank_corpus: 16,384 users per encode + rank pair); users shard with no data-path
    # collective, so this is also the whole job's time at 8 GPUs
    share = None
    if share_users:
        gs = torch.Generator(device=dev).manual_seed(55)
        hs = torch.randint(0, C5_N, (share_users, C5_L), generator=gs, device=dev, dtype=torch.int32)
        ls = torch.randint(1, C5_L + 1, (share_users,), generator=gs, device=dev)
        ms_ = torch.arange(C5_L, device=dev)[None, :] >= (C5_L - ls)[:, None]
        res = [None]

        def share_fn():
            res[0] = corpus.rank_corpus(table, hs, ms_, pk, C5_TOPK)

        corpus.rank_corpus(table, hs[:4096], ms_[:4096], pk, C5_TOPK)      # warm-up
        sec = _kernel_ms(share_fn, 1, 0, dev) / 1e3
        assert torch.isfinite(res[0][0]).all()
        share = {"users": share_users, "news": C5_N, "seconds": round(sec, 3),
                 "value": round(share_users * C5_N / sec, 1), "unit": "(user,news) pairs/s",
                 "what": "one GPU's share of BASELINE config 5 (1M users / 8 GPUs), encode + rank top-100 "
                         "in batches of 16,384 users; users shard with no collective, so 8 GPUs take the "
                         "same seconds for all 1M users"}
        del hs, ms_, res
    return {"workload": "config 5 full-corpus ranking (2048 users x 200k news, L=200, K=64, top-100)",
            "value": round(C5_U * C5_N / (ms / 1e3), 1), "unit": "(user,news) pairs/s", "dtype": "fp16",
            "ms_per_step": round(ms, 3), "steps": steps,
            "roofline": {"bound": "mfma", "achieved": round(tflops, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(tflops / PEAK_BF16_TFLOPS, 4),
                         "kernel": "ue_fused<fp16> + rk_fused<fp16> (ranker FLOPs over the whole step)",
                         "ranker_traffic": rk_pmc.get("hbm_bytes_per_launch") if rk_pmc else None,
                         "ranker_mfma_busy_pmc": rk_pmc.get("mfma_busy_frac") if rk_pmc else None},
            "per_gpu_share": share}


def run_corpus(args, rank, world, dev):
    """BASELINE config 5: every user against the whole 200k-news table (fp16), history 200, K=64,
    fused click score + running top-k (never materialising the U x N scores). One step = encode
    ``--batch`` users (default 2048) per GPU and rank them against the table; users shard over
    ranks (weak scaling, no data-path collective)."""
    from miner_amd import corpus, synthetic
    U = args.batch or C5_U
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
    tm = EventTimer(dev, 2)
    out = {}

    def step(i, timed):
        hid, mask = pool[i % len(pool)]
        e = tm.step() if timed else None
        if e:
            e[0].record(tm.stream)
        mui, proj = corpus.encode_users(table, mask, pk, his_ids=hid)
        if e:
            e[1].record(tm.stream)
        out[0] = corpus.rank_topk(mui, proj, table, C5_TOPK)
        if e:
            e[2].record(tm.stream)

    steps = args.steps if args.steps_set else 5
    warm = args.warmup if args.warmup_set else 1
    elapsed = timed_steps(step, steps, warm, world, dev)
    enc_ms, rank_ms = tm.mean_ms(0), tm.mean_ms(1)
    assert torch.isfinite(out[0][0]).all()
    if rank != 0:
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


# ---------------------------------------------------------------------------------------------
# the fused dense-row kernel as the workload
# ---------------------------------------------------------------------------------------------
def run_dense(args, rank, world, dev):
    """config 3 with history / candidates given as [B, L, d] / [B, C, d] rows (miner_score: the
    fused kernel with the weights per impression), bf16."""
    from miner_amd import ops, synthetic
    B = args.batch or 32768
    bf = torch.bfloat16
    pool = [synthetic.impressions(36, (rank * args.pool + p) * B, B, L=L, d=D, C=C, device=dev, dtype=bf)
            for p in range(args.pool)]
    W1, Q, W2 = synthetic.init_weights(36, D, DC, K, device=dev)
    pw16 = ops.pack_weights(W1, Q, W2, dtype=bf)
    tm = EventTimer(dev, 1)
    out = [None]

    def step(i, timed):
        imp = pool[i % len(pool)]
        e = tm.step() if timed else None
        if e:
            e[0].record(tm.stream)
        out[0] = ops.score(imp.history, imp.his_mask, imp.candidates, pw16)
        if e:
            e[1].record(tm.stream)

    elapsed = timed_steps(step, args.steps, args.warmup, world, dev)
    kern_ms = tm.mean_ms(0)
    assert torch.isfinite(out[0]).all()
    if rank != 0:
        return
    fl = flops_per_impression(L, K, D, DC, C) * B
    by = bytes_per_impression(L, D, C, 2) * B
    tflops = fl / (kern_ms / 1e3) / 1e12
    gbs = by / (kern_ms / 1e3) / 1e9
    pmc = load_pmc(args.traffic, f"L{L}_K{K}_d{D}_Dc{DC}_C{C}_bf16", B, "miner_score")
    line = {
        "metric": METRIC, "value": round(B * C * args.steps * world / elapsed, 1), "unit": "pairs/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic (seeded MIND-large-shaped impressions, random-init weights)",
        "config": {"workload": "config 3 MIND-large shape, dense rows", "history": L, "K": K, "d": D, "Dc": DC,
                   "candidates": C, "impressions_per_gpu_per_step": B, "global_batch": B * world,
                   "parallelism": f"dp{world} (impression shards, no data-path collective)"},
        "roofline": {"bound": "mfma", "achieved": round(tflops, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(tflops / PEAK_BF16_TFLOPS, 4),
                     "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None,
                     "kernel": "miner_fused<bf16,full>", "flops_per_launch": fl, "kernel_ms": round(kern_ms, 4),
                     "mfma_busy_pmc": pmc.get("mfma_busy_frac") if pmc else None},
        "roofline_hbm": {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(gbs / PEAK_HBM_GBS, 4), "algorithmic_bytes_per_launch": by},
        "cpu_baseline": cpu_baseline(args.cpu_seconds) if (world == 1 and not args.no_cpu) else None,
    }
    print(json.dumps(line), flush=True)


# ---------------------------------------------------------------------------------------------
# launcher and dry run
# ---------------------------------------------------------------------------------------------
def run_dry(args, rank, world, dev):
    """The launcher, the config-3 shard plan and the timing protocol without a GPU (gloo): a step is a
    small CPU matmul; every rank reports its shard of the one 3M-impression set, gathered to rank 0."""
    from miner_amd import distributed
    total = args.batch or NEWS_B
    start, count = distributed.shard_range(total, rank, world)
    a = torch.randn(64, 64)

    def step(i, timed):
        torch.mm(a, a)

    elapsed = timed_steps(step, args.steps, args.warmup, world, dev)
    shards = [(start, count)]
    if world > 1:
        shards = [None] * world
        dist.all_gather_object(shards, (start, count))
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": round(64 * args.steps * world / elapsed, 1), "unit": "pairs/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
                          "scaling": "strong" if world > 1 else "weak", "vs_baseline": None, "dtype": "fp32",
                          "data": "dry run (no kernel)",
                          "config": {"workload": "dry run: launcher, shard plan and timing protocol only",
                                     "global_batch": sum(c for _, c in shards), "shards": shards}}), flush=True)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n):
    """--gpus N without a torch.distributed environment: start N ranks as CHILD processes (the
    torch.distributed.run launcher, one process per GPU) before anything touches the GPU, and exit
    with their status — never an exec from this process."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__),
           *sys.argv[1:]]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks (one per GPU); default WORLD_SIZE or 1")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="config3", choices=["config3", "config3-dense", "fastformer", "corpus"])
    ap.add_argument("--batch", type=int, default=None, help="impressions (users) per GPU per step")
    ap.add_argument("--pool", type=int, default=2, help="distinct resident batches per GPU")
    ap.add_argument("--fp32-steps", type=int, default=2, help="(fastformer) fp32 parity-mode launches")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-dense", action="store_true", help="skip the dense-row kernel comparison")
    ap.add_argument("--no-config2", action="store_true", help="skip the config-2 / -4 / -5 sub-lines")
    ap.add_argument("--no-metrics", action="store_true", help="skip the device metric step")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--traffic-dense32", default=os.path.join(ROOT, "profiles", "pmc_traffic_dense_fp32.json"))
    ap.add_argument("--traffic-ff", default=os.path.join(ROOT, "profiles", "pmc_traffic_ff_bf16.json"))
    ap.add_argument("--traffic-rk", default=os.path.join(ROOT, "profiles", "pmc_traffic_rk_fp16.json"))
    ap.add_argument("--news-traffic32-loss", default=os.path.join(ROOT, "profiles", "pmc_traffic_news_x2_loss.json"))
    ap.add_argument("--news-traffic", default=os.path.join(ROOT, "profiles", "pmc_traffic_news.json"))
    ap.add_argument("--news-traffic32", default=os.path.join(ROOT, "profiles", "pmc_traffic_news_x2.json"))
    ap.add_argument("--news-traffic32x", default=os.path.join(ROOT, "profiles", "pmc_traffic_news_fp32.json"))
    ap.add_argument("--news-traffic32-full", default=os.path.join(ROOT, "profiles", "pmc_traffic_news_x2_full.json"))
    ap.add_argument("--news-traffic-c2", default=os.path.join(ROOT, "profiles", "pmc_traffic_news_c2.json"))
    ap.add_argument("--news-traffic-c2-32", default=os.path.join(ROOT, "profiles", "pmc_traffic_news_c2_x2.json"))
    ap.add_argument("--no-exact", action="store_true", help="skip the fp32-MFMA (news_score32) sub-line")
    ap.add_argument("--no-weak", action="store_true", help="N>1: skip the per-GPU 3M weak-scaling sub-field")
    ap.add_argument("--dry-run", action="store_true", help="CPU/gloo: launcher and timing protocol only")
    args = ap.parse_args()
    args.steps_set = "--steps" in sys.argv
    args.warmup_set = "--warmup" in sys.argv

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus is not None and args.gpus > 1:
        return launch_ranks(args.gpus)
    world = int(env_world or "1")
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: one rank per GPU")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        dev = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo")
        run_dry(args, rank, world, dev)
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        if world > 1:
            dist.init_process_group("nccl", device_id=dev)
        {"config3": run_news, "config3-dense": run_dense, "fastformer": run_fastformer,
         "corpus": run_corpus}[args.workload](args, rank, world, dev)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
