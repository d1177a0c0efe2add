"""Where the device metric step's time goes (bench.py metric_step): the per-impression kernel, the
copies back to the host, the host reductions and the exact global AUC, timed separately on the
bench's 3M x 40 shape.

    python tools/metric_probe.py [B] [C]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from miner_amd import metrics  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 3_000_000
C = int(sys.argv[2]) if len(sys.argv) > 2 else 40
dev = "cuda:0"
g = torch.Generator(device=dev).manual_seed(7)
s = torch.randn((B, C), generator=g, device=dev) * 0.02
lab = (torch.rand((B, C), generator=g, device=dev) < torch.sigmoid(2 * s / 0.02)).to(torch.uint8)
rows = torch.arange(B, device=dev)
lab[rows, s.argmax(1)] = 1
lab[rows, s.argmin(1)] = 0
offs = torch.arange(0, (B + 1) * C, C, dtype=torch.int32, device=dev)
p = torch.sigmoid(s).reshape(-1)
y = lab.reshape(-1)
names = ["auc", "group_auc", "mrr", "ndcg@5", "ndcg@10", "hit@5", "hit@10"]


def t(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best * 1e3


print(f"B={B} C={C}")
print(f"compute_metrics (all 7)      {t(lambda: metrics.compute_metrics(p, y, offs, names)):8.1f} ms")
print(f"per_impression (6 metrics)   {t(lambda: metrics.per_impression(p, y, offs, names[1:])):8.1f} ms")
print(f"global_auc                   {t(lambda: metrics.global_auc(p, y)):8.1f} ms")
