"""Host wall per eval-loop chunk with the eval loss (news.score with mui + eval_loss_partials), with
a fresh mui buffer per chunk or one reused buffer: does allocating 3.2 GB per chunk cost time?

    python tools/loss_probe.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from miner_amd import evaluation, news, ops, synthetic  # noqa: E402

dev = "cuda:0"
B, L, C, d, n_news = 32768, 50, 40, 768, 104000
g = torch.Generator(device=dev).manual_seed(1)
table = torch.randn((n_news, d), generator=g, device=dev) / d ** 0.5
lens = torch.randint(0, L + 1, (B,), generator=g, device=dev)
mask = torch.arange(L, device=dev)[None, :] >= (L - lens)[:, None]
hid = torch.randint(1, n_news, (B, L), generator=g, device=dev, dtype=torch.int32)
cid = torch.randint(1, n_news, (B, C), generator=g, device=dev, dtype=torch.int32)
lab = (torch.rand((B, C), generator=g, device=dev) < 0.1).to(torch.uint8)
W1, Q, W2 = synthetic.init_weights(1, d, 200, 32, device=dev)
nt = news.precompute(table, ops.pack_weights(W1, Q, W2))


def chunk(buf=None):
    s, mui = news.score(nt, hid, mask, cid, validate=False, return_user=True, user_out=buf)
    return evaluation.eval_loss_partials(mui, s, lab, first_sample=0, total_samples=B * C)


for name, buf in (("fresh buffer", None), ("reused buffer", torch.empty((B, 32, d), device=dev))):
    chunk(buf)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    acc = torch.zeros(2, dtype=torch.float64, device=dev)
    for _ in range(10):
        acc += chunk(buf)
    float(acc[0])
    print(f"{name}: {(time.perf_counter() - t0) / 10 * 1e3:.2f} ms per 32k chunk (score + mui + loss partials)")
