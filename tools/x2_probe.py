"""Time the fp32 news kernels on tables of several sizes (is the kernel gather-bound?).

    python tools/x2_probe.py [B] [reps] [n_news ...]

Prints the median HIP-event ms per launch of news_score_x2 (and news_score32 with PROBE_MFMA32=1)
for each table size, same impressions (ids folded into the table).
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from miner_amd import news, ops, synthetic  # noqa: E402

dev = "cuda:0"
B = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
sizes = [int(x) for x in sys.argv[3:]] or [104000, 20000, 4000]
L, C, d, K, Dc = 50, 40, int(os.environ.get("PROBE_D", "768")), 32, 200
g = torch.Generator(device=dev).manual_seed(36)
lens = torch.randint(0, L + 1, (B,), generator=g, device=dev)
mask = torch.arange(L, device=dev)[None, :] >= (L - lens)[:, None]
hid0 = torch.randint(1, 1 << 30, (B, L), generator=g, device=dev, dtype=torch.int32)
cid0 = torch.randint(1, 1 << 30, (B, C), generator=g, device=dev, dtype=torch.int32)
W1, Q, W2 = synthetic.init_weights(36, d, Dc, K, device=dev)
pw = ops.pack_weights(W1, Q, W2, dtype=torch.float32)
st = torch.cuda.current_stream()
kerns = ["x2"] + (["mfma32"] if os.environ.get("PROBE_MFMA32") else []) + (["bf16"] if os.environ.get("PROBE_BF16") else [])
for n in sizes:
    table = torch.randn((n, d), generator=g, device=dev) / d ** 0.5
    hid = torch.where(mask, hid0 % (n - 1) + 1, torch.zeros_like(hid0))
    cid = cid0 % (n - 1) + 1
    for kern in kerns:
        x2 = kern == "x2"
        if kern == "bf16":
            nt = news.precompute(table.to(torch.bfloat16), ops.pack_weights(W1, Q, W2, dtype=torch.bfloat16))
        else:
            nt = news.precompute(table, pw, x2=x2)
        news.score(nt, hid, mask, cid, validate=False, x2=x2)
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            news.score(nt, hid, mask, cid, validate=False, x2=x2)
            b.record(st)
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        ms = statistics.median(ts)
        print(f"{kern} n_news={n} ({n * d * 8 / 2**20:.0f} MiB E+proj): {ms:.3f} ms / {B} imp "
              f"({B * C / ms / 1e3:.1f} M pairs/s)", flush=True)
