"""A/B of news-path kernel variants in one process (interleaved), outputs compared.

    python tools/news_ab.py [fp32|bf16] [B] [reps]

Variant A = the default build path, variant B = MINER_NEWS_F32V1=1 (the round-1 fp32 kernel) for
fp32, or MINER_NEWS_CW64=1 for bf16. Prints per-variant scoring ms (HIP events, median of reps)
and the max relative difference of the scores between the variants.
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from miner_amd import news, ops, synthetic  # noqa: E402

dev = "cuda:0"
dt = torch.float32 if (len(sys.argv) < 2 or sys.argv[1] == "fp32") else torch.bfloat16
B = int(sys.argv[2]) if len(sys.argv) > 2 else 131072
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
alt = os.environ.get("AB_ALT", "MINER_NEWS_F32V1" if dt == torch.float32 else "MINER_NEWS_CW64")
altv = os.environ.get("AB_ALT_VALUE", "1")
n_news, L, C, d, K, Dc = 104000, 50, 40, int(os.environ.get("AB_D", "768")), 32, 200
g = torch.Generator(device=dev).manual_seed(36)
table = (torch.randn((n_news, d), generator=g, device=dev) / d ** 0.5).to(dt)
lens = torch.randint(0, L + 1, (B,), generator=g, device=dev)
mask = torch.arange(L, device=dev)[None, :] >= (L - lens)[:, None]
hid = torch.randint(1, n_news, (B, L), generator=g, device=dev, dtype=torch.int32)
hid[~mask] = 0
cid = torch.randint(1, n_news, (B, C), generator=g, device=dev, dtype=torch.int32)
W1, Q, W2 = synthetic.init_weights(36, d, Dc, K, device=dev)
nt = news.precompute(table, ops.pack_weights(W1, Q, W2, dtype=dt))
st = torch.cuda.current_stream()


def run(variant):
    if variant == "B":
        os.environ[alt] = altv
    else:
        os.environ.pop(alt, None)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    s = news.score(nt, hid, mask, cid, validate=False)
    b.record(st)
    torch.cuda.synchronize()
    return a.elapsed_time(b), s


sa = run("A")[1]
sb = run("B")[1]
ta, tb = [], []
for _ in range(reps):
    ta.append(run("A")[0])
    tb.append(run("B")[0])
rel = ((sa.double() - sb.double()).abs() / (sb.double().abs() + 1e-5 * sb.double().pow(2).mean().sqrt())).max()
ma, mb = statistics.median(ta), statistics.median(tb)
print(f"{dt} B={B}: A {ma:.3f} ms ({B * C / ma / 1e3:.1f} M pairs/s)  B({alt}) {mb:.3f} ms  "
      f"A/B {ma / mb:.3f}  max rel diff {float(rel):.2e}  finite {bool(torch.isfinite(sa).all())}", flush=True)
