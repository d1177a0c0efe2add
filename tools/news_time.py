"""Time the news path at config-3 shape: precompute over the table + scoring (HIP events)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from miner_amd import news, ops, synthetic  # noqa: E402

dev = "cuda:0"
n_news = int(sys.argv[1]) if len(sys.argv) > 1 else 104000
B = int(sys.argv[2]) if len(sys.argv) > 2 else 131072
dtype = torch.float32 if (len(sys.argv) > 3 and sys.argv[3] == "fp32") else torch.bfloat16
L, C, d, K, Dc = 50, 40, 768, 32, 200
g = torch.Generator(device=dev).manual_seed(36)
table = (torch.randn((n_news, d), generator=g, device=dev) / d ** 0.5).to(dtype)
lens = torch.randint(0, L + 1, (B,), generator=g, device=dev)
mask = torch.arange(L, device=dev)[None, :] >= (L - lens)[:, None]
hid = torch.randint(1, n_news, (B, L), generator=g, device=dev, dtype=torch.int32)
hid[~mask] = 0
cid = torch.randint(1, n_news, (B, C), generator=g, device=dev, dtype=torch.int32)
W1, Q, W2 = synthetic.init_weights(36, d, Dc, K, device=dev)
pw = ops.pack_weights(W1, Q, W2, dtype=dtype)
nt = news.precompute(table, pw)
s = news.score(nt, hid, mask, cid, validate=False)
torch.cuda.synchronize()
st = torch.cuda.current_stream()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
N = 10
tp = ts = 0.0
for _ in range(N):
    ev[0].record(st)
    nt = news.precompute(table, pw, out=nt)
    ev[1].record(st)
    s = news.score(nt, hid, mask, cid, validate=False)
    ev[2].record(st)
    torch.cuda.synchronize()
    tp += ev[0].elapsed_time(ev[1])
    ts += ev[1].elapsed_time(ev[2])
tp /= N
ts /= N
es = 2 if dtype == torch.bfloat16 else 4
byt = B * (2 * L * d * es + C * d * es + L * K * 4 + L * 4 + L + C * 4 + C * 4)
print(f"{dtype} n_news={n_news} B={B}: precompute {tp:.3f} ms, score {ts:.3f} ms -> "
      f"{B * C / ((tp + ts) / 1e3) / 1e6:.1f} M pairs/s (score alone {B * C / (ts / 1e3) / 1e6:.1f} M; "
      f"{byt / (ts / 1e3) / 1e9:.0f} GB/s algorithmic)", flush=True)
