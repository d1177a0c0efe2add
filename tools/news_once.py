"""Run the news-path scoring kernel `reps` times at config-3 shape (for rocprofv3 passes).

    python tools/news_once.py [fp32|bf16] [B] [reps] [d] [n_news] [full|pad] [loss]

``full``: every history holds L clicks (the bench's full_histories sub-line); ``loss``: the
eval-loss form (the per-impression disagreement D formed in the kernel, the bench's eval_with_loss).

fp32 runs the fp16-pair kernel news_score_x2 unless MINER_NEWS_FP32=mfma32 (news_score32). d = 256
with n_news = 65238 is config 2.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from miner_amd import news, ops, synthetic  # noqa: E402

dev = "cuda:0"
dt = torch.float32 if (len(sys.argv) < 2 or sys.argv[1] == "fp32") else torch.bfloat16
B = int(sys.argv[2]) if len(sys.argv) > 2 else 131072
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
d = int(sys.argv[4]) if len(sys.argv) > 4 else 768
n_news = int(sys.argv[5]) if len(sys.argv) > 5 else 104000
L, C, K, Dc = 50, 40, 32, 200
g = torch.Generator(device=dev).manual_seed(36)
table = (torch.randn((n_news, d), generator=g, device=dev) / d ** 0.5).to(dt)
full = len(sys.argv) > 6 and sys.argv[6] == "full"
lens = torch.full((B,), L, device=dev) if full else torch.randint(0, L + 1, (B,), generator=g, device=dev)
mask = torch.arange(L, device=dev)[None, :] >= (L - lens)[:, None]
hid = torch.randint(1, n_news, (B, L), generator=g, device=dev, dtype=torch.int32)
hid[~mask] = 0
cid = torch.randint(1, n_news, (B, C), generator=g, device=dev, dtype=torch.int32)
W1, Q, W2 = synthetic.init_weights(36, d, Dc, K, device=dev)
nt = news.precompute(table, ops.pack_weights(W1, Q, W2, dtype=dt))
loss = len(sys.argv) > 7 and sys.argv[7] == "loss"
for _ in range(reps):
    s = news.score(nt, hid, mask, cid, validate=False, disagreement=loss)
    s = s[0] if loss else s
torch.cuda.synchronize()
print("ok", float(s.float().abs().mean()))
