"""Timing of the wide path (miner_encode_users + miner_score_wide) on news ids.

    python tools/wide_time.py [B] [K] [L] [dtype]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from miner_amd import corpus, ops, synthetic  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
K = int(sys.argv[2]) if len(sys.argv) > 2 else 64
L = int(sys.argv[3]) if len(sys.argv) > 3 else 100
dt = torch.bfloat16 if (len(sys.argv) > 4 and sys.argv[4] == "bf16") else torch.float32
dev, n_news, d, C, Dc = "cuda:0", 104000, 768, 40, 200
g = torch.Generator(device=dev).manual_seed(1)
table = (torch.randn((n_news, d), generator=g, device=dev) / d ** 0.5).to(dt)
lens = torch.randint(0, L + 1, (B,), generator=g, device=dev)
mask = torch.arange(L, device=dev)[None, :] >= (L - lens)[:, None]
hid = torch.randint(1, n_news, (B, L), generator=g, device=dev, dtype=torch.int32)
cid = torch.randint(1, n_news, (B, C), generator=g, device=dev, dtype=torch.int32)
W1, Q, W2 = (w.to(dt) for w in synthetic.init_weights(1, d, Dc, K, device=dev))
pw = ops.pack_weights(W1, Q, W2)
enc = ops._wide_encoder(pw)
m8 = mask.view(torch.uint8)


def run():
    return ops.score_gather(table, hid, mask, cid, pw, validate=False)


run()
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
ev[0].record()
mui, proj = corpus.encode_users(table, mask, enc, his_ids=hid)
ev[1].record()
for _ in range(3):
    run()
ev[2].record()
torch.cuda.synchronize()
enc_ms = ev[0].elapsed_time(ev[1])
tot_ms = ev[1].elapsed_time(ev[2]) / 3
print(f"B={B} K={K} L={L} {dt}: encoder {enc_ms:.2f} ms, encoder + score_wide {tot_ms:.2f} ms "
      f"({B * C / tot_ms / 1e3:.1f} M pairs/s)")
