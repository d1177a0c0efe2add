"""Time config 5 (full-corpus ranking) pieces on one GPU: user encoder + users x news top-k."""
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from miner_amd import corpus, synthetic  # noqa: E402

dev = "cuda:0"
U = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
N = int(sys.argv[2]) if len(sys.argv) > 2 else 200000
L, K, d, Dc, topk = 200, 64, 768, 200, 100
dt = torch.float16
g = torch.Generator(device=dev).manual_seed(5)
table = (torch.randn((N, d), generator=g, device=dev) / d ** 0.5).to(dt)
hid = torch.randint(0, N, (U, L), generator=g, device=dev, dtype=torch.int32)
mask = torch.rand((U, L), generator=g, device=dev) > 0.2
W1, Q, W2 = synthetic.init_weights(5, d, Dc, K, device=dev)
pk = corpus.pack_encoder(W1, Q, W2, dtype=dt)
mui, proj = corpus.encode_users(table, mask, pk, his_ids=hid)
s, i = corpus.rank_topk(mui, proj, table, topk)
torch.cuda.synchronize()
e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
R = 3
te = tr = 0.0
for _ in range(R):
    e[0].record()
    mui, proj = corpus.encode_users(table, mask, pk, his_ids=hid)
    e[1].record()
    s, i = corpus.rank_topk(mui, proj, table, topk)
    e[2].record()
    torch.cuda.synchronize()
    te += e[0].elapsed_time(e[1]) / R
    tr += e[1].elapsed_time(e[2]) / R
pairs = U * N
fl_rank = pairs * (2 * 2 * K * d)
print(f"U={U} N={N}: encode {te:.2f} ms, rank {tr:.2f} ms -> {pairs / ((te + tr) / 1e3) / 1e9:.2f} G pairs/s; "
      f"rank {fl_rank / (tr / 1e3) / 1e12:.0f} TFLOP/s ({fl_rank / (tr / 1e3) / 1e12 / 2500 * 100:.1f}% of fp16 peak)", flush=True)
