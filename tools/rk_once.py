"""The bench's config-5 step (bench.py config5_subline: 2,048 users x 200,000 news, L = 200, K = 64,
d = 768, fp16, top-100) `reps` times, for rocprofv3 passes (tools/r06_pmc.sh).

    python tools/rk_once.py [reps]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from miner_amd import corpus, synthetic  # noqa: E402

dev = "cuda:0"
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
U, L, K, N, D, DC, TOPK = 2048, 200, 64, 200_000, 768, 200, 100
dt = torch.float16
g = torch.Generator(device=dev).manual_seed(5)
table = (torch.randn((N, D), generator=g, device=dev) / D ** 0.5).to(dt)
W1, Q, W2 = synthetic.init_weights(5, D, DC, K, device=dev)
pk = corpus.pack_encoder(W1, Q, W2, dtype=dt)
hid = torch.randint(0, N, (U, L), generator=g, device=dev, dtype=torch.int32)
lens = torch.randint(1, L + 1, (U,), generator=g, device=dev)
mask = torch.arange(L, device=dev)[None, :] >= (L - lens)[:, None]
for _ in range(reps):
    mui, proj = corpus.encode_users(table, mask, pk, his_ids=hid)
    s, i = corpus.rank_topk(mui, proj, table, TOPK)
torch.cuda.synchronize()
print("ok", float(s[:, 0].mean()))
