"""Config-5 ranker A/B in one process: the split form (news slices + merge, XCD-shared users) vs the
unsplit one (MINER_RK_SPLIT=0), interleaved on the same inputs; top-k must be identical.
    python tools/rk_ab.py [U] [N] [reps]"""
import os
import sys

import torch

sys.path.insert(0, ".")
from miner_amd import corpus, synthetic  # noqa: E402

dev = "cuda:0"
U = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
N = int(sys.argv[2]) if len(sys.argv) > 2 else 200000
R = int(sys.argv[3]) if len(sys.argv) > 3 else 3
L, K, d, Dc, topk = 200, 64, 768, 200, 100
dt = torch.float16
g = torch.Generator(device=dev).manual_seed(5)
table = (torch.randn((N, d), generator=g, device=dev) / d ** 0.5).to(dt)
hid = torch.randint(0, N, (U, L), generator=g, device=dev, dtype=torch.int32)
mask = torch.rand((U, L), generator=g, device=dev) > 0.2
W1, Q, W2 = synthetic.init_weights(5, d, Dc, K, device=dev)
pk = corpus.pack_encoder(W1, Q, W2, dtype=dt)
mui, proj = corpus.encode_users(table, mask, pk, his_ids=hid)
torch.cuda.synchronize()
fl = U * N * 2 * 2 * K * d
res = {}
for variant in ["split", "unsplit"] * R:
    os.environ["MINER_RK_SPLIT"] = "1" if variant == "split" else "0"
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    s, i = corpus.rank_topk(mui, proj, table, topk)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    res.setdefault(variant, []).append(ms)
    out = (s.clone(), i.clone())
    if variant in res and len(res[variant]) == 1:
        res[variant + "_out"] = out
ok = torch.equal(res["split_out"][0], res["unsplit_out"][0]) and torch.equal(res["split_out"][1], res["unsplit_out"][1])
for v in ["split", "unsplit"]:
    t = min(res[v])
    print(f"{v:8s} U={U} N={N}: {t:.2f} ms (all {[round(x, 2) for x in res[v]]}) -> "
          f"{fl / (t / 1e3) / 1e12:.0f} TFLOP/s = {fl / (t / 1e3) / 1e12 / 2500:.3f} of fp16 peak")
print("top-k identical:", ok, flush=True)
