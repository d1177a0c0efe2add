"""A/B of the config-5 ranker with the compile-time chunk count (default) against the run-time one
(AB_ENV, default MINER_RK_NCH_RT=1), interleaved in one process; top-k outputs compared exactly.

    python tools/corpus_ab.py [U] [N] [reps]
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from miner_amd import corpus, synthetic  # noqa: E402

dev = "cuda:0"
AB_ENV = os.environ.get("AB_ENV", "MINER_RK_NCH_RT")   # the variant B switch
U = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
N = int(sys.argv[2]) if len(sys.argv) > 2 else 200000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
L, K, d, Dc, topk = 200, 64, 768, 200, 100
dt = torch.float16
g = torch.Generator(device=dev).manual_seed(5)
table = (torch.randn((N, d), generator=g, device=dev) / d ** 0.5).to(dt)
hid = torch.randint(0, N, (U, L), generator=g, device=dev, dtype=torch.int32)
mask = torch.rand((U, L), generator=g, device=dev) > 0.2
W1, Q, W2 = synthetic.init_weights(5, d, Dc, K, device=dev)
pk = corpus.pack_encoder(W1, Q, W2, dtype=dt)
mui, proj = corpus.encode_users(table, mask, pk, his_ids=hid)


def run(rt):
    if rt:
        os.environ[AB_ENV] = "1"
    else:
        os.environ.pop(AB_ENV, None)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    out = corpus.rank_topk(mui, proj, table, topk)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b), out


oa, ob = run(False)[1], run(True)[1]
ta, tb = [], []
for _ in range(reps):
    ta.append(run(False)[0])
    tb.append(run(True)[0])
same = torch.equal(oa[0], ob[0]) and torch.equal(oa[1], ob[1])
print(f"rank U={U} N={N}: compile-time {statistics.median(ta):.2f} ms, run-time {statistics.median(tb):.2f} ms, "
      f"ratio {statistics.median(ta) / statistics.median(tb):.3f}, identical top-k {same}", flush=True)
