"""Interleaved A/B of the FastFormer kernel (config 4: 50k impressions, L=50, C=40, bf16) against
an experiment bit set of MINER_FF_ABL; prints median ms per launch and the max score difference.

    python tools/ff_ab.py ABL_VALUE [B] [reps]
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from miner_amd import fastformer as ff  # noqa: E402
from miner_amd import synthetic  # noqa: E402

v = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 50000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 7
dev = "cuda:0"
n_news = 65238
table = synthetic.news_table(1, n_news, 256, device=dev, dtype=torch.bfloat16)
beh = synthetic.behaviors(1, 0, B, L=50, n_news=n_news, C=40, device=dev)
packed = ff.pack(synthetic.fastformer_params(0).to(dev), torch.bfloat16)


def run(alt):
    if alt:
        os.environ["MINER_FF_ABL"] = v
    else:
        os.environ.pop("MINER_FF_ABL", None)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    s = ff.score_gather(table, beh.his_ids, beh.his_mask, beh.cand_ids, packed, cand_offsets=beh.cand_offsets,
                        validate=False)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b), s


sa, sb = run(False)[1], run(True)[1]
ta, tb = [], []
for _ in range(reps):
    ta.append(run(False)[0])
    tb.append(run(True)[0])
print(f"fastformer bf16 B={B}: A {statistics.median(ta):.3f} ms  B(MINER_FF_ABL={v}) {statistics.median(tb):.3f} ms  "
      f"A/B {statistics.median(ta) / statistics.median(tb):.3f}  max |diff| {float((sa - sb).abs().max()):.2e}", flush=True)
