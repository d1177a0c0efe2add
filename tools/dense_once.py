"""Run the fused dense-row kernel (miner_score: miner_fused) `reps` times at the config-3 shape, for
rocprofv3 passes (tools/r05_pmc.sh).

    python tools/dense_once.py [bf16|fp32] [B] [reps]

fp32 is the bf16x6 form (S1 / S5 on the bf16 matrix cores) unless MINER_DENSE_FP32=mfma32.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from miner_amd import ops, synthetic  # noqa: E402

dev = "cuda:0"
dt = torch.bfloat16 if (len(sys.argv) < 2 or sys.argv[1] == "bf16") else torch.float32
B = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
L, C, K, D, Dc = 50, 40, 32, 768, 200
imp = synthetic.impressions(36, 0, B, L=L, d=D, C=C, device=dev, dtype=dt)
W1, Q, W2 = synthetic.init_weights(36, D, Dc, K, device=dev)
pw = ops.pack_weights(W1, Q, W2, dtype=dt)
for _ in range(reps):
    s = ops.score(imp.history, imp.his_mask, imp.candidates, pw)
torch.cuda.synchronize()
print("ok", float(s.float().abs().mean()))
