"""A/B of the bf16 kernels on config 3 in one process: pair (workspace) vs single-impression."""
import sys, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from miner_amd import ops, synthetic
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
dev = "cuda"
imp = synthetic.impressions(36, 0, B, L=50, d=768, C=40, device=dev, dtype=torch.bfloat16)
W1, Q, W2 = synthetic.init_weights(36, 768, 200, 32, device=dev)
pw = ops.pack_weights(W1, Q, W2, dtype=torch.bfloat16)
res = {}
for rnd in range(3):
    for name, ws in (("pair", True), ("single", False)):
        for _ in range(2):
            ops.score(imp.history, imp.his_mask, imp.candidates, pw, use_workspace=ws)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            ops.score(imp.history, imp.his_mask, imp.candidates, pw, use_workspace=ws)
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / 10
        res.setdefault(name, []).append(ms)
for k, v in res.items():
    print(f"{k:7s} ms/launch {min(v):.4f} (runs {', '.join(f'{x:.4f}' for x in v)})  -> {B * 40 / min(v) * 1e3 / 1e6:.1f} M pairs/s")
