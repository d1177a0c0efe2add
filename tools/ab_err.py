"""A/B the fp32 score errors vs float64 of test_x2_error_vs_fp32_mfma[1.0-weighted] for the loaded lib:
prints the worst elements (b, c), their history length / unique count and the mui error there."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from miner_amd import news  # noqa: E402
from test_gpu_news import _setup, _f64_scores, FP32_KERNELS  # noqa: E402

table, hid, mask, cid, offs, W1, Q, W2 = _setup(34, 400, 50, 768, 6000, torch.float32)
ref = _f64_scores(table, hid, mask, cid, W1, Q, W2, "weighted")
for kern in FP32_KERNELS:
    os.environ["MINER_NEWS_FP32"] = kern
    nt = news.precompute(table, W1, Q, W2)
    s = news.score(nt, hid, mask, cid, score_type="weighted")
    torch.cuda.synchronize()
    e = (s.double().cpu() - ref).abs()
    top = torch.topk(e.flatten(), 4)
    out = []
    for v, i in zip(top.values.tolist(), top.indices.tolist()):
        b, c = divmod(i, e.shape[1])
        hb = hid[b].cpu()[mask[b].cpu()]
        out.append(f"(b={b} c={c} err={v:.3e} ref={float(ref[b, c]):.4e} len={len(hb)} uniq={len(set(hb.tolist()))})")
    print(kern, f"max={float(e.max()):.4e} rms={float(e.pow(2).mean().sqrt()):.4e}", *out, flush=True)
