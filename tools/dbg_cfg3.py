import os, sys, torch, numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from tests.conftest import load_golden
from miner_amd import news
g = load_golden("cfg3_slice")
dev = "cuda:0"
d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
for kern in ("mfma32", "x2"):
    os.environ["MINER_NEWS_FP32"] = kern
    nt = news.precompute(d(g["table"]), d(g["W1"]), d(g["Q"]), d(g["W2"]))
    for ret in (False, True):
        out = news.score(nt, d(g["his_ids"]), d(g["his_mask"]), d(g["cand_ids"]), return_user=ret)
        s = out[0] if ret else out
        torch.cuda.synchronize()
        err = (s.double().cpu() - torch.from_numpy(g["scores"]).double()).abs().amax(1)
        print(kern, "return_user" if ret else "plain", "per-imp max err", [f"{x:.2e}" for x in err.tolist()],
              "unique+1", [len(set(r)) for r in g["his_ids"].tolist()])
