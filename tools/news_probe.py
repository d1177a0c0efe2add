"""Diagnostic: news_score launch time vs news-table size and MINER_NEWS_ABL experiment bits, one
process (is the scoring kernel bound by the gather or by its own issue?). Config-3 shape.

    python tools/news_probe.py [--batch 131072] [--tables 4000,104000] [--abl 0,1,4]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from miner_amd import news, ops, synthetic  # noqa: E402

L, K, D, DC, C = 50, 32, 768, 200, 40


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=131072)
    ap.add_argument("--tables", default="4000,104000")
    ap.add_argument("--abl", default="0")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = "cuda:0"
    bf = torch.bfloat16
    W1, Q, W2 = synthetic.init_weights(36, D, DC, K, device=dev)
    pw = ops.pack_weights(W1, Q, W2, dtype=bf)
    for n in [int(x) for x in a.tables.split(",")]:
        g = torch.Generator(device=dev).manual_seed(36)
        table = (torch.randn((n, D), generator=g, device=dev) / D ** 0.5).to(bf)
        nt = news.precompute(table, pw)
        B = a.batch
        lens = torch.randint(0, L + 1, (B,), generator=g, device=dev)
        mask = torch.arange(L, device=dev)[None, :] >= (L - lens)[:, None]
        hid = torch.randint(1, n, (B, L), generator=g, device=dev, dtype=torch.int32)
        hid[~mask] = 0
        cid = torch.randint(1, n, (B, C), generator=g, device=dev, dtype=torch.int32)
        ref = None
        for rep in range(2):               # interleaved A/B, twice
            for abl in a.abl.split(","):
                os.environ["MINER_NEWS_ABL"] = abl
                out = news.score(nt, hid, mask, cid, validate=False)
                torch.cuda.synchronize()
                if ref is None:
                    ref = out.clone()
                same = bool(torch.equal(out, ref))
                s = torch.cuda.current_stream()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(a.iters):
                    news.score(nt, hid, mask, cid, validate=False)
                e1.record(s)
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / a.iters
                print(json.dumps({"n_news": n, "abl": int(abl), "rep": rep, "ms": round(ms, 4),
                                  "G_pairs_per_s": round(B * C / ms * 1e3 / 1e9, 4), "bit_equal": same}), flush=True)
        os.environ["MINER_NEWS_ABL"] = "0"
        del table, nt, hid, cid, mask, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
