"""The bench's headline step (config 3: per-news precompute of the 104,000 x 768 table + news_score_x2
over 3M impressions) with the two fp32 precompute forms, interleaved in one process on one box:
'pairs' = news.precompute (MINER_DTYPE_F32, the W1 / W2 products on fp16 pairs), 'mfma' = the same
step with the precompute's products on the fp32 MFMA (MINER_DTYPE_F32_MFMA) and the same pair split
after it. Prints the median ms per step and per precompute of each. Usage: python tools/pre_step_ab.py [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from miner_amd import _lib, news, ops, synthetic  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    dev = "cuda:0"
    B = 3_000_000
    g = torch.Generator().manual_seed(1)
    table = (torch.randn((bench.N_NEWS, bench.D), generator=g) / bench.D ** 0.5).to(dev)
    W1, Q, W2 = synthetic.init_weights(36, bench.D, bench.DC, bench.K, device=dev)
    pw = ops.pack_weights(W1, Q, W2, dtype=torch.float32)
    hid, mask, cid = bench.news_batch(7, B, bench.N_NEWS, dev)
    nt = news.precompute(table, pw, x2=True)
    lib = _lib.lib()

    def pre(form):
        if form == "pairs":
            return news.precompute(table, pw, out=nt, x2=True)
        st = torch.cuda.current_stream().cuda_stream
        rc = lib.miner_news_precompute(st, _lib.DTYPE_F32_MFMA, table.data_ptr(), bench.N_NEWS, pw.buf.data_ptr(),
                                       bench.D, bench.DC, bench.K, nt.logits.data_ptr(), nt.proj.data_ptr())
        assert rc == 0, rc
        news.split_x2(table, nt.x2.table2, nt.x2.table_unit)
        news.split_x2(nt.proj, nt.x2.proj2, nt.x2.proj_unit)
        return nt

    res = {"pairs": ([], []), "mfma": ([], [])}
    for i in range(reps + 2):
        for form in ("pairs", "mfma"):
            a, m, b = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            a.record()
            t = pre(form)
            m.record()
            news.score(t, hid, mask, cid, validate=False, x2=True)
            b.record()
            torch.cuda.synchronize()
            if i >= 2:
                res[form][0].append(a.elapsed_time(b))
                res[form][1].append(a.elapsed_time(m))
        print(f"rep {i}", flush=True)
    for form, (st, pr) in res.items():
        st, pr = sorted(st), sorted(pr)
        print(f"{form:5s}: step {st[len(st) // 2]:.3f} ms (min {st[0]:.3f}), precompute {pr[len(pr) // 2]:.3f} ms")


if __name__ == "__main__":
    main()
