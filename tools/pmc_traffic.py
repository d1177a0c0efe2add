"""Fold rocprofv3 PMC passes over bench.py into profiles/pmc_traffic.json (read by bench.py).

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py ...
    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES -d gpurun_out/pmc_sq ...
    python tools/pmc_traffic.py --batch 32768 gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_sq

Per launch of the bf16 scoring kernel (miner_fused<bf16, full>): the median over dispatches of each
counter (rows of one dispatch summed). HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are in KiB, and on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced stream
(16 B/lane loads and LDS-DMA alike), so hbm = (2·FETCH_SIZE + WRITE_SIZE)·1024. MFMA busy =
SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / XCDs · 4 SIMDs · CUs): GRBM_GUI_ACTIVE comes back
as one row per XCC, so the per-dispatch sum is XCDs x the kernel's busy cycles.
"""
import argparse
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.srcsha import KERNEL_SOURCES, source_sha16  # noqa: E402
KERNEL_TAG = "miner_fusedIDF16bLi0E"     # mangled miner_fused<__bf16, kFull, ...>
KERNEL_TAGS = [KERNEL_TAG, "miner_fused<__bf16, 0"]


def read_counters(d):
    per = defaultdict(lambda: defaultdict(float))   # dispatch -> counter -> value
    names = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                kn = row.get("Kernel_Name", "")
                if not any(tag in kn for tag in KERNEL_TAGS):
                    continue
                did = row.get("Dispatch_Id") or row.get("Correlation_Id")
                per[did][row["Counter_Name"]] += float(row["Counter_Value"])
                names[did] = kn
                SYMBOLS.add(kn)
    out = defaultdict(list)
    for did, cs in per.items():
        for c, v in cs.items():
            out[c].append(v)
    return {c: statistics.median(v) for c, v in out.items()}, len(per)


SYMBOLS = set()     # the kernel names the counter rows matched


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--batch", type=int, required=True)
    ap.add_argument("--cus", type=int, default=256)
    ap.add_argument("--xcds", type=int, default=8)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--news", action="store_true",
                    help="the news-path scoring kernel news_score<bf16, weighted, dense> (bench.py config3)")
    ap.add_argument("--news32", action="store_true",
                    help="the fp32 news-path scoring kernel news_score32<weighted, dense> (the bench headline)")
    ap.add_argument("--tag", action="append", default=None,
                    help="kernel-name substrings to match (mangled and demangled), with --workload / --kernel-name")
    ap.add_argument("--workload", default=None)
    ap.add_argument("--kernel-name", default=None)
    ap.add_argument("--source", default=None, choices=sorted(KERNEL_SOURCES),
                    help="kernel family whose sources the passes measured (bench.py rejects the file once they change)")
    args = ap.parse_args()
    workload, kernel = "L50_K32_d768_Dc200_C40_bf16", "miner_fused<bf16,full>"
    if args.tag:
        KERNEL_TAGS[:] = args.tag
        workload, kernel = args.workload, args.kernel_name or args.tag[0]
    if args.news:
        KERNEL_TAGS[:] = ["news_scoreIDF16bLi0ELb0E", "news_score<__bf16, 0, false>"]
        workload, kernel = "news_L50_K32_d768_C40_N104000_bf16", "news_score<bf16,weighted>"
        if args.out == os.path.join(ROOT, "profiles", "pmc_traffic.json"):
            args.out = os.path.join(ROOT, "profiles", "pmc_traffic_news.json")
    if args.news32:
        KERNEL_TAGS[:] = ["news_score32ILi0ELb0ELb0ELi24E", "news_score32<0, false, false, 24>", "news_score32<0, false, false, 24,"]
        workload, kernel = "news_L50_K32_d768_C40_N104000_fp32", "news_score<fp32,weighted>"
        if args.out == os.path.join(ROOT, "profiles", "pmc_traffic.json"):
            args.out = os.path.join(ROOT, "profiles", "pmc_traffic_news_fp32.json")
    med, n = {}, {}
    for d in args.dirs:
        if not os.path.isdir(d):
            continue
        m, k = read_counters(d)
        med.update(m)
        n[d] = k
    if "FETCH_SIZE" not in med or "WRITE_SIZE" not in med:
        sys.exit(f"missing FETCH_SIZE/WRITE_SIZE for {KERNEL_TAGS}: found {sorted(med)} ({n})")
    fetch = 2 * med["FETCH_SIZE"] * 1024
    write = med["WRITE_SIZE"] * 1024
    res = {
        "workload": workload, "batch": args.batch, "kernel": kernel,
        "dispatches": n, "FETCH_SIZE_KiB": med["FETCH_SIZE"], "WRITE_SIZE_KiB": med["WRITE_SIZE"],
        "hbm_read_bytes_per_launch": fetch, "hbm_write_bytes_per_launch": write,
        "hbm_bytes_per_launch": fetch + write,
        "correction": "reads = 2 x FETCH_SIZE (gfx950 half-count of 16B/lane streams), KiB -> bytes",
        "kernel_symbols": sorted(SYMBOLS),
    }
    src = args.source or ("news_x2" if args.tag and any("news_score_x2" in t for t in args.tag) else
                          "news" if (args.news or args.news32 or (args.tag and any("news_score" in t for t in args.tag)))
                          else "miner_score")
    res["source_files"] = list(KERNEL_SOURCES[src])
    res["source_sha16"] = source_sha16(KERNEL_SOURCES[src])
    if "SQ_VALU_MFMA_BUSY_CYCLES" in med and "GRBM_GUI_ACTIVE" in med:
        res["SQ_VALU_MFMA_BUSY_CYCLES"] = med["SQ_VALU_MFMA_BUSY_CYCLES"]
        res["GRBM_GUI_ACTIVE"] = med["GRBM_GUI_ACTIVE"]
        gui = med["GRBM_GUI_ACTIVE"] / args.xcds
        res["gpu_busy_cycles"] = gui
        res["mfma_busy_frac"] = med["SQ_VALU_MFMA_BUSY_CYCLES"] / (gui * 4 * args.cus)
        # SQ_VALU_MFMA_BUSY_CYCLES counts matrix-pipe cycles (32 per v_mfma_f32_32x32x16_bf16, 16 per
        # 16x16x32 f16/bf16, 64 per 32x32x2_f32, 32 per 16x16x4_f32): expressed in 16-cycle units,
        # which is the instruction count for the 16x16x32 kernels (news_score_x2, news_score<bf16>)
        res["mfma_busy_16cycle_units"] = med["SQ_VALU_MFMA_BUSY_CYCLES"] / 16
    for c in sorted(med):
        if c.startswith(("SQ_", "GRBM_")) and c not in res:
            res[c] = med[c]
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
