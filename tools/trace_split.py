"""Per-launch durations of the headline kernel from a rocprofv3 kernel trace, split by bench phase:
the bench launches news_score_x2<0, false, 12, 2, false> first for its main line (W warmup + K timed
steps), later again for the full-history sub-line, so the trace's overall average mixes the two.

    python tools/trace_split.py TRACE_CSV [--warmup 5] [--steps 20] > summary.json
"""
import argparse
import csv
import json
import statistics

HEADLINE = "news_score_x2<0, false, 12, 2, false>"   # <ST, RAGGED, NCH, SHP, LOSS>

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--steps", type=int, default=20)
args = ap.parse_args()
rows = [r for r in csv.DictReader(open(args.trace)) if HEADLINE in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
main = ms[:args.warmup + args.steps]
timed = main[args.warmup:]
rest = ms[args.warmup + args.steps:]
print(json.dumps({
    "kernel": HEADLINE, "launches": len(ms),
    "main_line": {"launches": len(main), "timed_launches": len(timed),
                  "timed_avg_ms": round(statistics.mean(timed), 4) if timed else None,
                  "timed_median_ms": round(statistics.median(timed), 4) if timed else None},
    "later_launches (full-history sub-line)": {"launches": len(rest),
                                               "avg_ms": round(statistics.mean(rest), 4) if rest else None},
    "all_avg_ms": round(statistics.mean(ms), 4) if ms else None}, indent=1))
