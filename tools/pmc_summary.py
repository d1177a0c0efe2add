"""Median per-dispatch PMC counters of one kernel from rocprofv3 --pmc output directories.

    python tools/pmc_summary.py KERNEL_SUBSTRING DIR [DIR ...]
"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

tag = sys.argv[1]
per = defaultdict(lambda: defaultdict(float))
for d in sys.argv[2:]:
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if tag not in row.get("Kernel_Name", ""):
                    continue
                did = (d, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                per[did][row["Counter_Name"]] += float(row["Counter_Value"])
vals = defaultdict(list)
for cs in per.values():
    for c, v in cs.items():
        vals[c].append(v)
out = {c: statistics.median(v) for c, v in sorted(vals.items())}
print(json.dumps(out, indent=1))
