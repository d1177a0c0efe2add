#!/bin/bash
# PMC passes (HBM bytes, L2 hits / misses, MFMA busy) of ranker builds: tools/rk_pmc.sh TAG VARIANT...
# (variants as tools/rk_ablate.py: built .so names, trailing "s" = the split form)
set -euo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="$1"; shift
O="$R/gpurun_out/$TAG"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  i=0
  for pass in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -k 10 -s KILL 150 rocprofv3 --pmc $pass --kernel-trace -d "$O/${v}_p$i" -o run --output-format csv -- \
      python3 "$R/tools/rk_ablate.py" "$v" > "$O/${v}_p$i.log" 2>&1
  done
done
find "$O" -name '*counter_collection.csv' | sort | while read f; do
  python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    if 'rk_fused' not in r['Kernel_Name']: continue
    acc[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']] += 1
for k in sorted(acc): print(sys.argv[1].split('/')[-2], k, '%.4g' % (acc[k] / max(1, n[k])), 'per dispatch over', n[k])
PY
done | tee "$O/pmc.txt"
