#!/bin/bash
# Config-5 ranker probe: time rk_fused at three table sizes (L2-resident, Infinity-Cache-resident,
# the bench's 200k rows), then PMC passes (HBM bytes, L2 hit rate, SQ busy) on the bench size.
set -euo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/${1:-rk_probe}"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python3 tools/rk_ablate.py 0 1 2 4 5 6 8 15 2>&1 | grep -v amdgpu.ids | tee -a "$O/ablate.txt"
cd /tmp && export TMPDIR=/tmp
i=0
for pass in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 150 rocprofv3 --pmc $pass --kernel-trace -d "$O/p$i" -o run --output-format csv -- \
    python3 "$R/tools/corpus_time.py" 2048 200000 > "$O/p$i.log" 2>&1
done
find "$O" -name '*counter_collection.csv' | while read f; do
  python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    if 'rk_fused' not in r['Kernel_Name']: continue
    acc[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']] += 1
for k in sorted(acc): print(sys.argv[1].split('/')[-3], k, acc[k] / max(1, n[k] // 1), 'over', n[k], 'rows')
PY
done | tee "$O/pmc.txt"
