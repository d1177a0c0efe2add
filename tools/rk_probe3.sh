set -euo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/rk_probe3"; mkdir -p "$O"
timeout -k 10 60 "$R/tools/mb/xcc_map" | tee "$O/xcc_map.txt"
cd /tmp && export TMPDIR=/tmp
i=0
for pass in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  MINER_RK_SPLIT=1 timeout -k 10 -s KILL 150 rocprofv3 --pmc $pass --kernel-trace -d "$O/s$i" -o run --output-format csv -- \
    python3 "$R/tools/corpus_time.py" 2048 200000 > "$O/s$i.log" 2>&1
done
find "$O" -name '*counter_collection.csv' | while read f; do
  python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    if 'rk_fused' not in r['Kernel_Name']: continue
    acc[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']] += 1
for k in sorted(acc): print(sys.argv[1].split('/')[-2], k, acc[k] / max(1, n[k]), 'over', n[k], 'rows')
PY
done | tee "$O/pmc.txt"
