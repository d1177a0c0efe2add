#!/bin/bash
# One GPU session for the config-3 news-path bench line: a kernel-trace profile of the bench
# command, the PMC passes (FETCH_SIZE / WRITE_SIZE / SQ, each its own run, kernel-trace only), the
# traffic summary (profiles/pmc_traffic_news.json, read by bench.py), then the bench line itself.
set -euo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-news}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
B=131072
echo "[news_profile] kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu --no-dense > "$O/bench_traced.json" 2> "$O/trace.err"
for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT"; do
  name=$(echo "$pass" | cut -d' ' -f1 | tr 'A-Z' 'a-z')
  echo "[news_profile] pmc $pass"
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $pass --kernel-trace -d "$O/pmc_$name" -o run --output-format csv -- \
    python3 "$R/bench.py" --no-cpu --no-dense --steps 4 --warmup 1 --fp32-steps 0 > "$O/pmc_$name.json" 2> "$O/pmc_$name.err"
done
python3 "$R/tools/pmc_traffic.py" --news --batch $B --out "$R/profiles/pmc_traffic_news.json" "$O"/pmc_* > "$O/pmc_traffic.txt"
cp "$R/profiles/pmc_traffic_news.json" "$O/pmc_traffic_news.json"
find "$O" -name '*kernel_stats.csv' -exec cp {} "$O/kernel_stats.csv" \; -quit
echo "[news_profile] bench"
timeout -k 10 400 python3 "$R/bench.py" > "$O/bench.json" 2> "$O/bench.err"
cat "$O/bench.json"
find "$O" -type f -size +4M -print -delete
echo "[news_profile] done"
