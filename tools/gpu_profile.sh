#!/bin/bash
# One GPU session: parity tests, the bench line, a kernel-trace profile of the same bench command,
# and the PMC passes (FETCH_SIZE / WRITE_SIZE / SQ in separate runs, kernel-trace only — no
# sys/runtime trace with --pmc). Every GPU step has its own time limit; the first failure ends it.
set -euo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-r01}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
B=32768
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  echo "[gpu_profile] tests"
  timeout -k 10 900 python3 -m pytest "$R/tests" -m gpu -x -q -p no:cacheprovider > "$O/gpu_tests.log" 2>&1
  timeout -k 10 300 python3 -c "import sys; sys.path.insert(0, \"$R\"); import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
  tail -1 "$O/smoke.log"
  tail -3 "$O/gpu_tests.log"
fi
echo "[gpu_profile] bench"
timeout -k 10 400 python3 "$R/bench.py" > "$O/bench.json" 2> "$O/bench.err"
cat "$O/bench.json"
echo "[gpu_profile] kernel trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu > "$O/bench_traced.json" 2> "$O/trace.err"
for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES"; do
  name=$(echo "$pass" | cut -d' ' -f1 | tr 'A-Z' 'a-z')
  echo "[gpu_profile] pmc $pass"
  timeout -k 10 300 rocprofv3 --pmc $pass --kernel-trace -d "$O/pmc_$name" -o run --output-format csv -- \
    python3 "$R/bench.py" --no-cpu --steps 4 --warmup 1 --fp32-steps 0 > "$O/pmc_$name.json" 2> "$O/pmc_$name.err"
done
python3 "$R/tools/pmc_traffic.py" --batch $B --out "$O/pmc_traffic.json" "$O"/pmc_*
# keep the summaries, drop bulky per-dispatch traces (gpurun copies back <= 64 MiB)
find "$O" -name '*kernel_stats.csv' -exec cp {} "$O/kernel_stats.csv" \; -quit
find "$O" -type f -size +4M -print -delete
du -sh "$O"
echo "[gpu_profile] done"
