#!/bin/bash
# Round-6 kernel trace of the default bench command: rocprofv3 --kernel-trace --stats (summary ->
# profiles/), the headline's timed launches split out (tools/trace_split.py). Usage: tools/r06_trace.sh TAG
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-r06trace}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
echo "[trace] kernel trace of the bench"
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- \
  python3 "$R/bench.py" > "$O/bench_traced.json" 2> "$O/trace.err" || { tail -20 "$O/trace.err"; exit 1; }
find "$O/trace" -name '*kernel_stats.csv' -exec cp {} "$O/kernel_stats.csv" \; -quit
python3 "$R/tools/trace_split.py" "$(find "$O/trace" -name '*kernel_trace.csv' | head -1)" > "$O/headline_trace_split.json"
cat "$O/headline_trace_split.json"
find "$O/trace" -type f -size +4M -print -delete
echo "[trace] done"
