#!/bin/bash
# rocprofv3 kernel trace of the default bench + the headline launches split by bench phase (tools/trace_split.py)
set -euo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r04tr"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- python3 "$R/bench.py" > "$O/bench_traced.json" 2> "$O/trace.err"
find "$O/trace" -name '*kernel_stats.csv' -exec cp {} "$O/kernel_stats.csv" \; -quit
python3 "$R/tools/trace_split.py" "$(find "$O/trace" -name '*kernel_trace.csv' | head -1)" > "$O/headline_trace_split.json"
cat "$O/headline_trace_split.json"
find "$O" -type f -size +4M -delete
