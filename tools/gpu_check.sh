#!/bin/bash
# GPU check: parity tests (every GPU test, one process), smoke, the default bench line.
set -euo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-check}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/gpu_tests.log" 2>&1 || { tail -40 "$O/gpu_tests.log"; exit 1; }
tail -3 "$O/gpu_tests.log"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
cat "$O/smoke.log"
timeout -k 10 400 python3 bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
cat "$O/bench.json"
