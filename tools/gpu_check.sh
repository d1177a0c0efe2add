#!/bin/bash
# GPU check: parity tests (every GPU test, one process), smoke, the default bench line.
#   tools/gpu_check.sh TAG [pytest -k expression]
set -euo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-check}"
K="${2:-}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python3 -u -m pytest tests -m gpu ${K:+-k "$K"} --maxfail 25 -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > "$O/gpu_tests.log" 2>&1 || { grep -E "FAILED|ERROR|passed|failed" "$O/gpu_tests.log" | tail -40; exit 1; }
tail -3 "$O/gpu_tests.log"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
cat "$O/smoke.log"
timeout -k 10 600 python3 bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
cat "$O/bench.json"
