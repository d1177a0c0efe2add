#!/bin/bash
# Round-5 GPU session: parity tests + smoke + bench, then (optional) the x2 stage profile and an
# interleaved A/B of x2 builds.   tools/r04_check.sh TAG [tests:0|1] [stages:0|1] [ab names...]
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-r05}"; TESTS="${2:-1}"; STAGES="${3:-0}"; shift 3 || true
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
if [ "$TESTS" = "1" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu --maxfail 25 -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > "$O/gpu_tests.log" 2>&1
  rc=$?; tail -3 "$O/gpu_tests.log"
  if [ $rc -ne 0 ]; then grep -E "FAILED|ERROR|Fatal|Abort" "$O/gpu_tests.log" | head -40; [ $rc -ge 124 ] && exit $rc; fi
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
  tail -2 "$O/smoke.log"
  timeout -k 10 600 python3 bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench.json'));print('value',d['value'],'kernel_ms',d['roofline']['kernel_ms'],'frac',d['roofline']['frac'])"
fi
if [ "$STAGES" = "1" ]; then
  timeout -k 10 300 python3 tools/news_stages.py --dtype x2 --batch 131072 > "$O/x2_stages.txt" 2>&1 || { tail -20 "$O/x2_stages.txt"; exit 1; }
  cat "$O/x2_stages.txt"
fi
if [ $# -gt 0 ]; then
  timeout -k 10 400 python3 tools/x2_ab.py "$@" > "$O/x2_ab.txt" 2>&1 || { tail -20 "$O/x2_ab.txt"; exit 1; }
  cat "$O/x2_ab.txt"
fi
