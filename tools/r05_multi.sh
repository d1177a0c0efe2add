#!/bin/bash
# Round-5 multi-purpose GPU session: tests, dense fp32 A/B builds, x2 A/B builds, then PMC passes.
#   tools/r05_multi.sh TAG "dense names" "x2 names" [pmc: dense|ff|all|none]
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-r05m}"; DENSE="${2:-}"; X2="${3:-}"; PMC="${4:-none}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests -m gpu --maxfail 25 -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > "$O/gpu_tests.log" 2>&1
rc=$?; tail -3 "$O/gpu_tests.log"
if [ $rc -ne 0 ]; then grep -E "FAILED|ERROR|Fatal|Abort" "$O/gpu_tests.log" | head -40; [ $rc -ge 124 ] && exit $rc; fi
if [ -n "$DENSE" ]; then
  timeout -k 10 400 python3 tools/dense_ab.py $DENSE $DENSE > "$O/dense_ab.txt" 2>&1 || { tail -20 "$O/dense_ab.txt"; exit 1; }
  cat "$O/dense_ab.txt"
fi
if [ -n "$X2" ]; then
  timeout -k 10 400 python3 tools/x2_ab.py $X2 > "$O/x2_ab.txt" 2>&1 || { tail -20 "$O/x2_ab.txt"; exit 1; }
  cat "$O/x2_ab.txt"
fi
if [ "$PMC" != none ]; then
  bash tools/r05_pmc.sh "$TAG/pmc" "$PMC" > "$O/pmc.log" 2>&1 || { tail -20 "$O/pmc.log"; exit 1; }
  tail -5 "$O/pmc.log"
  cat "$O"/pmc/traffic_*.txt 2>/dev/null | head -60
fi
echo "[multi] done"
