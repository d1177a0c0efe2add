#!/bin/bash
# Round 6 GPU session: the whole -m gpu suite, then an optional interleaved news_x2 A/B
# (tools/x2_ab.py names). Usage: tools/r06_check.sh TAG [AB NAMES...]
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="$1"; shift
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
echo "[chk] gpu tests"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$O/gpu_tests.log" 2>&1 || { tail -60 "$O/gpu_tests.log"; exit 1; }
tail -3 "$O/gpu_tests.log"
if [ "$#" -gt 0 ]; then
  echo "[chk] A/B"
  timeout -k 10 400 python -u tools/x2_ab.py "$@" > "$O/ab.txt" 2>&1 || { tail -20 "$O/ab.txt"; exit 1; }
  cat "$O/ab.txt"
fi
