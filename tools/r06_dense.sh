#!/bin/bash
# Round 6, dense fp32 on fp16 pairs: the stage profile of the fp32 kernel (stamps build), then the
# whole GPU test suite. Usage: tools/r06_dense.sh TAG
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-r06dense}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
echo "[dense] stages"
timeout -k 10 300 python3 -u tools/stage_profile.py --dtype f32 --batch 8192 > "$O/stages_f32.txt" 2>&1 || { tail -20 "$O/stages_f32.txt"; exit 1; }
cat "$O/stages_f32.txt"
echo "[dense] gpu tests"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { tail -40 "$O/gpu_tests.log"; exit 1; }
tail -3 "$O/gpu_tests.log"
echo "[dense] done"
