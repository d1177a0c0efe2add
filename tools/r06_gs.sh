#!/bin/bash
# Round 6: the eval-loss Gram spread over the four mui waves. GPU tests of the news path + eval loop,
# then interleaved A/B of news_x2.hip builds (tools/bisect/libx2_<name>.so, tools/x2_ab.py --build):
# plain scoring and the eval-loss form. Usage: tools/r06_gs.sh TAG NAME1 NAME2 ...
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="$1"; shift
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
echo "[gs] tests"
timeout -k 10 900 python -u -m pytest tests/test_gpu_news.py tests/test_gpu_eval_loop.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1 || { tail -40 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
echo "[gs] A/B plain"
timeout -k 10 300 python -u tools/x2_ab.py "$@" > "$O/ab_plain.txt" 2>&1 || { tail -20 "$O/ab_plain.txt"; exit 1; }
cat "$O/ab_plain.txt"
echo "[gs] A/B loss"
X2AB_LOSS=1 timeout -k 10 300 python -u tools/x2_ab.py "$@" > "$O/ab_loss.txt" 2>&1 || { tail -20 "$O/ab_loss.txt"; exit 1; }
cat "$O/ab_loss.txt"
