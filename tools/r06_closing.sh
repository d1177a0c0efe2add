#!/bin/bash
# Round-6 closing session: the whole GPU suite, smoke, the default bench line, then the kernel trace
# of the same bench command. Usage: tools/r06_closing.sh TAG
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-r06close}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
echo "[close] gpu tests"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { tail -40 "$O/gpu_tests.log"; exit 1; }
tail -2 "$O/gpu_tests.log"
echo "[close] smoke"
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1 || { tail -20 "$O/smoke.txt"; exit 1; }
cat "$O/smoke.txt"
bash "$R/tools/r06_final.sh" "${TAG}_bench" || exit 1
bash "$R/tools/r06_trace.sh" "${TAG}_trace" || exit 1
echo "[close] done"
