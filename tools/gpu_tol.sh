# full GPU suite with every parity check recorded (test, tolerance, worst fraction)
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/tol; mkdir -p $O; rm -f $O/tol.jsonl
MINER_TOL_REPORT=$O/tol.jsonl timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
