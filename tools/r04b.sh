set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${1:-r04b}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_news.py tests/test_gpu_eval_loop.py tests/test_gpu_fullsize.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; grep -E "^FAILED|Error" $O/tests.log | head -20
[ $rc -ge 124 ] && exit $rc
shift || true
bash tools/r04_check.sh ${O#gpurun_out/} 0 1 "$@"
