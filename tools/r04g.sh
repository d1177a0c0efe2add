# Round-4 GPU session: news-path parity tests + x2 A/B (X2AB names)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${1:-r04g}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_news.py tests/test_gpu_eval_loop.py tests/test_gpu_fullsize.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; grep -E "^FAILED|Error" $O/tests.log | head -20
[ $rc -ge 124 ] && exit $rc
timeout -k 10 400 python3 tools/x2_ab.py ${X2AB:-cur3 pad ahead cexp} > "$O/x2_ab.txt" 2>&1 || { tail -20 "$O/x2_ab.txt"; exit 1; }
cat "$O/x2_ab.txt"
