set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/x6; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_news.py tests/test_gpu_eval_loop.py tests/test_gpu_modules.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
export AB_ALT=MINER_NEWS_ABL AB_ALT_VALUE=4096
timeout -k 10 300 python3 tools/news_ab.py fp32 131072 7 2>&1 | grep -v amdgpu.ids | tee $O/ab.txt
