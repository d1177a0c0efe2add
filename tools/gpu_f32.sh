set -euo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/f32
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_news.py tests/test_gpu_eval_loop.py tests/test_gpu_modules.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/f32/tests.log 2>&1 || { tail -30 gpurun_out/f32/tests.log; exit 1; }
tail -2 gpurun_out/f32/tests.log
timeout -k 10 300 python3 tools/news_ab.py fp32 131072 5
export AB_ALT=MINER_NEWS_ABL
for v in 8 4; do AB_ALT_VALUE=$v timeout -k 10 300 python3 tools/news_ab.py fp32 131072 3; done
