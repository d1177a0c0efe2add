set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/x6abl; mkdir -p $O; : > $O/abl.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_news.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
export AB_ALT=MINER_NEWS_F32MFMA
timeout -k 10 120 python3 tools/news_ab.py fp32 131072 5 2>&1 | grep -v amdgpu.ids | tee -a $O/abl.txt
timeout -k 10 120 python3 tools/news_stages.py 2>&1 | grep -v amdgpu.ids | tee $O/x6.txt
