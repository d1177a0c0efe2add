set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/stages; mkdir -p $O
timeout -k 10 120 python3 tools/news_stages.py 2>&1 | grep -v amdgpu.ids | tee $O/x6.txt
MINER_NEWS_F32MFMA=1 timeout -k 10 120 python3 tools/news_stages.py 2>&1 | grep -v amdgpu.ids | tee $O/native.txt
