set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab; mkdir -p $O; : > $O/ab.txt
export AB_ALT=MINER_NEWS_ABL
for v in $AB_LIST; do echo "abl=$v" | tee -a $O/ab.txt; AB_ALT_VALUE=$v timeout -k 10 120 python3 tools/news_ab.py ${AB_DT:-fp32} 131072 5 2>&1 | grep -v amdgpu.ids | tee -a $O/ab.txt; done
