# Round-4 GPU session: bf16 news kernel early-DMA A/B (config 3 and config 2) + the config-2 bf16 stage profile
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${1:-r04n}; mkdir -p $O
timeout -k 10 300 python3 tools/bisect_news.py --dtype bf16 --B 1000000 wt:late wt:dearly > $O/bf16_ab.txt 2>&1 || { tail -20 $O/bf16_ab.txt; exit 1; }
cat $O/bf16_ab.txt
timeout -k 10 300 python3 tools/bisect_news.py --dtype bf16 --B 50000 --d 256 --n-news 65238 wt:late wt:dearly > $O/c2_ab.txt 2>&1 || { tail -20 $O/c2_ab.txt; exit 1; }
cat $O/c2_ab.txt
timeout -k 10 300 python3 tools/news_stages.py --dtype bf16 --d 256 --n-news 65238 --batch 50000 > $O/c2_stages.txt 2>&1 || { tail -20 $O/c2_stages.txt; exit 1; }
cat $O/c2_stages.txt
