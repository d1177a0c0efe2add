#!/bin/bash
# PMC passes for the bench's fp32_mfma_exact sub-line (news_score32, MINER_NEWS_FP32=mfma32) ->
# profiles/pmc_traffic_news_fp32.json, bound to news.hip's sources.   tools/r04_fp32x.sh TAG [B]
set -euo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-r04fx}"; B="${2:-3000000}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
export MINER_NEWS_FP32=mfma32
i=0
for pass in "FETCH_SIZE" "WRITE_SIZE" \
            "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  echo "[profile] fp32 exact pmc pass $i"
  timeout -k 10 -s KILL 150 rocprofv3 --pmc $pass --kernel-trace -d "$O/fx_p$i" -o run --output-format csv -- \
    python3 "$R/tools/news_once.py" fp32 "$B" 3 > "$O/fx_p$i.log" 2>&1
done
python3 "$R/tools/pmc_traffic.py" --news32 --source news --batch "$B" "$O"/fx_p* > "$O/traffic_fx.txt"
cp "$R/profiles/pmc_traffic_news_fp32.json" "$O/"
find "$O" -type f -size +4M -print -delete
echo "[profile] done"
