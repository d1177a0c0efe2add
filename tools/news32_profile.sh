#!/bin/bash
# One GPU session for the config-3 bench line (fp32 headline + bf16 mode) at the bench's batch:
#   1. rocprofv3 --kernel-trace --stats of the default bench command (its summary goes to profiles/),
#   2. PMC passes over tools/news_once.py for news_score32 (fp32) and news_score (bf16): HBM traffic
#      (FETCH_SIZE / WRITE_SIZE, each its own run) and the SQ issue counters (VALU / SALU / LDS / MFMA),
#   3. the traffic files bench.py reads (profiles/pmc_traffic_news{,_fp32}.json), then the bench line.
#   tools/news32_profile.sh TAG [B]
set -euo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-news32}"; B="${2:-3000000}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
echo "[profile] kernel trace of the bench"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- \
  python3 "$R/bench.py" > "$O/bench_traced.json" 2> "$O/trace.err"
find "$O/trace" -name '*kernel_stats.csv' -exec cp {} "$O/kernel_stats.csv" \; -quit
for DT in fp32 bf16; do
  i=0
  for pass in "FETCH_SIZE" "WRITE_SIZE" \
              "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
              "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE GRBM_COUNT" \
              "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_CYCLES_VALU SQ_INST_CYCLES_SALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC"; do
    i=$((i+1))
    echo "[profile] $DT pmc pass $i: $pass"
    timeout -k 10 -s KILL 150 rocprofv3 --pmc $pass --kernel-trace -d "$O/${DT}_p$i" -o run --output-format csv -- \
      python3 "$R/tools/news_once.py" "$DT" "$B" 3 > "$O/${DT}_p$i.log" 2>&1
  done
done
python3 "$R/tools/pmc_traffic.py" --news32 --batch "$B" "$O"/fp32_p* > "$O/traffic_fp32.txt"
python3 "$R/tools/pmc_traffic.py" --news --batch "$B" "$O"/bf16_p* > "$O/traffic_bf16.txt"
cp "$R/profiles/pmc_traffic_news_fp32.json" "$R/profiles/pmc_traffic_news.json" "$O/"
echo "[profile] bench"
timeout -k 10 400 python3 "$R/bench.py" > "$O/bench.json" 2> "$O/bench.err"
cat "$O/bench.json"
find "$O" -type f -size +4M -print -delete
echo "[profile] done"
