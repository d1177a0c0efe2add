#!/bin/bash
# Round-5 GPU profiling session of the bench line (tools/r05_profile.sh TAG [B]):
#   1. PMC files of the dense miner_fused kernels and ff_fused<bf16> (tools/r05_pmc.sh),
#   2. rocprofv3 --kernel-trace --stats of the default bench command (summary -> profiles/),
#   3. PMC passes over tools/news_once.py (each counter group its own run) for the config-3 fp32
#      headline kernel news_score_x2, the bf16 kernel, and the config-2 (d = 256) forms of both,
#   4. the traffic / busy files bench.py reads (profiles/pmc_traffic_news*.json), then the bench line.
# The x2 tags are substrings of the demangled names news_score_x2<ST, RAGGED, NCH, SHP, LOSS, R3>.
set -euo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-r05}"; B="${2:-3000000}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
[ -n "${SKIP_PMC:-}" ] || bash "$R/tools/r05_pmc.sh" "$TAG" all   # SKIP_PMC=1: taken in an earlier call
cd /tmp && export TMPDIR=/tmp
echo "[profile] kernel trace of the bench"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- \
  python3 "$R/bench.py" > "$O/bench_traced.json" 2> "$O/trace.err"
find "$O/trace" -name '*kernel_stats.csv' -exec cp {} "$O/kernel_stats.csv" \; -quit
python3 "$R/tools/trace_split.py" "$(find "$O/trace" -name '*kernel_trace.csv' | head -1)" > "$O/headline_trace_split.json"
SQ1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
SQ2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
SQ3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_CYCLES_VALU SQ_INST_CYCLES_SALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC"
run_passes() {   # name dtype batch d n_news npasses [full]
  local NM="$1" DT="$2" BB="$3" DD="$4" NN="$5" NP="$6" FULL="${7:-}" i=0
  for pass in "FETCH_SIZE" "WRITE_SIZE" "$SQ2" "$SQ1" "$SQ3"; do
    i=$((i+1))
    [ "$i" -gt "$NP" ] && break
    echo "[profile] $NM pmc pass $i"
    timeout -k 10 -s KILL 150 rocprofv3 --pmc $pass --kernel-trace -d "$O/${NM}_p$i" -o run --output-format csv -- \
      python3 "$R/tools/news_once.py" "$DT" "$BB" 3 "$DD" "$NN" $FULL > "$O/${NM}_p$i.log" 2>&1
  done
}
run_passes x2 fp32 "$B" 768 104000 5
run_passes x2full fp32 "$B" 768 104000 2 full
run_passes bf16 bf16 "$B" 768 104000 5
run_passes c2x2 fp32 50000 256 65238 3
run_passes c2bf16 bf16 50000 256 65238 3
P="$R/tools/pmc_traffic.py"
python3 "$P" --batch "$B" --tag "news_score_x2<0, false, 12, 2, false, false>" \
  --workload news_L50_K32_d768_C40_N104000_fp32 --kernel-name "news_score_x2<weighted,dense,12,MIND>" \
  --out "$R/profiles/pmc_traffic_news_x2.json" "$O"/x2_p* > "$O/traffic_x2.txt"
python3 "$P" --batch "$B" --tag "news_score_x2<0, false, 12, 2, false, false>" \
  --workload news_L50_K32_d768_C40_N104000_fp32_full --kernel-name "news_score_x2<weighted,dense,12,MIND>" \
  --out "$R/profiles/pmc_traffic_news_x2_full.json" "$O"/x2full_p* > "$O/traffic_x2full.txt"
python3 "$P" --batch "$B" --news "$O"/bf16_p* > "$O/traffic_bf16.txt"
python3 "$P" --batch 50000 --tag "news_score_x2<0, false, 4, 2, false, false>" \
  --workload news_L50_K32_d256_C40_N65238_fp32 --kernel-name "news_score_x2<weighted,dense,4,MIND>" \
  --out "$R/profiles/pmc_traffic_news_c2_x2.json" "$O"/c2x2_p* > "$O/traffic_c2x2.txt"
python3 "$P" --batch 50000 --tag news_scoreIDF16bLi0ELb0ELi3ELi64ELi4ELi1E --tag "news_score<__bf16, 0, false, 3, 64, 4, 1>" \
  --workload news_L50_K32_d256_C40_N65238_bf16 --kernel-name "news_score<bf16,weighted,4 chunks,MIND>" \
  --out "$R/profiles/pmc_traffic_news_c2.json" "$O"/c2bf16_p* > "$O/traffic_c2bf16.txt"
for i in 1 2 3; do   # news_score32 (MINER_NEWS_FP32=mfma32: the bench's fp32_mfma_exact sub-line)
  pass="FETCH_SIZE"; [ $i = 2 ] && pass="WRITE_SIZE"; [ $i = 3 ] && pass="$SQ2"
  echo "[profile] news32 pmc pass $i"
  MINER_NEWS_FP32=mfma32 timeout -k 10 -s KILL 150 rocprofv3 --pmc $pass --kernel-trace -d "$O/n32_p$i" -o run --output-format csv -- \
    python3 "$R/tools/news_once.py" fp32 "$B" 3 > "$O/n32_p$i.log" 2>&1
done
python3 "$P" --batch "$B" --news32 "$O"/n32_p* > "$O/traffic_news32.txt"
cp "$R"/profiles/pmc_traffic*.json "$O/"
echo "[profile] bench"
timeout -k 10 400 python3 "$R/bench.py" > "$O/bench.json" 2> "$O/bench.err"
cat "$O/bench.json"
find "$O" -type f -size +4M -print -delete
echo "[profile] done"
