#!/bin/bash
# Round-5 closing session for news_x2.hip's build flags (tools/r05_x2flags.sh TAG): the GPU test
# suite, the x2 counter files (config-3 MIND shape, its full-history form, config 2) re-taken on the
# new build, then the bench line. Each counter group is its own rocprofv3 run.
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-r05x}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
echo "[x2f] gpu tests"
timeout -k 10 600 python -u -m pytest "$R/tests" -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 \
  || { tail -30 "$O/gpu_tests.log"; exit 1; }
tail -1 "$O/gpu_tests.log"
cd /tmp && export TMPDIR=/tmp
SQ1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
SQ2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
SQ3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_CYCLES_VALU SQ_INST_CYCLES_SALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC"
run_passes() {   # name dtype batch d n_news npasses [full]
  local NM="$1" DT="$2" BB="$3" DD="$4" NN="$5" NP="$6" FULL="${7:-}" i=0
  for pass in "FETCH_SIZE" "WRITE_SIZE" "$SQ2" "$SQ1" "$SQ3"; do
    i=$((i+1))
    [ "$i" -gt "$NP" ] && break
    echo "[x2f] $NM pmc pass $i"
    timeout -k 10 -s KILL 150 rocprofv3 --pmc $pass --kernel-trace -d "$O/${NM}_p$i" -o run --output-format csv -- \
      python3 "$R/tools/news_once.py" "$DT" "$BB" 3 "$DD" "$NN" $FULL > "$O/${NM}_p$i.log" 2>&1 \
      || { echo "[x2f] $NM pass $i failed"; tail -5 "$O/${NM}_p$i.log"; return 1; }
  done
}
run_passes x2 fp32 3000000 768 104000 5 || exit 1
run_passes x2full fp32 3000000 768 104000 2 full || exit 1
run_passes c2x2 fp32 50000 256 65238 3 || exit 1
P="$R/tools/pmc_traffic.py"
python3 "$P" --batch 3000000 --tag "news_score_x2<0, false, 12, 2, false, false>" \
  --workload news_L50_K32_d768_C40_N104000_fp32 --kernel-name "news_score_x2<weighted,dense,12,MIND>" \
  --out "$R/profiles/pmc_traffic_news_x2.json" "$O"/x2_p* > "$O/traffic_x2.txt" || exit 1
python3 "$P" --batch 3000000 --tag "news_score_x2<0, false, 12, 2, false, false>" \
  --workload news_L50_K32_d768_C40_N104000_fp32_full --kernel-name "news_score_x2<weighted,dense,12,MIND>" \
  --out "$R/profiles/pmc_traffic_news_x2_full.json" "$O"/x2full_p* > "$O/traffic_x2full.txt" || exit 1
python3 "$P" --batch 50000 --tag "news_score_x2<0, false, 4, 2, false, false>" \
  --workload news_L50_K32_d256_C40_N65238_fp32 --kernel-name "news_score_x2<weighted,dense,4,MIND>" \
  --out "$R/profiles/pmc_traffic_news_c2_x2.json" "$O"/c2x2_p* > "$O/traffic_c2x2.txt" || exit 1
cp "$R"/profiles/pmc_traffic_news_x2.json "$R"/profiles/pmc_traffic_news_x2_full.json "$R"/profiles/pmc_traffic_news_c2_x2.json "$O/"
echo "[x2f] bench"
timeout -k 10 400 python3 "$R/bench.py" > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
find "$O" -type f -size +4M -delete
echo "[x2f] done"
