#!/bin/bash
# Round-5 closing GPU session (tools/r05_final.sh TAG): the whole GPU test suite and smoke(), the
# PMC files whose sources or build flags changed since tools/r05_profile.sh (ff_fused<bf16> now
# built without SLP vectorizing; news_score32 for the fp32_mfma_exact sub-line), then the bench line.
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-r05f}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
echo "[final] gpu tests"
timeout -k 10 900 python -u -m pytest "$R/tests" -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 \
  || { tail -30 "$O/gpu_tests.log"; exit 1; }
tail -3 "$O/gpu_tests.log"
echo "[final] smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
tail -2 "$O/smoke.log"
bash "$R/tools/r05_pmc.sh" "$TAG" ff > "$O/pmc_ff.log" 2>&1 || { tail -5 "$O/pmc_ff.log"; exit 1; }
cd /tmp && export TMPDIR=/tmp
SQ1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
SQ2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
[ -n "${SKIP_N32:-}" ] && PASSES="" || PASSES=1
for pass in ${PASSES:+"FETCH_SIZE" "WRITE_SIZE" "$SQ2" "$SQ1"}; do
  i=$((i+1))
  echo "[final] news32 pmc pass $i"
  MINER_NEWS_FP32=mfma32 timeout -k 10 -s KILL 150 rocprofv3 --pmc $pass --kernel-trace -d "$O/n32_p$i" -o run --output-format csv -- \
    python3 "$R/tools/news_once.py" fp32 3000000 3 > "$O/n32_p$i.log" 2>&1 || { tail -5 "$O/n32_p$i.log"; exit 1; }
done
[ -n "$PASSES" ] && { python3 "$R/tools/pmc_traffic.py" --batch 3000000 --news32 "$O"/n32_p* > "$O/traffic_news32.txt" || exit 1; }
echo "[final] bench"
timeout -k 10 400 python3 "$R/bench.py" > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
cp "$R"/profiles/pmc_traffic*.json "$O/"
find "$O" -type f -size +4M -delete
echo "[final] done"
