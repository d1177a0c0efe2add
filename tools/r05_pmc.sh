#!/bin/bash
# Round-5 PMC session (counter files for the dense miner_fused kernel in
# both fp32 forms' default (bf16x6) and bf16, and for ff_fused<bf16>). Each counter group is its own
# rocprofv3 run (kernel trace only, no sys/runtime trace with --pmc), then tools/pmc_traffic.py folds
# the passes into profiles/pmc_traffic_*.json bound to the kernel sources' sha.
#   tools/r05_pmc.sh TAG [which: dense ff wide all]
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-r05pmc}"; WHICH="${2:-all}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
SQ1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
SQ2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
SQ3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_CYCLES_VALU SQ_INST_CYCLES_SALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC"
passes() {   # name cmd...
  local NM="$1"; shift
  local i=0
  for pass in "FETCH_SIZE" "WRITE_SIZE" "$SQ2" "$SQ1" "$SQ3"; do
    i=$((i+1))
    echo "[pmc] $NM pass $i"
    timeout -k 10 -s KILL 150 rocprofv3 --pmc $pass --kernel-trace -d "$O/${NM}_p$i" -o run --output-format csv -- \
      "$@" > "$O/${NM}_p$i.log" 2>&1 || { echo "[pmc] $NM pass $i failed"; tail -5 "$O/${NM}_p$i.log"; return 1; }
  done
}
P="$R/tools/pmc_traffic.py"
if [ "$WHICH" = dense ] || [ "$WHICH" = all ]; then
  passes dbf16 python3 "$R/tools/dense_once.py" bf16 32768 3 || exit 1
  passes dfp32 python3 "$R/tools/dense_once.py" fp32 8192 3 || exit 1
  python3 "$P" --batch 32768 --source miner_score "$O"/dbf16_p* > "$O/traffic_dense_bf16.txt"
  python3 "$P" --batch 8192 --tag "miner_fusedIfLi0E" --tag "miner_fused<float, 0" --source miner_score \
    --workload L50_K32_d768_Dc200_C40_fp32 --kernel-name "miner_fused<fp32,full> (bf16x6 S1/S5)" \
    --out "$R/profiles/pmc_traffic_dense_fp32.json" "$O"/dfp32_p* > "$O/traffic_dense_fp32.txt"
fi
if [ "$WHICH" = ff ] || [ "$WHICH" = all ]; then
  passes ffbf16 python3 "$R/tools/ff_time.py" --B 50000 --iters 2 || exit 1
  python3 "$P" --batch 50000 --tag "ff_fusedIDF16bLb1E" --tag "ff_fused<__bf16, true>" --tag "ff_fused<bool _Accum" --source fastformer \
    --workload ff_L50_H256_C40_bf16 --kernel-name "ff_fused<bf16,gather>" \
    --out "$R/profiles/pmc_traffic_ff_bf16.json" "$O"/ffbf16_p* > "$O/traffic_ff_bf16.txt"
fi
if [ "$WHICH" = ffqfold ]; then     # the FF_QFOLD=1 build (tools/ff_flag_ab.py --build qfold -DFF_QFOLD=1)
  passes ffq python3 "$R/tools/ff_flag_ab.py" qfold || exit 1
  python3 "$P" --batch 50000 --tag "ff_fusedIDF16bLb1E" --tag "ff_fused<__bf16, true>" --tag "ff_fused<bool _Accum" --source fastformer \
    --workload ff_L50_H256_C40_bf16_qfold --kernel-name "ff_fused<bf16,gather> FF_QFOLD=1" \
    --out "$R/profiles/pmc_traffic_ff_bf16_qfold.json" "$O"/ffq_p* > "$O/traffic_ff_bf16_qfold.txt"
fi
cp "$R"/profiles/pmc_traffic*.json "$O/" 2>/dev/null
find "$O" -type f -size +4M -print -delete
echo "[pmc] done"
