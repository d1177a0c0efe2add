#!/bin/bash
# PMC passes (each its own run, kernel-trace only) over tools/news_once.py; summary to stdout.
#   tools/news_pmc.sh TAG [fp32|bf16] [B]
set -euo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-pmc}"; DT="${2:-fp32}"; B="${3:-131072}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
i=0
for pass in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
            "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE GRBM_COUNT" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_CYCLES_VALU SQ_INST_CYCLES_SALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $pass --kernel-trace -d "$O/p$i" -o run --output-format csv -- \
    python3 "$R/tools/news_once.py" "$DT" "$B" 3 > "$O/p$i.log" 2>&1
done
python3 "$R/tools/pmc_summary.py" news_score "$O"/p* | tee "$O/summary.json"
find "$O" -type f -size +4M -delete
