#!/bin/bash
# PMC passes over the FastFormer kernel (tools/ff_time.py): SQ stall breakdown, then the counters
# given as extra passes. Kernel-trace only (no sys/runtime trace with --pmc).
set -euo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/${TAG:-ffpmc}"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
B=${B:-20000}
rocprofv3 -L > "$O/counters.txt" 2>&1 || true
i=0
for pass in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES" "$@"; do
  i=$((i+1))
  echo "[ff_pmc] pass $i: $pass"
  timeout -k 10 300 rocprofv3 --pmc $pass --kernel-trace -d "$O/p$i" -o run --output-format csv -- \
    python3 "$R/tools/ff_time.py" --B $B --iters 2 > "$O/p$i.log" 2>&1
done
find "$O" -type f -size +4M -print -delete
echo "[ff_pmc] done"
