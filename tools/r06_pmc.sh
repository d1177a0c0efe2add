#!/bin/bash
# Round-6 counter session: every PMC file the bench line binds, re-taken on the round's sources (each
# counter group its own rocprofv3 run, kernel trace only; tools/pmc_traffic.py folds the passes and
# binds them to the kernel family's source sha). Usage: tools/r06_pmc.sh TAG [groups...]
# groups: x2 x2loss x2full c2x2 bf16 c2bf16 news32 dense ff rk (default: all)
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-r06pmc}"; shift || true
GROUPS_="${*:-x2 x2loss x2full c2x2 bf16 c2bf16 news32 dense ff rk}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
SQ1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
SQ2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
SQ3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_CYCLES_VALU SQ_INST_CYCLES_SALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC"
passes() {   # name npasses cmd...
  local NM="$1" NP="$2"; shift 2
  local i=0
  for pass in "FETCH_SIZE" "WRITE_SIZE" "$SQ2" "$SQ1" "$SQ3"; do
    i=$((i+1))
    [ "$i" -gt "$NP" ] && break
    echo "[pmc] $NM pass $i"
    timeout -k 10 -s KILL 180 rocprofv3 --pmc $pass --kernel-trace -d "$O/${NM}_p$i" -o run --output-format csv -- \
      "$@" > "$O/${NM}_p$i.log" 2>&1 || { echo "[pmc] $NM pass $i failed"; tail -5 "$O/${NM}_p$i.log"; return 1; }
  done
}
has() { case " $GROUPS_ " in *" $1 "*) return 0;; esac; return 1; }
P="$R/tools/pmc_traffic.py"
NO="$R/tools/news_once.py"
B=3000000
if has x2; then
  passes x2 5 python3 "$NO" fp32 $B 3 768 104000 || exit 1
  python3 "$P" --batch $B --tag "news_score_x2<0, false, 12, 2, false>" --tag news_score_x2ILi0ELb0ELi12ELi2ELb0EE \
    --workload news_L50_K32_d768_C40_N104000_fp32 --kernel-name "news_score_x2<weighted,dense,12,MIND>" \
    --out "$R/profiles/pmc_traffic_news_x2.json" "$O"/x2_p* > "$O/traffic_x2.txt" || exit 1
fi
if has x2loss; then
  passes x2loss 5 python3 "$NO" fp32 $B 3 768 104000 pad loss || exit 1
  python3 "$P" --batch $B --tag "news_score_x2<0, false, 12, 2, true>" --tag news_score_x2ILi0ELb0ELi12ELi2ELb1EE \
    --workload news_L50_K32_d768_C40_N104000_fp32_loss --kernel-name "news_score_x2<weighted,dense,12,MIND,LOSS>" \
    --out "$R/profiles/pmc_traffic_news_x2_loss.json" "$O"/x2loss_p* > "$O/traffic_x2loss.txt" || exit 1
fi
if has x2full; then
  passes x2full 2 python3 "$NO" fp32 $B 3 768 104000 full || exit 1
  python3 "$P" --batch $B --tag "news_score_x2<0, false, 12, 2, false>" --tag news_score_x2ILi0ELb0ELi12ELi2ELb0EE \
    --workload news_L50_K32_d768_C40_N104000_fp32_full --kernel-name "news_score_x2<weighted,dense,12,MIND>" \
    --out "$R/profiles/pmc_traffic_news_x2_full.json" "$O"/x2full_p* > "$O/traffic_x2full.txt" || exit 1
fi
if has c2x2; then
  passes c2x2 3 python3 "$NO" fp32 50000 3 256 65238 || exit 1
  python3 "$P" --batch 50000 --tag "news_score_x2<0, false, 4, 2, false>" --tag news_score_x2ILi0ELb0ELi4ELi2ELb0EE \
    --workload news_L50_K32_d256_C40_N65238_fp32 --kernel-name "news_score_x2<weighted,dense,4,MIND>" \
    --out "$R/profiles/pmc_traffic_news_c2_x2.json" "$O"/c2x2_p* > "$O/traffic_c2x2.txt" || exit 1
fi
if has bf16; then
  passes bf16 5 python3 "$NO" bf16 $B 3 768 104000 || exit 1
  python3 "$P" --batch $B --tag news_scoreIDF16bLi0ELb0ELi1ELi128ELi6ELi0EE --tag "news_score<__bf16, 0, false, 1, 128, 6, 0>" \
    --source news --workload news_L50_K32_d768_C40_N104000_bf16 --kernel-name "news_score<bf16,weighted>" \
    --out "$R/profiles/pmc_traffic_news.json" "$O"/bf16_p* > "$O/traffic_bf16.txt" || exit 1
fi
if has c2bf16; then
  passes c2bf16 3 python3 "$NO" bf16 50000 3 256 65238 || exit 1
  python3 "$P" --batch 50000 --tag news_scoreIDF16bLi0ELb0ELi3ELi64ELi4ELi1E --tag "news_score<__bf16, 0, false, 3, 64, 4, 1>" \
    --source news --workload news_L50_K32_d256_C40_N65238_bf16 --kernel-name "news_score<bf16,weighted,4 chunks,MIND>" \
    --out "$R/profiles/pmc_traffic_news_c2.json" "$O"/c2bf16_p* > "$O/traffic_c2bf16.txt" || exit 1
fi
if has news32; then   # news_score32 (MINER_NEWS_FP32=mfma32: the bench's fp32_mfma_exact sub-line)
  export MINER_NEWS_FP32=mfma32
  passes n32 3 python3 "$NO" fp32 $B 3 || exit 1
  unset MINER_NEWS_FP32
  python3 "$P" --batch $B --news32 --source news "$O"/n32_p* > "$O/traffic_news32.txt" || exit 1
fi
if has dense; then
  passes dbf16 5 python3 "$R/tools/dense_once.py" bf16 32768 3 || exit 1
  passes dfp32 5 python3 "$R/tools/dense_once.py" fp32 8192 3 || exit 1
  python3 "$P" --batch 32768 --source miner_score "$O"/dbf16_p* > "$O/traffic_dense_bf16.txt" || exit 1
  python3 "$P" --batch 8192 --tag "miner_fusedIfLi0E" --tag "miner_fused<float, 0" --source miner_score \
    --workload L50_K32_d768_Dc200_C40_fp32 --kernel-name "miner_fused<fp32,full> (bf16x6 S1/S5)" \
    --out "$R/profiles/pmc_traffic_dense_fp32.json" "$O"/dfp32_p* > "$O/traffic_dense_fp32.txt" || exit 1
fi
if has ff; then
  passes ffbf16 5 python3 "$R/tools/ff_time.py" --B 50000 --iters 2 --dense || exit 1
  python3 "$P" --batch 50000 --tag "ff_fusedIDF16bLb0E" --tag "ff_fused<__bf16, false>" --source fastformer \
    --workload ff_L50_H256_C40_bf16_dense --kernel-name "ff_fused<bf16,dense rows>" \
    --out "$R/profiles/pmc_traffic_ff_bf16.json" "$O"/ffbf16_p* > "$O/traffic_ff_bf16.txt" || exit 1
fi
if has rk; then
  passes rk 5 python3 "$R/tools/rk_once.py" 3 || exit 1
  python3 "$P" --batch 2048 --tag rk_fusedIDF16_ --tag "rk_fused<_Float16" --source corpus \
    --workload rk_U2048_N200000_L200_K64_d768_top100_fp16 --kernel-name "rk_fused<fp16,weighted,K=64,d=768>" \
    --out "$R/profiles/pmc_traffic_rk_fp16.json" "$O"/rk_p* > "$O/traffic_rk.txt" || exit 1
fi
cp "$R"/profiles/pmc_traffic*.json "$O/" 2>/dev/null
find "$O" -type f -size +4M -print -delete
echo "[pmc] done"
