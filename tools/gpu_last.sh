#!/bin/bash
# A/B of the DMA-issue priority in the production build, then the round-end check and profile set.
set -euo pipefail
TAG="${1:-r02_final9}"
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python3 tools/bisect_news.py --dtype fp32 --B 1000000 --reps 7 84dbcff a7ef53f a7ef53f 84dbcff 2>&1 | grep -v amdgpu.ids > gpurun_out/$TAG/ab_prio.txt
cat gpurun_out/$TAG/ab_prio.txt
bash tools/gpu_check.sh $TAG
bash tools/news32_profile.sh ${TAG}p
