#!/bin/bash
# Round-end check: the plain-scoring A/B at d = 256 (fp32), then every GPU test, smoke, the default
# bench, and the profile set (rocprofv3 trace + PMC passes + bench).
set -euo pipefail
TAG="${1:-r02_final}"
mkdir -p gpurun_out/$TAG
AB_D=256 AB_ALT=MINER_NEWS_PLAIN_RT timeout -k 10 200 python3 tools/news_ab.py fp32 400000 9 2>&1 | grep -v amdgpu.ids > gpurun_out/$TAG/ab_plain_d256.txt
cat gpurun_out/$TAG/ab_plain_d256.txt
bash tools/gpu_check.sh $TAG
bash tools/news32_profile.sh ${TAG}p
