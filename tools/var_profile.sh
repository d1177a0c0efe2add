set -euo pipefail
for v in MINER_PF_S13 MINER_PF_S16; do
  echo "=== $v"
  timeout -k 10 200 python3 tools/stage_profile.py --variant $v 2>&1 | grep -v amdgpu.ids
  timeout -k 10 200 python3 tools/stage_profile.py --variant $v --pair 2>&1 | grep -v amdgpu.ids
done
