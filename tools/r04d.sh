# Round-4 GPU A/B session: x2 variants (X2AB) and config-2 bf16 variants (C2AB)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/${1:-r04d}; mkdir -p $O
timeout -k 10 400 python3 tools/x2_ab.py ${X2AB:-cexp cur cur2 cur2_dsplit} > "$O/x2_ab.txt" 2>&1 || { tail -20 "$O/x2_ab.txt"; exit 1; }
cat "$O/x2_ab.txt"
timeout -k 10 300 python3 tools/bisect_news.py --dtype bf16 --B 400000 --d 256 --n-news 65238 ${C2AB:-wt:c2base wt:c2cw128 wt:c2cw128s} > "$O/c2_ab.txt" 2>&1 || { tail -20 "$O/c2_ab.txt"; exit 1; }
cat "$O/c2_ab.txt"
