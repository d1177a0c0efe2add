set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/r05t"; mkdir -p "$O"
timeout -k 10 300 python -u tools/x2_ab.py base noslp > "$O/x2_noslp_ab.txt" 2>&1 || exit 1
timeout -k 10 200 python -u tools/dense_flag_ab.py base noslp > "$O/dense_noslp_ab.txt" 2>&1 || exit 1
timeout -k 10 200 python -u tools/dense_flag_ab.py --dtype bf16 --B 32768 base noslp > "$O/dense_bf16_noslp_ab.txt" 2>&1 || exit 1
timeout -k 10 300 python -u tools/rk_ablate.py 0 0n > "$O/rk_noslp_ab.txt" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- python3 "$R/bench.py" > "$O/bench_traced.json" 2> "$O/trace.err" || exit 1
python3 "$R/tools/trace_split.py" "$(find "$O/trace" -name '*kernel_trace.csv' | head -1)" > "$O/headline_trace_split.json"
find "$O/trace" -name '*kernel_stats.csv' -exec cp {} "$O/kernel_stats.csv" \; -quit
find "$O" -type f -size +4M -delete
