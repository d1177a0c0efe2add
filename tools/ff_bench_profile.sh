set -euo pipefail
R="$(pwd)"
O="$R/gpurun_out/ffbench"
mkdir -p "$O"
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q -p no:cacheprovider > "$O/gpu_tests.log" 2>&1; tail -2 "$O/gpu_tests.log"
timeout -k 10 300 python3 bench.py > "$O/bench_c3.json" 2> "$O/bench_c3.err"; cat "$O/bench_c3.json"
timeout -k 10 300 python3 bench.py --workload fastformer > "$O/bench_ff.json" 2> "$O/bench_ff.err"; cat "$O/bench_ff.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- python3 "$R/bench.py" --workload fastformer --no-cpu --steps 20 > "$O/bench_ff_traced.json" 2> "$O/trace.err"
find "$O" -name '*kernel_stats.csv' -exec cp {} "$O/ff_kernel_stats.csv" \; -quit
find "$O" -type f -size +4M -delete
echo done
