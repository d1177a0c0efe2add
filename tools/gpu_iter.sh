# quick GPU iteration: parity tests, per-stage profile of the single kernel, bench line
set -euo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$R/gpurun_out/iter"
mkdir -p "$O"
timeout -k 10 600 python3 -m pytest "$R/tests" -m gpu -x -q -p no:cacheprovider > "$O/gpu_tests.log" 2>&1 || { tail -30 "$O/gpu_tests.log"; exit 1; }
tail -2 "$O/gpu_tests.log"
timeout -k 10 300 python3 "$R/tools/stage_profile.py" > "$O/stages.txt" 2>&1 || { tail -20 "$O/stages.txt"; exit 1; }
cat "$O/stages.txt"
timeout -k 10 300 python3 "$R/bench.py" --no-cpu --fp32-steps 1 > "$O/bench.json" 2> "$O/bench.err"
python3 -c "import json;b=json.load(open('$O/bench.json'));print('VALUE',b['value'],b['roofline']['kernel_ms'],b['roofline']['frac'])"
