#!/bin/bash
# Round-6 closing session, part 2: the remaining counter groups (tools/r06_pmc.sh), then the bench
# line on the same tree. Usage: tools/r06_final.sh TAG [pmc groups...]
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-r06fin}"; shift || true
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
if [ "$#" -gt 0 ]; then bash "$R/tools/r06_pmc.sh" "${TAG}_pmc" "$@" || exit 1; fi
echo "[fin] bench"
cd "$R"
timeout -k 10 900 python3 "$R/bench.py" > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
python3 - "$O/bench.json" <<'PY'
import json, sys
t = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", t["value"], "ms/step", t["ms_per_step"], "roof", t["roofline"]["frac"], "traffic", t["roofline"].get("traffic"))
print("loss", t["eval_with_loss"]["vs_plain_kernel"], "pmc", t["pmc_status"])
print("c5 share", t["config5"]["per_gpu_share"])
PY
echo "[fin] done"
