#!/bin/bash
# Round 6, the split off-diagonal Gram with raw-published operands: news / eval-loop GPU tests, the
# A/B against the previous kept form, the x2-family counter files re-taken (news_x2.hip changed).
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-r06_fin2}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
bash tools/r06_gs.sh "$TAG" gs5 gs8 || exit 1
bash tools/r06_pmc.sh "${TAG}_pmc" x2 x2loss x2full c2x2 || exit 1
echo "[fin2] done"
