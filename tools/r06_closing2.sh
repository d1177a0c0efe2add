#!/bin/bash
# Round-6 closing session 2: the dense counter files re-taken (miner_score.hip changed), then the
# whole GPU suite, smoke, the bench line and its kernel trace. Usage: tools/r06_closing2.sh TAG
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="${1:-r06close2}"
bash "$R/tools/r06_pmc.sh" "${TAG}_pmc" dense || exit 1
bash "$R/tools/r06_closing.sh" "$TAG" || exit 1
