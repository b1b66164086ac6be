#!/bin/bash
# Round-4 profile sets (build-matched PMC summaries) for P3 and W2-length:
# kernel trace + FETCH_SIZE / WRITE_SIZE passes + summary + bench line each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROUND=${ROUND:-r04} CFG=P3 PUSHES=8 bash scripts/gpu_profile_round.sh || exit $?
ROUND=${ROUND:-r04} CFG=W2-length PUSHES=6 EV=50000000 bash scripts/gpu_profile_round.sh || exit $?
exit 0
