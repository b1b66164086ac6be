#!/bin/bash
# Profile sets (build-matched PMC summaries) for the two bench configs with a
# committed summary, P3 and W2-length: kernel trace + FETCH_SIZE / WRITE_SIZE
# passes + summary + bench line each (scripts/gpu_profile_round.sh).
#   ROUND=r05 bash scripts/gpu_profile_all.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROUND=${ROUND:?set ROUND, e.g. r05} CFG=P3 PUSHES=8 bash scripts/gpu_profile_round.sh || exit $?
ROUND=${ROUND} CFG=W2-length PUSHES=6 EV=50000000 bash scripts/gpu_profile_round.sh || exit $?
exit 0
