#!/bin/bash
# Round-4 final record at HEAD: scripts/gpu_r04d.sh (tests, smoke, config 2 + 5 profiles, SQ passes, 10M line),
# then config 4's profile (scripts/gpu_c4.sh).
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_r04d.sh || exit $?
ROUND=r04 bash scripts/gpu_c4.sh
