#!/bin/bash
# Round-5 batch: every -m gpu test, the FS_KEY_REGS A/B, then the config-2 round profile (kernel trace, FETCH /
# WRITE passes, bench line with its traffic).
cd "$GRAFT_REPO_ROOT" || exit 1
TESTS=1 bash scripts/gpu_libab.sh default kreg || exit $?
ROUND=r05 SKIP_TESTS=1 SKIP_DEDUP=1 bash scripts/gpu_profile.sh
