#!/bin/bash
# Round-end evidence at HEAD: every -m gpu test, smoke(), then config-5 profiles (kernel trace, FETCH/WRITE passes,
# bench line with its traffic) -- outputs under gpurun_out/.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit $?
ROUND=r03 ONLY=dedup bash scripts/gpu_configs.sh
