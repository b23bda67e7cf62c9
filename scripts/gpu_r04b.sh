#!/bin/bash
# Every -m gpu test (one process), then the end-to-end drop-in timing with a profile.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python scripts/e2e.py --profile > gpurun_out/e2e.log 2> gpurun_out/e2e_prof.log || exit $?
