#!/bin/bash
# every -m gpu test, then the config-2 bench line twice (envab format)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/envab.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
bash scripts/gpu_envab.sh KW_X=1
