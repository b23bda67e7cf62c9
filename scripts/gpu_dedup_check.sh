#!/bin/bash
# The dedup GPU tests, then the config-5 bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dedup.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_dedup_tests.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --workload dedup --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/check_dedup.log 2>&1
