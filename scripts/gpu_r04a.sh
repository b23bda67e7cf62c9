#!/bin/bash
# Round-4 batch: config-3 10M GPU tests, e2e with a profile, config-4 profile at HEAD, an --inflight 2 line.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_c3.py -x -v -s --timeout 500 --timeout-method thread > gpurun_out/c3_tests.log 2>&1 || exit $?
timeout -k 10 300 python scripts/e2e.py --profile > gpurun_out/e2e.log 2> gpurun_out/e2e_prof.log || exit $?
ROUND=r04 bash scripts/gpu_c4.sh || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-sample 0 --inflight 2 > gpurun_out/bench_inflight2.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-sample 0 > gpurun_out/bench_c2.log 2>&1 || exit $?
