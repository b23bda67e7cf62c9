#!/bin/bash
# Config 3 on one GPU: the 10M-document GPU tests, then bench lines at 1M (config 2) and 10M (config 3, N = 1).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_c3.py -x -v -s --timeout 500 --timeout-method thread ${C3_K:+-k "$C3_K"} > gpurun_out/c3_tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-sample 0 > gpurun_out/bench_c2.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-sample 0 --total-docs 10000000 > gpurun_out/bench_c3n1.log 2>&1 || exit $?
timeout -k 10 120 python scripts/dump_hits.py > gpurun_out/dump_hits.log 2>&1 || exit $?
timeout -k 10 300 python scripts/e2e.py > gpurun_out/e2e.log 2>&1 || exit $?
