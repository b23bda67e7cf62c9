#!/bin/bash
# Config 4 (~50k-pattern KB): GPU parity vs the fixture and the live oracle, then a short kb50k bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_c4.py -x -v --timeout 300 --timeout-method thread > gpurun_out/c4_tests.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --workload kb50k --steps 3 --warmup 1 --cpu-sample ${CPU_SAMPLE:-0} > gpurun_out/bench_c4.log 2>&1 || exit $?
