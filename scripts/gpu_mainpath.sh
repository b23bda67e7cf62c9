#!/bin/bash
# Main-path parity (-m gpu tests of the keyword scan: parity, capacity, config 3 at 10M, config 4) and then the
# config-2 and config-4 bench lines, two runs each (scripts/gpu_libab.sh):  bash scripts/gpu_mainpath.sh [tags...]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_capacity.py tests/test_gpu_c3.py tests/test_c4.py \
  -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/mainpath_tests.log 2>&1 || exit $?
T=${*:-default}
bash scripts/gpu_libab.sh $T && BENCH_ARGS='--workload kb50k' bash scripts/gpu_libab.sh $T
