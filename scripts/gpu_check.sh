#!/bin/bash
# Every -m gpu test (one process), then a short bench line per workload named on the command line.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest_rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for w in "$@"; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/check_$w.log 2>&1 || exit $?
done
