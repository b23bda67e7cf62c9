#!/bin/bash
# The dedup GPU tests (one process), then config 5's bench line; KT=1 adds a kernel-trace run.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dedup.py -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/dedup_tests.log 2>&1
rc=$?; echo "pytest_rc=$rc" >> gpurun_out/dedup_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --workload dedup --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/dedup_bench.log 2>&1 || exit $?
if [ -n "$KT" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt_dedup -o run -- \
      python3 bench.py --workload dedup --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/dedup_kt.log 2>&1 || exit $?
fi
