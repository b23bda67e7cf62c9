#!/bin/bash
# Re-entry check: all GPU tests, bench, timing-variant breakdown, stage variants.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest_rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/bench.log 2>&1 || exit $?
KW_DUMP_TIMING=1 KW_LIB=$PWD/advanced_scrapper_amd/lib/libkwmatch_timing.so timeout -k 10 300 python bench.py --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/timing.log 2>&1 || exit $?
for st in 0 1; do
  KW_LIB=$PWD/advanced_scrapper_amd/lib/libkwmatch_stage$st.so timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/stage$st.log 2>&1 || exit $?
done
