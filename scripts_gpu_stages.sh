#!/bin/bash
# Parity tests + stage breakdown of the fast path (profiling variants built with -DFK_STAGE) + full bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest_rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for st in 0 1 2; do
  KW_LIB=$PWD/advanced_scrapper_amd/lib/libkwmatch_stage$st.so timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/stage$st.log 2>&1
  rc=$?; echo "rc=$rc" >> gpurun_out/stage$st.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/stage3.log 2>&1
echo "rc=$?" >> gpurun_out/stage3.log
