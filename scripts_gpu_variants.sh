#!/bin/bash
# Parity tests, then a short bench per library variant: bash scripts_gpu_variants.sh [tag ...]
# (tag "" = the default libkwmatch.so; others = lib/libkwmatch_<tag>.so built by build.build_kwmatch_variant)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest_rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/bench_default.log 2>&1 || exit $?
for t in "$@"; do
  KW_LIB=$PWD/advanced_scrapper_amd/lib/libkwmatch_$t.so timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bench_$t.log 2>&1 || exit $?
done
