#!/bin/bash
# One development iteration on the GPU box: every -m gpu test, a bench line, then a kernel trace with every
# kernel on one stream (KW_SERIAL=1: isolated durations) and (PMC=1) SQ counters of that serial run.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-sample 0 > gpurun_out/bench_iter.log 2>&1 || exit $?
KW_SERIAL=1 bash scripts/gpu_ktrace.sh serial default $VARIANTS || exit $?
if [ -n "$PMC" ]; then KW_SERIAL=1 bash scripts/gpu_pmc.sh pmcser || exit $?; fi
