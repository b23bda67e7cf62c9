#!/bin/bash
# Round-4 record at HEAD: every -m gpu test, smoke, the config-2 and config-5 profiles (kernel stats, PMC
# FETCH/WRITE, bench lines with traffic), the config-2 SQ passes, the 10M one-GPU line.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
ROUND=r04 SKIP_TESTS=1 bash scripts/gpu_profile.sh || exit $?
bash scripts/gpu_sq.sh r04sq || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-sample 0 --total-docs 10000000 > gpurun_out/bench_c3n1.log 2>&1
