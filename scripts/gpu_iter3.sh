#!/bin/bash
# every -m gpu test, then a kernel-trace profile of the default bench (per-kernel averages)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt3 -o run -- \
    python3 bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/kt3.log 2>&1 || exit $?
python3 scripts/kstats.py gpurun_out/kt3
