#!/bin/bash
# every -m gpu test, smoke(), and the default bench line (the driver's round-end sequence)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/final_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/final_bench.log 2>&1
