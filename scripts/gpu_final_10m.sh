#!/bin/bash
# Round-end check plus the 10M-article lines: every -m gpu test, smoke(), the default bench line, config 3 on one
# GPU (10M articles, one scan) and config 4 at 10M.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_final_check.sh || exit $?
timeout -k 10 500 python bench.py --total-docs 10000000 --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/final_c3.log 2>&1 || exit $?
timeout -k 10 500 python bench.py --workload kb50k --total-docs 10000000 --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/final_c4_10m.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload kb50k > gpurun_out/final_c4.log 2>&1
