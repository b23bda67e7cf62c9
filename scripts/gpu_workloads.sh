#!/bin/bash
# The other BASELINE configs' bench lines: config 4 (kb50k) and config 5 (dedup).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --workload kb50k --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/wl_kb50k.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --workload dedup --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/wl_dedup.log 2>&1 || exit $?
