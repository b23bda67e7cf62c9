#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
KW_DEBUG_TASKS=1 timeout -k 10 200 python bench.py --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/dbg_tasks.log 2>&1
