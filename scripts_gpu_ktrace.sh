#!/bin/bash
# Kernel-trace stats of a short bench run: bash scripts_gpu_ktrace.sh <outdir> [bench args...]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
out=$1; shift
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$out -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 "$@" > gpurun_out/$out.log 2>&1
