#!/bin/bash
# Kernel-trace stats (KW_SERIAL=1: one stream) of short bench runs at several corpus sizes: bash scripts/gpu_sizes.sh N...
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp KW_SERIAL=1
mkdir -p gpurun_out
for n in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sizes/$n -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 --docs-per-gpu $n --traffic-json none > gpurun_out/sizes_$n.log 2>&1 || exit $?
done
