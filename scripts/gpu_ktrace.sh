#!/bin/bash
# Kernel-trace stats of short bench runs per library variant: bash scripts/gpu_ktrace.sh <outdir> tag... (default = lib)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
out=$1; shift
mkdir -p gpurun_out
for tag in "$@"; do
  if [ "$tag" = default ]; then V=""; else V="--lib-variant $tag"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$out/$tag -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 $V > gpurun_out/${out}_$tag.log 2>&1 || exit $?
done
