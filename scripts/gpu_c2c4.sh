#!/bin/bash
# The default config-2 bench line (twice), config 4 at 1M (twice) and at 10M articles (once), one GPU.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 3 --cpu-sample 0 > gpurun_out/c2_$rep.log 2>&1 || exit $?
done
for rep in 1 2; do
  timeout -k 10 300 python bench.py --workload kb50k --steps 20 --warmup 3 --cpu-sample 0 > gpurun_out/c4_$rep.log 2>&1 || exit $?
done
timeout -k 10 500 python bench.py --workload kb50k --total-docs 10000000 --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/c4_10m.log 2>&1
