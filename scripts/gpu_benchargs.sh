#!/bin/bash
# Bench lines for several argument sets: bash scripts/gpu_benchargs.sh "--inflight 1" "--inflight 2" ...  (dev aid)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-sample 0 $a > gpurun_out/args_$i.log 2>&1 || exit $?
  echo "$a" >> gpurun_out/args_$i.log
done
