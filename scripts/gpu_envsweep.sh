#!/bin/bash
# Bench lines under several environment settings: bash scripts/gpu_envsweep.sh "VAR=a" "VAR=b" ...  (dev aid)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/sweep_$i.log 2>&1 || exit $?
  echo "$e" >> gpurun_out/sweep_$i.log
done
