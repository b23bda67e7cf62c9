#!/bin/bash
# Bench under each environment assignment given on the command line, e.g. KW_TASK_G=2,4,4,2;
# BENCH_ARGS (env) adds bench.py arguments, e.g. "--workload kb50k"
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 $BENCH_ARGS > gpurun_out/env_$i.log 2>&1 || exit $?
  echo "$e" >> gpurun_out/env_$i.log
done
