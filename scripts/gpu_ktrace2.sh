#!/bin/bash
# Kernel-trace stats of a short bench run per workload named on the command line (match / kb50k / dedup).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_$w -o run -- \
      python3 bench.py --workload $w --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/kt_$w.log 2>&1 || exit $?
done
