#!/bin/bash
# Isolated kernel durations: every kernel of the scan on one stream (KW_SERIAL=1), rocprofv3 kernel-trace stats.
#   bash scripts/gpu_serial.sh <outdir> [bench args...]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp KW_DEV=1
mkdir -p gpurun_out
out=$1; shift
KW_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$out -o run -- python3 bench.py --steps 5 --warmup 1 --cpu-sample 0 "$@" > gpurun_out/$out.log 2>&1 || exit $?
python3 scripts/kstats.py gpurun_out/$out
