#!/bin/bash
# Config 4 (52k-name synthetic KB) at its stated 10M articles on one GPU: kernel trace, then the bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt_c4_10m -o run -- \
    python3 bench.py --workload kb50k --total-docs 10000000 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bench_kt_c4_10m.log 2>&1 || exit $?
timeout -k 10 500 python bench.py --workload kb50k --total-docs 10000000 --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/bench_c4_10m.log 2>&1
echo "rc=$?" >> gpurun_out/bench_c4_10m.log
