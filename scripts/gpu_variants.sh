#!/bin/bash
# Bench each profiling/tuning variant lib/libkwmatch_<tag>.so named on the command line (plus the default);
# KW_DUMP_TIMING=1 makes FK_TIMING builds print their per-phase cycle counters.  BENCH_ARGS adds bench flags.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export KW_DUMP_TIMING=1
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-sample 0 $BENCH_ARGS > gpurun_out/var_default.log 2>&1 || exit $?
for tag in "$@"; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-sample 0 --lib-variant $tag $BENCH_ARGS > gpurun_out/var_$tag.log 2>&1 || exit $?
done
