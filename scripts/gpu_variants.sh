#!/bin/bash
# Bench each profiling/tuning variant lib/libkwmatch_<tag>.so named on the command line (plus the default).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/var_default.log 2>&1 || exit $?
for tag in "$@"; do
  KW_LIB=$PWD/advanced_scrapper_amd/lib/libkwmatch_$tag.so timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/var_$tag.log 2>&1 || exit $?
done
