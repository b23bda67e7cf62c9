#!/bin/bash
# __graft_entry__.smoke() on the GPU, then the bench for each library variant tag given.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
exec_bench() { timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-sample 0 > "$1" 2>&1; }
exec_bench gpurun_out/var_default.log || exit $?
for tag in "$@"; do
  KW_LIB=$PWD/advanced_scrapper_amd/lib/libkwmatch_$tag.so exec_bench gpurun_out/var_$tag.log || exit $?
done
