#!/bin/bash
# One SQ counter pass per library variant tag (250k documents):  bash scripts_gpu_pmc_var.sh <outdir> tag...
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
out=$1; shift
for tag in "$@"; do
  if [ "$tag" = default ]; then unset KW_LIB; else export KW_LIB=$PWD/advanced_scrapper_amd/lib/libkwmatch_$tag.so; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/$out/$tag -o run -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 --docs-per-gpu 250000 > gpurun_out/${out}_$tag.log 2>&1 || exit $?
done
