#!/bin/bash
# usage: pmc.sh <libtag or ""> <outdir>
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
LIBV=""; if [ -n "$1" ]; then LIBV="KW_LIB=$PWD/advanced_scrapper_amd/lib/libkwmatch_$1.so"; fi
env $LIBV true
export KW_LIB=${1:+$PWD/advanced_scrapper_amd/lib/libkwmatch_$1.so}
[ -z "$KW_LIB" ] && unset KW_LIB
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/$2 -o run -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 --docs-per-gpu 250000 > gpurun_out/$2.log 2>&1
