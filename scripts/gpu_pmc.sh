#!/bin/bash
# SQ instruction / cycle counters per kernel of a 250k-document bench run, two passes:
#   bash scripts/gpu_pmc.sh <outdir> [library variant tag]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
V=""; if [ -n "$2" ]; then V="--lib-variant $2"; fi
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/$1/a -o run -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 --docs-per-gpu 250000 --traffic-json none $V > gpurun_out/$1_a.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/$1/b -o run -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 --docs-per-gpu 250000 --traffic-json none $V > gpurun_out/$1_b.log 2>&1
