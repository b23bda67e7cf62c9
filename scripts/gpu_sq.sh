#!/bin/bash
# SQ instruction / wait / LDS counters per kernel of a config-2 bench run (1M docs, one step), three
# separate rocprofv3 --pmc passes (each within the 8-SQ-counter limit):
#   [BENCH_ARGS='--workload kb50k'] bash scripts/gpu_sq.sh <outdir> [docs]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
D=${2:-1000000}
B="python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 --docs-per-gpu $D --traffic-json none $BENCH_ARGS"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/$1/a -o run -- $B > gpurun_out/$1_a.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/$1/b -o run -- $B > gpurun_out/$1_b.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL --output-format csv -d gpurun_out/$1/c -o run -- $B > gpurun_out/$1_c.log 2>&1
echo "sq_rc=$?" >> gpurun_out/$1_c.log
