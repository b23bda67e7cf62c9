#!/bin/bash
# SQ counters and HBM traffic of the dedup kernels (config 5 at 100M rows, one step), three rocprofv3 --pmc passes.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python3 bench.py --workload dedup --steps 1 --warmup 0 --cpu-sample 0 --rows-per-gpu 100000000"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/sqdd/a -o run -- $B > gpurun_out/sqdd_a.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/sqdd/b -o run -- $B > gpurun_out/sqdd_b.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/sqdd/c -o run -- $B > gpurun_out/sqdd_c.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/sqdd/d -o run -- $B > gpurun_out/sqdd_d.log 2>&1
