#!/bin/bash
# GPU session script: parity tests, bench, rocprofv3 kernel-trace summary.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest_rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench_rc=$rc" >> gpurun_out/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 1 --cpu-sample 0 > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
echo "prof_rc=$?" >> "$GRAFT_REPO_ROOT/gpurun_out/prof.log"
