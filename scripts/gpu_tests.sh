#!/bin/bash
# Every -m gpu test, one process, per-test timeouts; then (optionally) one bench command given as arguments.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest_rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ $# -gt 0 ]; then timeout -k 10 600 "$@" > gpurun_out/bench_cmd.log 2>&1; echo "rc=$?" >> gpurun_out/bench_cmd.log; fi
