#!/bin/bash
# Parity tests (all -m gpu) + one short bench (dev loop); extra args: more bench workloads (e.g. kb50k)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest_rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/var_default.log 2>&1 || exit $?
for w in "$@"; do
  timeout -k 10 400 python bench.py --workload $w --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/wl_$w.log 2>&1 || exit $?
done
