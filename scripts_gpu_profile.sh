#!/bin/bash
# Round profile: parity tests, rocprofv3 kernel-trace stats, PMC traffic passes (FETCH_SIZE / WRITE_SIZE in
# separate runs), then the full bench (with cpu_baseline) reading the traffic JSON.  Outputs under gpurun_out/.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROUND:-r01}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o run -- \
    python3 bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/bench_kt.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -o run -- \
    python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bench_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -o run -- \
    python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bench_write.log 2>&1 || exit $?
python3 profiles/pmc_traffic.py gpurun_out/traffic_$R.json gpurun_out/prof_fetch gpurun_out/prof_write \
    docs_per_gpu=1000000 seed=20250905 > gpurun_out/traffic.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --traffic-json gpurun_out/traffic_$R.json > gpurun_out/bench.log 2>&1
echo "rc=$?" >> gpurun_out/bench.log
