#!/bin/bash
# Config 5 only: kernel trace + the FETCH_SIZE / WRITE_SIZE passes + the bench line reading them.
#   ROUND=r04 bash scripts/gpu_dedup_prof.sh        outputs under gpurun_out/
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROUND:-r04}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt_dedup_$R -o run -- \
    python3 bench.py --workload dedup --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bench_kt_dedup_$R.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch_dedup_$R -o run -- \
    python3 bench.py --workload dedup --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/bench_fetch_dedup_$R.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write_dedup_$R -o run -- \
    python3 bench.py --workload dedup --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/bench_write_dedup_$R.log 2>&1 || exit $?
python3 profiles/pmc_traffic.py gpurun_out/traffic_dedup_$R.json gpurun_out/prof_fetch_dedup_$R gpurun_out/prof_write_dedup_$R \
    rows_per_gpu=500000000 seed=20250905 > gpurun_out/traffic_dedup_$R.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --workload dedup --traffic-json gpurun_out/traffic_dedup_$R.json > gpurun_out/bench_dedup_$R.log 2>&1
