#!/bin/bash
# Config 4 (the ~52k-name synthetic KB) at HEAD: kernel-trace stats, the FETCH_SIZE / WRITE_SIZE passes, the
# traffic JSON, and the bench line reading it.   ROUND=r04 bash scripts/gpu_c4.sh
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROUND:-r04}
LIBSHA=$(sha256sum advanced_scrapper_amd/lib/libkwmatch.so | cut -d' ' -f1)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt_c4_$R -o run -- \
    python3 bench.py --workload kb50k --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/bench_kt_c4_$R.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch_c4_$R -o run -- \
    python3 bench.py --workload kb50k --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bench_fetch_c4_$R.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write_c4_$R -o run -- \
    python3 bench.py --workload kb50k --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bench_write_c4_$R.log 2>&1 || exit $?
python3 profiles/pmc_traffic.py gpurun_out/traffic_c4_$R.json gpurun_out/prof_fetch_c4_$R gpurun_out/prof_write_c4_$R \
    scans=auto:kw_filter_kernel docs_per_gpu=1000000 seed=20250905 workload=kb50k library_sha256=$LIBSHA > gpurun_out/traffic_c4_$R.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --workload kb50k --traffic-json gpurun_out/traffic_c4_$R.json > gpurun_out/bench_c4_$R.log 2>&1
echo "rc=$?" >> gpurun_out/bench_c4_$R.log
