#!/bin/bash
# Round profile: every -m gpu test, smoke(), rocprofv3 kernel-trace stats, PMC traffic passes (FETCH_SIZE /
# WRITE_SIZE in separate runs), then the full bench (with cpu_baseline) reading the traffic JSON.
#   ROUND=r02 [SKIP_TESTS=1] [SKIP_MAIN=1] [SKIP_DEDUP=1] bash scripts/gpu_profile.sh     outputs under gpurun_out/
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROUND:-r02}
LIBSHA=$(sha256sum advanced_scrapper_amd/lib/libkwmatch.so | cut -d' ' -f1)
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/gpu_tests_$R.log 2>&1 || exit $?
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$R.log 2>&1 || exit $?
fi
if [ -z "$SKIP_MAIN" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt_$R -o run -- \
      python3 bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/bench_kt_$R.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch_$R -o run -- \
      python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bench_fetch_$R.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write_$R -o run -- \
      python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bench_write_$R.log 2>&1 || exit $?
  python3 profiles/pmc_traffic.py gpurun_out/traffic_$R.json gpurun_out/prof_fetch_$R gpurun_out/prof_write_$R \
      scans=auto:kw_filter_kernel docs_per_gpu=1000000 seed=20250905 library_sha256=$LIBSHA > gpurun_out/traffic_$R.log 2>&1 || exit $?
  timeout -k 10 600 python bench.py --traffic-json gpurun_out/traffic_$R.json > gpurun_out/bench_$R.log 2>&1
  echo "rc=$?" >> gpurun_out/bench_$R.log
fi
# config 5 (dedup, 500M rows): kernel trace + the two PMC passes (one step each) + its bench line
if [ -z "$SKIP_DEDUP" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt_dedup_$R -o run -- \
      python3 bench.py --workload dedup --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bench_kt_dedup_$R.log 2>&1 || exit $?
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch_dedup_$R -o run -- \
      python3 bench.py --workload dedup --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/bench_fetch_dedup_$R.log 2>&1 || exit $?
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write_dedup_$R -o run -- \
      python3 bench.py --workload dedup --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/bench_write_dedup_$R.log 2>&1 || exit $?
  python3 profiles/pmc_traffic.py gpurun_out/traffic_dedup_$R.json gpurun_out/prof_fetch_dedup_$R gpurun_out/prof_write_dedup_$R \
      scans=auto:dd_transform_kernel rows_per_gpu=500000000 seed=20250905 library_sha256=$LIBSHA > gpurun_out/traffic_dedup_$R.log 2>&1 || exit $?
  timeout -k 10 600 python bench.py --workload dedup --traffic-json gpurun_out/traffic_dedup_$R.json > gpurun_out/bench_dedup_$R.log 2>&1
  echo "rc=$?" >> gpurun_out/bench_dedup_$R.log
fi
