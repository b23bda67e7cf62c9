#!/bin/bash
# The other BASELINE configs at HEAD: end-to-end drop-in timing (scripts/e2e.py), config 4 (kb50k) and
# config 5 (dedup): rocprofv3 kernel-trace stats, FETCH_SIZE / WRITE_SIZE passes, then each bench line.
#   ROUND=r03 [ONLY="e2e c4 dedup"] bash scripts/gpu_configs.sh        outputs under gpurun_out/
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROUND:-r03}
ONLY=${ONLY:-"e2e c4 dedup"}
prof() {   # prof <tag> <bench args...>
  local t=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt_${t}_$R -o run -- \
      python3 bench.py "$@" --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bench_kt_${t}_$R.log 2>&1 || return $?
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch_${t}_$R -o run -- \
      python3 bench.py "$@" --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/bench_fetch_${t}_$R.log 2>&1 || return $?
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write_${t}_$R -o run -- \
      python3 bench.py "$@" --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/bench_write_${t}_$R.log 2>&1 || return $?
}
for w in $ONLY; do
  case $w in
  e2e)
    timeout -k 10 600 python scripts/e2e.py --docs 200000 > gpurun_out/e2e_$R.log 2>&1 || exit $? ;;
  c4)
    prof c4 --workload kb50k || exit $?
    python3 profiles/pmc_traffic.py gpurun_out/traffic_c4_$R.json gpurun_out/prof_fetch_c4_$R gpurun_out/prof_write_c4_$R \
        docs_per_gpu=1000000 seed=20250905 > gpurun_out/traffic_c4_$R.log 2>&1 || exit $?
    timeout -k 10 600 python bench.py --workload kb50k --cpu-sample 16 > gpurun_out/bench_c4_$R.log 2>&1 || exit $? ;;
  dedup)
    prof dedup --workload dedup || exit $?
    python3 profiles/pmc_traffic.py gpurun_out/traffic_dedup_$R.json gpurun_out/prof_fetch_dedup_$R gpurun_out/prof_write_dedup_$R \
        rows_per_gpu=500000000 seed=20250905 > gpurun_out/traffic_dedup_$R.log 2>&1 || exit $?
    timeout -k 10 600 python bench.py --workload dedup --traffic-json gpurun_out/traffic_dedup_$R.json > gpurun_out/bench_dedup_$R.log 2>&1 || exit $? ;;
  esac
done
echo done > gpurun_out/configs_$R.done
