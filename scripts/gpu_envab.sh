#!/bin/bash
# A/B of environment knobs on the bench line: [BENCH_ARGS=...] bash scripts/gpu_envab.sh "VAR=a" "VAR=b" ... (each: 2 runs)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp KW_DEV=1
mkdir -p gpurun_out
i=0
for kv in "$@"; do
  for rep in 1 2; do
    env $kv timeout -k 10 200 python bench.py --steps 30 --warmup 3 --cpu-sample 0 $BENCH_ARGS > gpurun_out/envab_${i}_${rep}.log 2>&1 || exit $?
    echo "$kv rep$rep $(grep '^{' gpurun_out/envab_${i}_${rep}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels_ms_avg']; print(d['ms_per_step'], d['config']['hits_digest'], 'filter', k['filter'], 'probe', k['probe'], 'epi', k['epilogue'], 'tasks', k['tasks'])")" >> gpurun_out/envab.txt
  done
  i=$((i+1))
done
cat gpurun_out/envab.txt
