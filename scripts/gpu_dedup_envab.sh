#!/bin/bash
# A/B of environment knobs on config 5's bench line: bash scripts/gpu_dedup_envab.sh "VAR=a" "VAR=b" ... (one run each)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
i=0
for kv in "$@"; do
  env $kv timeout -k 10 300 python bench.py --workload dedup --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/dedup_env$i.log 2>&1 || exit $?
  echo "$kv $(grep '^{' gpurun_out/dedup_env$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernels_ms_avg'])")" >> gpurun_out/dedup_envab.txt
  i=$((i+1))
done
cat gpurun_out/dedup_envab.txt
