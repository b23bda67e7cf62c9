#!/bin/bash
# bench lines of "ENV=VAL:variant" pairs (variant 'default' = the in-tree library):
#   bash scripts/gpu_varenv.sh KW_SIDE_PRIO=1:pkw6 KW_X=1:default ...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -f gpurun_out/varenv.txt
i=0
for pair in "$@"; do
  kv=${pair%%:*}; v=${pair##*:}
  if [ "$v" = default ]; then a=""; else a="--lib-variant $v"; fi
  env $kv timeout -k 10 200 python bench.py --steps 30 --warmup 3 --cpu-sample 0 $a > gpurun_out/varenv_$i.log 2>&1 || exit $?
  echo "$pair $(grep '^{' gpurun_out/varenv_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels_ms_avg']; print(d['ms_per_step'], d['config']['hits_digest'], 'filter', k['filter'], 'probe', k['probe'], 'epi', k['epilogue'], 'tasks', k['tasks'])")" >> gpurun_out/varenv.txt
  i=$((i+1))
done
cat gpurun_out/varenv.txt
