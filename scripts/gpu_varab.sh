#!/bin/bash
# A/B of library variants on the bench line (2 runs each, default first): bash scripts/gpu_varab.sh tag...
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for tag in default "$@"; do
  if [ "$tag" = default ]; then V=""; else V="--lib-variant $tag"; fi
  for rep in 1 2; do
    timeout -k 10 200 python bench.py --steps 30 --warmup 3 --cpu-sample 0 $V $BENCH_ARGS > gpurun_out/varab_${tag}_${rep}.log 2>&1 || exit $?
    echo "$tag rep$rep $(grep '^{' gpurun_out/varab_${tag}_${rep}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels_ms_avg']; print(d['ms_per_step'], d['value'], d['config']['hits_digest'], 'filter', k['filter'], 'probe', k['probe'], 'epi', k['epilogue'], 'tasks', k['tasks'])")" >> gpurun_out/varab.txt
  done
done
cat gpurun_out/varab.txt
