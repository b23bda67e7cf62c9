#!/bin/bash
# bench lines of the default library and of timing variants: bash scripts/gpu_varab2.sh tag1 tag2 ...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -f gpurun_out/varab.txt
for v in default "$@"; do
  if [ "$v" = default ]; then a=""; else a="--lib-variant $v"; fi
  timeout -k 10 200 python bench.py --steps 30 --warmup 3 --cpu-sample 0 $a > gpurun_out/varab_$v.log 2>&1 || exit $?
  echo "$v $(grep '^{' gpurun_out/varab_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels_ms_avg']; print(d['ms_per_step'], d['config']['hits_digest'], 'filter', k['filter'], 'probe', k['probe'], 'epi', k['epilogue'], 'tasks', k['tasks'])")" >> gpurun_out/varab.txt
done
cat gpurun_out/varab.txt
