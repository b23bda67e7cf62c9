#!/bin/bash
# A/B of (library variant, bench arguments) pairs on the config-2 bench line, REPS runs each (default 2):
#   bash scripts/gpu_ab.sh "default|" "h8|--inflight 2" ...      (variant "default" = lib/libkwmatch.so)
# One summary line per run in gpurun_out/ab.txt.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
REPS=${REPS:-2}
i=0
for spec in "$@"; do
  tag=${spec%%|*}; args=${spec#*|}
  if [ "$tag" = default ]; then V=""; else V="--lib-variant $tag"; fi
  for rep in $(seq 1 $REPS); do
    i=$((i+1))
    timeout -k 10 240 python bench.py --steps 30 --warmup 3 --cpu-sample 0 $V $args > gpurun_out/ab_${i}.log 2>&1 || exit $?
    echo "$tag [$args] rep$rep $(grep '^{' gpurun_out/ab_${i}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels_ms_avg']; print(d['ms_per_step'], d['value'], d['config'].get('hits_digest'), 'cand', d['scan_stats']['candidates'], d['scan_stats']['candidates_stage2'], ' '.join(f'{a} {b:.3f}' for a, b in k.items()))")" >> gpurun_out/ab.txt
  done
done
cat gpurun_out/ab.txt
