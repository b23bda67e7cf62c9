#!/bin/bash
# A/B of library variants on the config-5 (dedup) bench line, one run each: bash scripts/gpu_dedup_libab.sh default p82 ...
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for tag in "$@"; do
  if [ "$tag" = default ]; then V=""; else V="--lib-variant $tag"; fi
  timeout -k 10 300 python bench.py --workload dedup --steps 5 --warmup 1 --cpu-sample 0 $V > gpurun_out/ddab_${tag}.log 2>&1 || exit $?
  echo "$tag $(grep '^{' gpurun_out/ddab_${tag}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels_ms_avg']; print(d['ms_per_step'], d['value'], ' '.join(f'{a} {b:.3f}' for a, b in k.items()))")" >> gpurun_out/ddab.txt
done
cat gpurun_out/ddab.txt
