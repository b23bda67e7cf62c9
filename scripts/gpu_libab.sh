#!/bin/bash
# A/B of library variants (lib/libkwmatch_<tag>.so, build.build_kwmatch_variant; "default" = lib/libkwmatch.so) on
# the config-2 bench line, two runs each:  bash scripts/gpu_libab.sh default a4 a6 ...   (TESTS=1: -m gpu first)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 1200 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "pytest_rc=$rc" >> gpurun_out/gpu_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
for tag in "$@"; do
  if [ "$tag" = default ]; then V=""; else V="--lib-variant $tag"; fi
  for rep in 1 2; do
    timeout -k 10 240 python bench.py --steps 30 --warmup 3 --cpu-sample 0 $V $BENCH_ARGS > gpurun_out/libab_${tag}_${rep}.log 2>&1 || exit $?
    echo "$tag rep$rep $(grep '^{' gpurun_out/libab_${tag}_${rep}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels_ms_avg']; print(d['ms_per_step'], d['value'], d['config'].get('hits_digest'), 'cand', d['scan_stats']['candidates'], d['scan_stats']['candidates_stage2'], ' '.join(f'{a} {b:.3f}' for a, b in k.items()))")" >> gpurun_out/libab.txt
  done
done
cat gpurun_out/libab.txt
