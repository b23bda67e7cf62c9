#!/bin/bash
# Config-4 big-document route check: the config-4 whole-corpus test (default and KW_TEST_BIGQ=0), the config-2/4
# bench lines (2 runs each) and config 4 at 10M (deferred_docs should be 0).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_c4.py -m gpu -k whole_corpus > gpurun_out/bigq_test.log 2>&1 || exit $?
REPS=2 bash scripts/gpu_ab.sh "default|" "default|--workload kb50k" || exit $?
timeout -k 10 500 python bench.py --workload kb50k --total-docs 10000000 --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/c4_10m.log 2>&1 || exit $?
grep '^{' gpurun_out/c4_10m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('10M', d['value'], d['ms_per_step'], d['config']['hits_digest'], {k: d['scan_stats'][k] for k in ('deferred_docs','deferred_item_caps','big_docs','resolved_docs')})"
