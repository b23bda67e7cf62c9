#!/bin/bash
# FETCH_SIZE / time of the filter kernel per library variant (config 2): bash scripts/gpu_fetch_ab.sh default t40 ...
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for tag in "$@"; do
  if [ "$tag" = default ]; then V=""; else V="--lib-variant $tag"; fi
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/fab_$tag -o run -- \
      python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 $V > gpurun_out/fab_$tag.log 2>&1 || exit $?
  python3 - "$tag" <<'PY' >> gpurun_out/fetch_ab.txt
import csv, glob, json, sys
tag = sys.argv[1]
v = [float(r['Counter_Value']) for fn in glob.glob(f'gpurun_out/fab_{tag}/**/*counter_collection.csv', recursive=True)
     for r in csv.DictReader(open(fn)) if 'kw_filter_kernel' in r['Kernel_Name'] and r['Counter_Name'] == 'FETCH_SIZE']
d = json.loads([l for l in open(f'gpurun_out/fab_{tag}.log') if l.startswith('{')][0])
print(tag, 'filter FETCH_SIZE KiB', round(sum(v) / len(v)), 'x2 GB', round(2 * sum(v) / len(v) * 1024 / 1e9, 3),
      'filter ms', d['roofline']['kernel_ms_avg'], 'step ms', d['ms_per_step'], d['config']['hits_digest'])
PY
done
cat gpurun_out/fetch_ab.txt
