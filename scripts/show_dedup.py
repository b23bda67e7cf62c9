"""Print the dedup bench lines of gpurun_out/dedup_*.log."""
import glob
import json

for f in sorted(glob.glob('gpurun_out/dedup_*.log')):
    try:
        j = json.loads(open(f).read().strip().splitlines()[-1])
        print(f, j['value'], j['ms_per_step'], j['roofline']['kernels_ms_avg'], j['config']['kept'], j['config']['duplicates'])
    except Exception as e:   # noqa: BLE001 (a failed run's log)
        print(f, 'no line:', e)
