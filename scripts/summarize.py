"""Print the bench JSON lines and test tails gpurun merged back into gpurun_out/ (dev helper)."""
import glob
import json
import os

for fn in sorted(glob.glob('gpurun_out/*.log')):
    lines = open(fn, errors='replace').read().splitlines()
    js = [x for x in lines if x.startswith('{')]
    if js:
        j = json.loads(js[-1])
        r = j.get('roofline') or {}
        print(os.path.basename(fn), j['value'], j['unit'], 'frac', r.get('frac'), r.get('kernels_ms_avg'))
        print('   ', j.get('scan_stats'))
        if j.get('cpu_baseline'):
            print('   cpu', j['cpu_baseline'])
    else:
        print(os.path.basename(fn), '|', ' / '.join(lines[-3:])[-400:])
