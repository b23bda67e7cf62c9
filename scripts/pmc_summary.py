"""Summarise rocprofv3 counter CSVs under gpurun_out/<dir>/<tag>/ per kernel (sums over dispatches)."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
only = sys.argv[2] if len(sys.argv) > 2 else ''
for tagdir in sorted(glob.glob(os.path.join(root, '*'))):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for fn in glob.glob(os.path.join(tagdir, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(fn)):
            k = r['Kernel_Name'].split('(')[0].replace('kw::', '')
            acc[k][r['Counter_Name']] += float(r['Counter_Value'])
    for k, v in acc.items():
        if 'rocclr' in k or (only and only not in k):
            continue
        print(os.path.basename(tagdir), k, ' '.join(f"{a.replace('SQ_', '')}={b:.3g}" for a, b in sorted(v.items())))
