"""Per-kernel average durations (ms) of rocprofv3 --stats CSVs: python scripts/kstats.py <dir>... (dev helper)."""
import csv
import glob
import os
import sys

for root in sys.argv[1:]:
    for fn in sorted(glob.glob(os.path.join(root, '**', '*kernel_stats.csv'), recursive=True)):
        print(fn)
        for r in csv.DictReader(open(fn)):
            if 'kw::' in r['Name'] or 'dd_' in r['Name']:
                print(f"   {r['Name'].split('(')[0].replace('kw::', ''):28s} {r['Calls']:>4} {float(r['AverageNs']) / 1e6:8.3f}")
