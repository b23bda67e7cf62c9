"""One scan's kernel timeline from a rocprofv3 kernel trace (the second-to-last filter launch): start / end in us
from the filter's start.   python scripts/timeline.py <trace dir> (dev helper)"""
import csv
import glob
import os
import sys

fn = glob.glob(os.path.join(sys.argv[1], '**', '*kernel_trace.csv'), recursive=True)[0]
rows = sorted(csv.DictReader(open(fn)), key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'kw_filter_kernel' in r['Kernel_Name']]
i0, i1 = idx[-2], idx[-1]
t0 = int(rows[i0]['Start_Timestamp'])
for r in rows[i0:i1]:
    n = r['Kernel_Name'].split('(')[0].replace('kw::', '')[:28]
    s = (int(r['Start_Timestamp']) - t0) / 1000
    e = (int(r['End_Timestamp']) - t0) / 1000
    print(f"{n:30s} {s:9.1f} {e:9.1f} {e - s:8.1f}  q{r['Queue_Id']}")
