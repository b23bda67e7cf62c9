"""SQ counter table per kernel from the three rocprofv3 --pmc passes of scripts/gpu_sq.sh.

    python scripts/sq_table.py gpurun_out/r03_sq profiles/r03_sq.csv [algorithmic bytes per launch]

Counters are summed over a kernel's dispatches and divided by the dispatch
count (per launch).  Derived columns (per launch):
  valu_per_64B   SQ_INSTS_VALU wave-instructions per 64 article bytes (= VALU
                 instructions per byte position when a lane takes one position)
  lds_per_64B    SQ_INSTS_LDS per 64 article bytes
  bank_conflict  SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra LDS cycles / all LDS-array cycles)
  wait_any, wait_inst_any, active_inst_any   fractions of SQ_WAVE_CYCLES (disjoint; sum ~ 1)
  wait_inst_lds  SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES (LDS issue stall, a part of wait_inst_any)
  valu_active    SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES
"""
import collections
import csv
import glob
import os
import sys


def load(root):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for fn in glob.glob(os.path.join(root, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(fn)):
            k = r['Kernel_Name'].split('(')[0].replace('kw::', '').replace('dd::', '')
            if 'rocclr' in k:
                continue
            acc[k][r['Counter_Name']] += float(r['Counter_Value'])
            disp[(k, r['Counter_Name'])].add(r['Dispatch_Id'])
    out = {}
    for k, v in acc.items():
        out[k] = {c: x / max(1, len(disp[(k, c)])) for c, x in v.items()}
        out[k]['dispatches'] = max(len(disp[(k, c)]) for c in v)
    return out


def main():
    root, dst = sys.argv[1], sys.argv[2]
    nbytes = float(sys.argv[3]) if len(sys.argv) > 3 else 2285796280.0
    tab = load(root)
    counters = sorted({c for v in tab.values() for c in v if c.startswith('SQ_')})
    rows = []
    for k, v in sorted(tab.items(), key=lambda kv: -kv[1].get('SQ_WAVE_CYCLES', 0)):
        wc = v.get('SQ_WAVE_CYCLES', 0) or 1.0
        d = {'kernel': k, 'dispatches': v['dispatches']}
        d.update({c: f"{v.get(c, 0):.6g}" for c in counters})
        d['valu_per_64B'] = f"{v.get('SQ_INSTS_VALU', 0) * 64 / nbytes:.4g}"
        d['lds_per_64B'] = f"{v.get('SQ_INSTS_LDS', 0) * 64 / nbytes:.4g}"
        idx = v.get('SQ_LDS_IDX_ACTIVE', 0)
        d['bank_conflict'] = f"{v.get('SQ_LDS_BANK_CONFLICT', 0) / idx:.4g}" if idx else ''
        for a, b in (('wait_any', 'SQ_WAIT_ANY'), ('wait_inst_any', 'SQ_WAIT_INST_ANY'),
                     ('active_inst_any', 'SQ_ACTIVE_INST_ANY'), ('wait_inst_lds', 'SQ_WAIT_INST_LDS'),
                     ('valu_active', 'SQ_ACTIVE_INST_VALU')):
            d[a] = f"{v.get(b, 0) / wc:.4g}"
        rows.append(d)
    with open(dst, 'w', newline='') as fh:
        w = csv.DictWriter(fh, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(rows)
    for d in rows:
        print(d['kernel'], {k: d[k] for k in ('valu_per_64B', 'lds_per_64B', 'bank_conflict', 'wait_any',
                                             'wait_inst_any', 'active_inst_any', 'wait_inst_lds', 'valu_active')})


if __name__ == '__main__':
    main()
