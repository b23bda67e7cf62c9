"""Per-kernel SQ counters and HBM bytes of scripts/gpu_sq_dedup.sh's passes (gpurun_out/sqdd/{a,b,c,d})."""
import sys

sys.path.insert(0, 'scripts')
from sq_table import load  # noqa: E402

root = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/sqdd'
p = [load(f'{root}/{x}') for x in 'abcd']
for k in sorted(p[0], key=lambda k: -p[0][k].get('SQ_WAVE_CYCLES', 0)):
    x = {}
    for q in p:
        x.update(q.get(k, {}))
    wc = x.get('SQ_WAVE_CYCLES', 1) or 1
    print(f"{k:24s} waves {x.get('SQ_WAVES', 0):8.0f} valu {x.get('SQ_INSTS_VALU', 0):9.3g} salu {x.get('SQ_INSTS_SALU', 0):9.3g} "
          f"lds {x.get('SQ_INSTS_LDS', 0):8.3g} vmem_rd {x.get('SQ_INSTS_VMEM_RD', 0):8.3g} vmem_wr {x.get('SQ_INSTS_VMEM_WR', 0):8.3g}")
    print(f"{'':24s} wait_any {x.get('SQ_WAIT_ANY', 0) / wc:.2f} wait_inst_any {x.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} "
          f"active_any {x.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} valu_active {x.get('SQ_ACTIVE_INST_VALU', 0) / wc:.2f} "
          f"fetch {x.get('FETCH_SIZE', 0) / 1e6:.3g} GB write {x.get('WRITE_SIZE', 0) / 1e6:.3g} GB")
