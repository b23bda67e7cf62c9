"""Print ms_per_step of each gpurun_out/sweep_<i>.log written by gpu_envsweep.sh (dev aid)."""
import glob
import json
import re

for p in sorted(glob.glob('gpurun_out/sweep_*.log'), key=lambda s: int(re.findall(r'\d+', s)[-1])):
    lines = open(p).read().splitlines()
    js = [x for x in lines if x.startswith('{')]
    print(p, lines[-1] if lines else '', json.loads(js[-1])['ms_per_step'] if js else lines[-3:])
