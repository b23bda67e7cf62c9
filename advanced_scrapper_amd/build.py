"""Build the in-tree native libraries (no JIT cache, nothing pip-installed).

* ``lib/libkwmatch.so`` — HIP kernels + C-ABI, ``hipcc --offload-arch=gfx950``
* ``lib/libsynth.so``   — host C corpus generator (bench/test data)

Run ``python -m advanced_scrapper_amd.build``.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
LIB = os.path.join(HERE, 'lib')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = os.environ.get('KW_OFFLOAD_ARCH', 'gfx950')


def _run(cmd):
    print(' '.join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def _stale(target, sources):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def build_kwmatch(force: bool = False) -> str:
    os.makedirs(LIB, exist_ok=True)
    out = os.path.join(LIB, 'libkwmatch.so')
    srcs = _kw_sources()
    if force or _stale(out, srcs):
        units = [s for s in srcs if s.endswith('.hip')]
        _run([HIPCC, f'--offload-arch={ARCH}', '-O3', '-std=c++17', '-shared', '-fPIC', '-Wall',
              '-o', out] + units + ['-ldl'])
    return out


def _kw_sources():
    srcs = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(('.hip', '.hpp')))
    srcs.append(os.path.join(HERE, '..', 'include', 'kwmatch.h'))
    return srcs


def build_kwmatch_variant(tag: str, defines, force: bool = False) -> str:
    """Tuning variant ``lib/libkwmatch_<tag>.so`` built with extra -D defines of the documented tuning knobs
    (waves per SIMD, grids, pool sizes; entries starting with '-' are passed as compiler flags).  Only
    ``bench.py --lib-variant`` loads one (``_native`` refuses ``KW_LIB`` otherwise); results are the same."""
    os.makedirs(LIB, exist_ok=True)
    out = os.path.join(LIB, f'libkwmatch_{tag}.so')
    srcs = _kw_sources()
    if force or _stale(out, srcs):
        units = [s for s in srcs if s.endswith('.hip')]
        _run([HIPCC, f'--offload-arch={ARCH}', '-O3', '-std=c++17', '-shared', '-fPIC'] +
             [d if d.startswith('-') else f'-D{d}' for d in defines] + ['-o', out] + units + ['-ldl'])
    return out


def build_synth(force: bool = False) -> str:
    os.makedirs(LIB, exist_ok=True)
    out = os.path.join(LIB, 'libsynth.so')
    src = os.path.join(CSRC, 'synth.c')
    if force or _stale(out, [src]):
        _run(['gcc', '-O2', '-fopenmp', '-fPIC', '-shared', '-Wall', '-o', out, src])
    return out


def build_kwrows(force: bool = False) -> str:
    """``lib/libkwrows.so``: host C assembly of the output rows' JSON cells (csrc/kwrows.c)."""
    os.makedirs(LIB, exist_ok=True)
    out = os.path.join(LIB, 'libkwrows.so')
    src = os.path.join(CSRC, 'kwrows.c')
    if force or _stale(out, [src]):
        _run(['gcc', '-O2', '-fopenmp', '-fPIC', '-shared', '-Wall', '-o', out, src])
    return out


def build_kwcsv(force: bool = False) -> str:
    """``lib/libkwcsv.so``: host C CSV tokenizer of the article ingest and the output sort (csrc/kwcsv.c)."""
    os.makedirs(LIB, exist_ok=True)
    out = os.path.join(LIB, 'libkwcsv.so')
    src = os.path.join(CSRC, 'kwcsv.c')
    if force or _stale(out, [src]):
        _run(['gcc', '-O2', '-fopenmp', '-fPIC', '-shared', '-Wall', '-o', out, src])
    return out


def build_all(force: bool = False):
    return build_kwmatch(force), build_synth(force), build_kwrows(force), build_kwcsv(force)


if __name__ == '__main__':
    build_all(force='--force' in sys.argv)
