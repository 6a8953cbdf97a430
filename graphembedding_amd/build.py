"""Build libsiamese_hip.so in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
from __future__ import annotations

import os
import subprocess
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(_HERE, 'csrc')
OUT = os.path.join(_HERE, 'lib', 'libsiamese_hip.so')
SOURCES = ['siamese_hip.hip', 'sg_generic.hip', 'sg_fast.hip']
HEADERS = ['sg_common.h', 'sg_plan.h', 'sg_fast_kernel.h']
ARCH = os.environ.get('SG_OFFLOAD_ARCH', 'gfx950')


def _stale() -> bool:
    if not os.path.isfile(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(os.path.dirname(_HERE), 'include', 'siamese_hip.h'))
    return any(os.path.isfile(d) and os.path.getmtime(d) > t for d in deps)


def build_hip(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    hipcc = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
    cmd = [hipcc, '--offload-arch={}'.format(ARCH), '-O3', '-std=c++17', '-fPIC', '-shared',
           '-Wall', '-Wno-unused-function', '-Wno-unused-variable', '-o', OUT + '.tmp']
    cmd += [os.path.join(CSRC, s) for s in SOURCES]
    if verbose:
        print(' '.join(cmd))
    r = subprocess.run(cmd, cwd=CSRC, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError('hipcc failed building libsiamese_hip.so')
    os.replace(OUT + '.tmp', OUT)
    return OUT


if __name__ == '__main__':
    print(build_hip(force='--force' in sys.argv, verbose=True))
