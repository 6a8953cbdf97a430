"""Dump the device assembly of every library source with the product build's options
(graphembedding_amd/build.py), to compare two trees' code objects: a refactor that must not
change the kernels (e.g. pruning dead compile-time variants) leaves the dumps identical.
Usage: python scripts/isa_dump.py OUTDIR"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from graphembedding_amd import build as B  # noqa: E402

out = os.path.abspath(sys.argv[1])
os.makedirs(out, exist_ok=True)
base = ['/opt/rocm/bin/hipcc', '--offload-arch=' + B.ARCH, '-O3', '-std=c++17', '-fPIC',
        '-fno-slp-vectorize', '--cuda-device-only', '-S', '-w']
procs = []
for src in B.SOURCES:
    dst = os.path.join(out, src + '.s')
    cmd = base + B.SOURCE_FLAGS.get(src, []) + [os.path.join(B.CSRC, src), '-o', dst]
    procs.append((src, dst, subprocess.Popen(cmd, cwd=B.CSRC)))
bad = 0
for src, dst, p in procs:
    if p.wait() != 0:
        print('failed', src)
        bad = 1
        continue
    # drop comments, debug/metadata lines that name files, and the ident string
    keep = []
    for line in open(dst):
        s = line.split(';')[0].rstrip() if not line.lstrip().startswith('.') else line.rstrip()
        if not s or s.lstrip().startswith(('.file', '.ident', '.loc', '.amdgpu_metadata')):
            continue
        keep.append(s)
    with open(dst + '.norm', 'w') as f:
        f.write('\n'.join(keep) + '\n')
    print(src, len(keep), 'lines')
sys.exit(bad)
