"""Build libsiamese_hip.so in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
from __future__ import annotations

import os
import subprocess
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(_HERE, 'csrc')
OUT = os.path.join(_HERE, 'lib', 'libsiamese_hip.so')
SOURCES = ['siamese_hip.hip', 'sg_generic.hip', 'sg_fast.hip', 'sg_fast_att.hip', 'sg_fast32.hip',
           'sg_sampler.hip', 'sg_web.hip']
HEADERS = ['sg_common.h', 'sg_plan.h', 'sg_mfma.h']
# MI355X only: the kernels use gfx950's 160 KB LDS (web_wgrad_kernel_b3 holds ≈66.6 KB),
# its MFMA shapes and wave64 layouts; there is no other target
ARCH = 'gfx950'


def _fingerprint(defines=(), extra=(), per_source=None) -> str:
    """The compiler options a build used (written next to the library)."""
    import json
    return json.dumps({'arch': ARCH, 'defines': list(defines), 'extra': list(extra),
                       'per_source': per_source or SOURCE_FLAGS}, sort_keys=True)


def _stale() -> bool:
    if not os.path.isfile(OUT):
        return True
    # a library built with other options (an A/B variant written over the default path)
    # is stale even when newer than every source
    try:
        with open(OUT + '.flags') as f:
            if f.read() != _fingerprint():
                return True
    except OSError:
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(os.path.dirname(_HERE), 'include', 'siamese_hip.h'))
    deps.append(os.path.abspath(__file__))
    return any(os.path.isfile(d) and os.path.getmtime(d) > t for d in deps)


# per-source compiler options (A/B-measured): the fused AIDS700nef kernel schedules for
# ILP (max-ilp: +1.2%; the capacity-32 kernel measured 0.8% slower with it), the
# capacity-32 kernel with the AMDGPU register-pressure trackers (+0.5%), the graph-store
# (C5) kernels for ILP (+1.0%: 4.006 vs 3.965 M pairs/s, profiles/r03_c5ab/)
# (the capacity-32 and graph-store kernels keep the packed split3 residuals, SG_SPLIT_PK=1:
# C4 152.5 / 152.3 against 151.6 / 151.9 M pairs/s without, C5 4.85 / 4.84 against 4.84 /
# 4.83; sg_fast runs 1.7% faster without them, profiles/r05_l)
SOURCE_FLAGS = {'sg_fast.hip': ['-mllvm', '-amdgpu-sched-strategy=max-ilp'],
                'sg_fast_att.hip': ['-mllvm', '-amdgpu-sched-strategy=max-ilp'],
                'sg_fast32.hip': ['-mllvm', '-amdgpu-use-amdgpu-trackers', '-DSG_SPLIT_PK=1'],
                # the graph-store kernels: the default scheduler measured 4.90 / 4.90
                # against 4.85 / 4.86 M pairs/s with max-ilp on C5 (profiles/r05_ee)
                'sg_web.hip': ['-DSG_SPLIT_PK=1']}


def build_hip(force: bool = False, verbose: bool = False, out: str = None, defines=()) -> str:
    """Build the library in-tree; `out`/`defines` build an A/B variant (e.g. -DSG_FAST_TIMING=1).
    Each source compiles to its own object (in parallel), then one link."""
    if out is None and not force and not _stale():
        return OUT
    dst = os.path.abspath(out) if out else OUT
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    hipcc = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
    base = [hipcc, '--offload-arch={}'.format(ARCH), '-O3', '-std=c++17', '-fPIC',
            # packed f32 VALU (SLP) blocks DPP fusion and stalls beside MFMA
            '-fno-slp-vectorize',
            '-Wall', '-Wno-unused-function', '-Wno-unused-variable']
    # A/B options (defines, SG_EXTRA_FLAGS, SG_FLAGS_<SRC>) apply to variants built to an
    # explicit `out` only: the production library at OUT is always the default build
    variant = out is not None
    extra = os.environ.get('SG_EXTRA_FLAGS', '').split() if variant else []
    defines = tuple(defines) if variant else ()
    # defines, SG_EXTRA_FLAGS (-D...) and SG_FLAGS_<SRC> can all carry timing-ablation or
    # A/B macros: no variant build may write the product library path
    if variant and os.path.abspath(dst) == os.path.abspath(OUT):
        raise RuntimeError('A/B variant builds (out=...) never go to the product library '
                           'path {}'.format(OUT))
    base += ['-D' + d for d in defines]
    base += extra
    per_source = {}
    import tempfile
    with tempfile.TemporaryDirectory(prefix='sg_build_') as tmp:
        procs, objs = [], []
        for src in SOURCES:
            obj = os.path.join(tmp, src + '.o')
            # A/B of one source's options: SG_FLAGS_SG_FAST="..." replaces sg_fast.hip's
            flags = SOURCE_FLAGS.get(src, [])
            env_key = 'SG_FLAGS_' + src.split('.')[0].upper()
            if variant and env_key in os.environ:
                flags = os.environ[env_key].split()
            if flags:
                per_source[src] = flags
            cmd = base + flags + ['-c', os.path.join(CSRC, src), '-o', obj]
            if verbose:
                print(' '.join(cmd))
            procs.append((src, subprocess.Popen(cmd, cwd=CSRC, stdout=subprocess.PIPE,
                                                stderr=subprocess.STDOUT, text=True)))
            objs.append(obj)
        failed = []
        for src, pr in procs:
            log = pr.communicate()[0]
            if pr.returncode != 0:
                failed.append(src)
                sys.stderr.write(log)
        if failed:
            raise RuntimeError('hipcc failed building libsiamese_hip.so: {}'.format(failed))
        link = [hipcc, '--offload-arch={}'.format(ARCH), '-fPIC', '-shared', '-o',
                dst + '.tmp'] + objs
        if verbose:
            print(' '.join(link))
        r = subprocess.run(link, cwd=CSRC, capture_output=True, text=True)
        if r.returncode != 0:
            sys.stderr.write(r.stdout + r.stderr)
            raise RuntimeError('hipcc failed linking libsiamese_hip.so')
    os.replace(dst + '.tmp', dst)
    with open(dst + '.flags', 'w') as f:
        f.write(_fingerprint(defines, extra, per_source))
    return dst


if __name__ == '__main__':
    # python -m graphembedding_amd.build [--force] [--out PATH] [-DNAME=VAL ...]
    a = sys.argv[1:]
    out = a[a.index('--out') + 1] if '--out' in a else None
    defs = [x[2:] for x in a if x.startswith('-D')]
    print(build_hip(force='--force' in a, verbose=True, out=out, defines=defs))
