"""libsiamese_hip.so loads on a CPU-only host, exports every symbol of
include/siamese_hip.h, and validates models (host-only entry points)."""
import ctypes
import os
import re

import pytest

from _fixtures import AVERAGE_STACK, small_problem
from graphembedding_amd import _lib
from graphembedding_amd.build import build_hip

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope='module')
def L():
    build_hip()
    return _lib.lib()


def header_symbols():
    src = open(os.path.join(ROOT, 'include', 'siamese_hip.h')).read()
    return sorted(set(re.findall(r'^\s*(?:int32_t|int64_t)\s+(sg_\w+)\s*\(', src, re.M)))


def test_exports_every_header_symbol(L):
    syms = header_symbols()
    assert set(syms) == set(_lib.EXPORTED_SYMBOLS), syms
    for s in syms:
        assert hasattr(L, s), s
    assert L.sg_version() >= 10000


def test_record_layout(L):
    assert _lib.record_bytes(10) == 896          # 896 B per fp32 pair record
    assert _lib.record_bytes(30) == 4 * (2 * 900 + 60 + 4)
    assert _lib.record_bytes(0) == 0
    assert _lib.record_bytes(10, 'bf16') == 496   # §8(d) bf16 figure (492) + tag word
    assert L.sg_record_bytes_ex(10, 7) == 0       # unknown dtype


def _model(prob, **kw):
    f = prob.flags
    return _lib.make_model(prob.layers, prob.d_in, prob.n_max, 1 - f.dropout, f.final_act,
                           f.sim_kernel, f.yeta, kw.get('loss_mode', 'broadcast'),
                           kw.get('ntn_mode', 'reference'))


def test_validate_paths_and_param_counts(L):
    prob = small_problem()
    n, path = _lib.validate(_model(prob))
    assert path == 1 and n == prob.params.size            # default stack → fused kernel
    n2, path2 = _lib.validate(_model(prob, loss_mode='aligned', ntn_mode='intended'))
    assert path2 == 1 and n2 == n
    avg = small_problem(flags_overrides=AVERAGE_STACK)
    n3, path3 = _lib.validate(_model(avg))
    assert path3 == 1 and n3 == avg.params.size           # tuning.py stack → fused (AVG)
    att = small_problem(flags_overrides=dict(AVERAGE_STACK, layer_2='Attention:input_dim=16'))
    n4, path4 = _lib.validate(_model(att))
    assert path4 == 1 and n4 == att.params.size           # Attention pooling → fused (ATT)
    dot = small_problem(flags_overrides=dict(num_layers=5, layer_4='Dot'))
    n5, path5 = _lib.validate(_model(dot))
    assert path5 == 0 and n5 == dot.params.size           # generic kernel
    assert _lib.workspace_bytes(_model(prob), 490000) > 0


def test_validate_rejects_bad_models(L):
    prob = small_problem()
    m = _model(prob)
    m.layers[3].output_dim = 4          # Padding smaller than NTN input_dim
    with pytest.raises(_lib.SiameseHipError):
        _lib.validate(m)
    m = _model(prob)
    m.num_layers = 1
    with pytest.raises(_lib.SiameseHipError, match='SG_ERR_ARG'):
        _lib.validate(m)
    m = _model(prob)
    m.layers[0].sparse_inputs = 0       # the feature layer must be sparse (model_mse.py:14-19)
    with pytest.raises(_lib.SiameseHipError, match='SG_ERR_ARG'):
        _lib.validate(m)
    m = _model(prob)
    m.layers[2].kind = _lib.SG_GCN      # GCN after... fine shape-wise but Dense dims break it
    m.layers[2].input_dim = 16
    m.layers[2].output_dim = 1
    m.layers[2].sparse_inputs = 0
    n, path = _lib.validate(m)          # GCN-GCN-GCN-Pad-NTN is a valid reference stack
    assert path == 0


def test_store_source_checks(L):
    """sg_*_src argument checks (host side, before any launch): the store-sourced
    entries serve the fused paths only, and the store must match n_max."""
    import torch
    fake = torch.zeros(4, dtype=torch.int32)   # host tensors: only the pointers are read
    dev = (fake, fake, fake)
    dot = small_problem(flags_overrides=dict(num_layers=5, layer_4='Dot'))
    m0 = _model(dot)                                               # generic path 0
    assert _lib.validate(m0)[1] == 0
    with pytest.raises(_lib.SiameseHipError, match='SG_ERR_UNSUPPORTED'):
        _lib.pair_order_src(m0, _lib.pair_source(dev, 10), 4, fake, fake, stream=0)
    m1 = _model(small_problem())                                   # path 1, store n_max 12
    with pytest.raises(_lib.SiameseHipError, match='SG_ERR_ARG'):
        _lib.pair_order_src(m1, _lib.pair_source(dev, 12), 4, fake, fake, stream=0)
    c4 = small_problem(n_graphs=6, n_pairs=4, n_lo=20, n_hi=30, n_max=30)
    m2 = _lib.make_model(c4.layers, c4.d_in, 32, 0.9, c4.flags.final_act, c4.flags.sim_kernel,
                         c4.flags.yeta)
    assert _lib.validate(m2)[1] == 2
    with pytest.raises(_lib.SiameseHipError, match='SG_ERR_ARG'):   # store n_max != 32
        _lib.pair_order_src(m2, _lib.pair_source(dev, 30), 4, fake, fake, stream=0)
    with pytest.raises(_lib.SiameseHipError, match='SG_ERR_ARG'):   # no store
        _lib.forward_src(m2, _lib.SgPairSource(), 4, 0, fake, 1, fake, stream=0)
    m3 = _lib.make_model(c4.layers, c4.d_in, 32, 0.9, c4.flags.final_act, c4.flags.sim_kernel,
                         c4.flags.yeta, adj_dtype="bf16")
    with pytest.raises(_lib.SiameseHipError, match='SG_ERR_UNSUPPORTED'):   # bf16 Â
        _lib.pair_order_src(m3, _lib.pair_source(dev, 32), 4, fake, fake, stream=0)


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, 'LIB_PATH', str(tmp_path / 'nope.so'))
    monkeypatch.setattr(_lib, '_lib', None)
    with pytest.raises(_lib.SiameseHipError, match='no CPU fallback'):
        _lib.lib()


@pytest.mark.parametrize('macro', ['SG32_ABL_NOREC', 'SG32_ABL_NONTN', 'SG_WEB_ABL_NOH2'])
def test_timing_ablation_macro_alone_does_not_compile(macro):
    """A timing ablation (results invalid) compiles only with SG_TIMING_ABLATION_BUILD
    also set (sg_common.h #error), so a hand build cannot yield a silently wrong .so."""
    import subprocess
    hipcc = '/opt/rocm/bin/hipcc'
    if not os.path.isfile(hipcc):
        pytest.skip('no hipcc')
    hdr = os.path.join(ROOT, 'graphembedding_amd', 'csrc', 'sg_common.h')
    base = [hipcc, '--offload-arch=gfx950', '-std=c++17', '-E', '-x', 'hip', hdr, '-o',
            os.devnull]
    bad = subprocess.run(base + ['-D' + macro], capture_output=True, text=True)
    assert bad.returncode != 0 and 'timing ablation' in bad.stderr
    ok = subprocess.run(base + ['-D' + macro, '-DSG_TIMING_ABLATION_BUILD'],
                        capture_output=True, text=True)
    assert ok.returncode == 0, ok.stderr[-2000:]
