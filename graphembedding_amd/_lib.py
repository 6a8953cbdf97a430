"""ctypes binding of libsiamese_hip.so (C-ABI declared in include/siamese_hip.h).

The product path has no CPU fallback: if the HIP library is missing or cannot
be loaded this module raises, loudly, on first use.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
# SG_LIB overrides the in-tree library (A/B builds of kernel variants)
LIB_PATH = os.environ.get('SG_LIB') or os.path.join(_HERE, 'lib', 'libsiamese_hip.so')
if not os.path.isabs(LIB_PATH) and not os.path.exists(LIB_PATH):
    LIB_PATH = os.path.join(os.path.dirname(_HERE), LIB_PATH)   # relative to the repo root

SG_OK, SG_ERR_ARG, SG_ERR_UNSUPPORTED, SG_ERR_HIP, SG_ERR_SHAPE = 0, 1, 2, 3, 4
_ERR_NAMES = {1: 'SG_ERR_ARG', 2: 'SG_ERR_UNSUPPORTED', 3: 'SG_ERR_HIP', 4: 'SG_ERR_SHAPE'}

SG_GCN, SG_DENSE, SG_PADDING, SG_AVERAGE, SG_ATTENTION, SG_NTN, SG_DOT = 1, 2, 3, 4, 5, 6, 7
KIND_CODES = {'GraphConvolution': SG_GCN, 'Dense': SG_DENSE, 'Padding': SG_PADDING,
              'Average': SG_AVERAGE, 'Attention': SG_ATTENTION, 'NTN': SG_NTN, 'Dot': SG_DOT}
ACT_CODES = {'identity': 0, 'relu': 1, 'sigmoid': 2, 'tanh': 3}
FINAL_GAUSSIAN, FINAL_IDENTITY, FINAL_RELU, FINAL_SIGMOID, FINAL_TANH = 0, 1, 2, 3, 4
LOSS_BROADCAST, LOSS_ALIGNED = 0, 1
NTN_REFERENCE, NTN_INTENDED = 0, 1
SG_MAX_LAYERS = 8


class SgLayer(ctypes.Structure):
    _fields_ = [('kind', ctypes.c_int32), ('input_dim', ctypes.c_int32),
                ('output_dim', ctypes.c_int32), ('act', ctypes.c_int32),
                ('bias', ctypes.c_int32), ('dropout', ctypes.c_int32),
                ('sparse_inputs', ctypes.c_int32), ('padding_value', ctypes.c_float)]


class SgModel(ctypes.Structure):
    _fields_ = [('num_layers', ctypes.c_int32), ('d_in', ctypes.c_int32),
                ('n_max', ctypes.c_int32), ('final_act', ctypes.c_int32),
                ('loss_mode', ctypes.c_int32), ('ntn_mode', ctypes.c_int32),
                ('keep_prob', ctypes.c_float), ('yeta', ctypes.c_float),
                ('layers', SgLayer * SG_MAX_LAYERS), ('adj_dtype', ctypes.c_int32)]


class SgCsrStore(ctypes.Structure):
    """sg_csr_store_t: host struct of device pointers (graph-store path, config C5)."""
    _fields_ = [('n_graphs', ctypes.c_int32), ('n_max', ctypes.c_int32),
                ('node_off', ctypes.c_void_p), ('types', ctypes.c_void_p),
                ('row_ptr', ctypes.c_void_p), ('col', ctypes.c_void_p), ('val', ctypes.c_void_p),
                ('max_nnz', ctypes.c_int32)]


class SgPairSource(ctypes.Structure):
    """sg_pair_source_t: host struct of device pointers (store-sourced pairs, library 1.6)."""
    _fields_ = [('adj', ctypes.c_void_p), ('types', ctypes.c_void_p), ('n', ctypes.c_void_p),
                ('n_graphs', ctypes.c_int32), ('n_max', ctypes.c_int32),
                ('pair_idx', ctypes.c_void_p), ('grid_base', ctypes.c_int64),
                ('labels', ctypes.c_void_p), ('status', ctypes.c_void_p)]


class SgFeed(ctypes.Structure):
    """sg_feed_t: host struct of device pointers (one step's get_feed_dict)."""
    _fields_ = [('kind', ctypes.c_int32), ('state', ctypes.c_void_p), ('sigma', ctypes.c_void_p),
                ('n', ctypes.c_int32), ('dens_order', ctypes.c_void_p), ('bins', ctypes.c_void_p),
                ('item_table', ctypes.c_void_p), ('n_bins', ctypes.c_int32),
                ('bin_size', ctypes.c_int32), ('batch', ctypes.c_int32), ('compat', ctypes.c_int32),
                ('label_matrix', ctypes.c_void_p), ('label_n', ctypes.c_int32),
                ('store_adj', ctypes.c_void_p), ('store_types', ctypes.c_void_p),
                ('store_n', ctypes.c_void_p), ('n_graphs', ctypes.c_int32),
                ('n_max', ctypes.c_int32), ('adj_dtype', ctypes.c_int32)]


class SgAdamArgs(ctypes.Structure):
    """sg_adam_args_t: the Adam state and hyper-parameters of sg_train_step."""
    _fields_ = [('m', ctypes.c_void_p), ('v', ctypes.c_void_p), ('lr', ctypes.c_float),
                ('beta1', ctypes.c_float), ('beta2', ctypes.c_float), ('eps', ctypes.c_float),
                ('weight_decay', ctypes.c_float), ('beta_powers', ctypes.c_void_p),
                ('reg_loss_out', ctypes.c_void_p)]


class SiameseHipError(RuntimeError):
    pass


_lib = None


def lib():
    """Load the HIP library (raises SiameseHipError if it is missing)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.isfile(LIB_PATH):
        raise SiameseHipError(
            'libsiamese_hip.so not found at {} — run `python -c "import __graft_entry__ as g; '
            'g.build()"` (hipcc --offload-arch=gfx950). There is no CPU fallback.'.format(LIB_PATH))
    try:   # bring up torch's HIP runtime before the library's first HIP call
        import torch
        torch.cuda.is_available()
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    c_i32, c_i64, c_u64, c_f = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_float
    vp = ctypes.c_void_p
    pm = ctypes.POINTER(SgModel)
    L.sg_version.restype = c_i32
    L.sg_record_bytes.argtypes = [c_i32]
    L.sg_record_bytes.restype = c_i64
    L.sg_record_bytes_ex.argtypes = [c_i32, c_i32]
    L.sg_record_bytes_ex.restype = c_i64
    L.sg_model_validate.argtypes = [pm, ctypes.POINTER(c_i64), ctypes.POINTER(c_i32)]
    L.sg_model_validate.restype = c_i32
    L.sg_workspace_bytes.argtypes = [pm, c_i64]
    L.sg_workspace_bytes.restype = c_i64
    L.sg_pack_pairs.argtypes = [vp, vp, vp, c_i32, c_i32, vp, vp, c_i64, vp, vp, vp]
    L.sg_pack_pairs.restype = c_i32
    L.sg_pack_pairs_ex.argtypes = [vp, vp, vp, c_i32, c_i32, c_i32, vp, vp, c_i64, vp, vp, vp]
    L.sg_pack_pairs_ex.restype = c_i32
    L.sg_label_stats.argtypes = [vp, c_i64, c_i32, vp, vp, vp]
    L.sg_label_stats.restype = c_i32
    L.sg_label_stats_ex.argtypes = [vp, c_i64, c_i32, c_i32, vp, vp, vp]
    L.sg_label_stats_ex.restype = c_i32
    L.sg_forward.argtypes = [pm, vp, c_i64, c_i64, vp, c_u64, vp, vp, vp]
    L.sg_forward.restype = c_i32
    L.sg_fwd_bwd.argtypes = [pm, vp, c_i64, c_i64, c_i64, vp, c_u64, vp, c_i32, vp, vp, vp, vp, vp]
    L.sg_fwd_bwd.restype = c_i32
    L.sg_forward_ex.argtypes = [pm, vp, vp, c_i64, c_i64, vp, c_u64, vp, vp, vp]
    L.sg_forward_ex.restype = c_i32
    L.sg_fwd_bwd_ex.argtypes = [pm, vp, vp, c_i64, c_i64, c_i64, vp, c_u64, vp, c_i32, vp, vp,
                                vp, vp, vp]
    L.sg_fwd_bwd_ex.restype = c_i32
    L.sg_pair_order_workspace_bytes.argtypes = [pm, c_i64]
    L.sg_pair_order_workspace_bytes.restype = c_i64
    L.sg_pair_order.argtypes = [pm, vp, c_i64, vp, vp, vp]
    L.sg_pair_order.restype = c_i32
    L.sg_pair_order_cls.argtypes = [pm, vp, c_i64, vp, vp, vp, vp]
    L.sg_pair_order_cls.restype = c_i32
    L.sg_forward_cls.argtypes = [pm, vp, vp, vp, c_i64, c_i64, vp, c_u64, vp, vp, vp]
    L.sg_forward_cls.restype = c_i32
    L.sg_fwd_bwd_cls.argtypes = [pm, vp, vp, vp, c_i64, c_i64, c_i64, vp, c_u64, vp, c_i32, vp,
                                 vp, vp, vp, vp]
    L.sg_fwd_bwd_cls.restype = c_i32
    L.sg_train_step.argtypes = [pm, vp, vp, vp, c_i64, c_i64, c_i64, vp, c_u64, vp, c_i32, vp,
                                vp, vp, vp, ctypes.POINTER(SgAdamArgs), vp]
    L.sg_train_step.restype = c_i32
    L.sg_train_step_dseed.argtypes = [pm, vp, vp, c_i64, c_i64, c_i64, vp, vp, vp, c_i32, vp,
                                      vp, vp, vp, ctypes.POINTER(SgAdamArgs), vp]
    L.sg_train_step_dseed.restype = c_i32
    L.sg_sampler_random.argtypes = [vp, vp, c_i32, c_i64, vp, vp]
    L.sg_sampler_random.restype = c_i32
    L.sg_sampler_density.argtypes = [vp, vp, vp, c_i32, c_i32, vp, c_i64, vp, vp]
    L.sg_sampler_density.restype = c_i32
    L.sg_adam_tf.argtypes = [vp, vp, vp, vp, c_i64, c_f, c_f, c_f, c_f, c_f, vp, vp, vp]
    L.sg_adam_tf.restype = c_i32
    L.sg_adam_workspace_bytes.argtypes = [c_i64]
    L.sg_adam_workspace_bytes.restype = c_i64
    L.sg_adam_tf_ex.argtypes = [vp, vp, vp, vp, c_i64, c_f, c_f, c_f, c_f, c_f, vp, vp, vp, vp]
    L.sg_adam_tf_ex.restype = c_i32
    L.sg_fwd_bwd_dseed.argtypes = [pm, vp, vp, c_i64, c_i64, c_i64, vp, vp, vp, c_i32, vp, vp,
                                   vp, vp, vp]
    L.sg_fwd_bwd_dseed.restype = c_i32
    L.sg_seed_advance.argtypes = [vp, c_u64, vp]
    L.sg_seed_advance.restype = c_i32
    L.sg_feed_step.argtypes = [ctypes.POINTER(SgFeed), vp, vp, vp, vp, vp, vp]
    L.sg_feed_step.restype = c_i32
    pc = ctypes.POINTER(SgCsrStore)
    L.sg_web_workspace_bytes.argtypes = [pm, c_i64]
    L.sg_web_workspace_bytes.restype = c_i64
    L.sg_web_workspace_bytes_ex.argtypes = [pm, c_i64, c_i64]
    L.sg_web_workspace_bytes_ex.restype = c_i64
    L.sg_web_release.argtypes = []
    L.sg_web_release.restype = ctypes.c_int32
    L.sg_web_forward.argtypes = [pm, pc, vp, c_i64, c_i64, vp, c_u64, vp, vp, c_i64, vp]
    L.sg_web_forward.restype = c_i32
    L.sg_web_fwd_bwd.argtypes = [pm, pc, vp, vp, c_i64, c_i64, c_i64, vp, c_u64, vp, c_i32, vp,
                                 vp, vp, vp, c_i64, vp]
    L.sg_web_fwd_bwd.restype = c_i32
    ps = ctypes.POINTER(SgPairSource)
    L.sg_pair_order_src.argtypes = [pm, ps, c_i64, vp, vp, vp]
    L.sg_pair_order_src.restype = c_i32
    L.sg_forward_src.argtypes = [pm, ps, vp, c_i64, c_i64, vp, c_u64, vp, vp, vp]
    L.sg_forward_src.restype = c_i32
    L.sg_fwd_bwd_src.argtypes = [pm, ps, vp, c_i64, c_i64, c_i64, vp, c_u64, vp, c_i32, vp, vp,
                                 vp, vp, vp]
    L.sg_fwd_bwd_src.restype = c_i32
    _lib = L
    return L


PATH_NAMES = {0: 'generic', 1: 'fused', 2: 'fused32', 3: 'web'}
PATH_WEB = 3

EXPORTED_SYMBOLS = ('sg_version', 'sg_record_bytes', 'sg_record_bytes_ex', 'sg_model_validate',
                    'sg_workspace_bytes', 'sg_pack_pairs', 'sg_pack_pairs_ex', 'sg_label_stats',
                    'sg_label_stats_ex', 'sg_forward', 'sg_fwd_bwd', 'sg_adam_tf',
                    'sg_forward_ex', 'sg_fwd_bwd_ex', 'sg_pair_order',
                    'sg_pair_order_workspace_bytes', 'sg_sampler_random', 'sg_sampler_density',
                    'sg_adam_workspace_bytes', 'sg_adam_tf_ex', 'sg_web_workspace_bytes',
                    'sg_web_workspace_bytes_ex', 'sg_web_release',
                    'sg_web_forward', 'sg_web_fwd_bwd', 'sg_fwd_bwd_dseed', 'sg_seed_advance',
                    'sg_feed_step', 'sg_pair_order_src', 'sg_forward_src', 'sg_fwd_bwd_src',
                    'sg_pair_order_cls', 'sg_forward_cls', 'sg_fwd_bwd_cls', 'sg_train_step',
                    'sg_train_step_dseed')

# class_start entries of sg_pair_order_cls (include/siamese_hip.h SG_FAST_CLASSES_P1)
FAST_CLASSES_P1 = 5

# sg_dtype: storage type of Â in the pair records
DTYPES = {'f32': 0, 'bf16': 1}


def dtype_code(dtype) -> int:
    if isinstance(dtype, int):
        return dtype
    if dtype not in DTYPES:
        raise RuntimeError('Unknown record dtype {}'.format(dtype))
    return DTYPES[dtype]


def check(rc: int, what: str) -> None:
    if rc != SG_OK:
        raise SiameseHipError('{} failed: {} ({})'.format(what, _ERR_NAMES.get(rc, rc), rc))


def final_act_code(final_act: str, sim_kernel: str) -> int:
    if final_act == 'sim_kernel':
        if sim_kernel == 'gaussian':
            return FINAL_GAUSSIAN
        if sim_kernel == 'identity':
            return FINAL_IDENTITY
        raise RuntimeError('Unknown sim kernel {}'.format(sim_kernel))
    codes = {'identity': FINAL_IDENTITY, 'relu': FINAL_RELU, 'sigmoid': FINAL_SIGMOID,
             'tanh': FINAL_TANH}
    if final_act not in codes:
        raise RuntimeError('Unknown activation function {}'.format(final_act))
    return codes[final_act]


def make_model(layers: List[dict], d_in: int, n_max: int, keep_prob: float, final_act: str,
               sim_kernel: str, yeta: float, loss_mode: str = 'broadcast',
               ntn_mode: str = 'reference', adj_dtype='f32') -> SgModel:
    """Layer dicts (graphembedding_amd.layers_factory format) → sg_model_t."""
    if len(layers) > SG_MAX_LAYERS:
        raise RuntimeError('at most {} layers supported'.format(SG_MAX_LAYERS))
    m = SgModel()
    m.num_layers = len(layers)
    m.d_in = int(d_in)
    m.n_max = int(n_max)
    m.final_act = final_act_code(final_act, sim_kernel)
    m.loss_mode = {'broadcast': LOSS_BROADCAST, 'aligned': LOSS_ALIGNED}[loss_mode]
    m.ntn_mode = {'reference': NTN_REFERENCE, 'intended': NTN_INTENDED}[ntn_mode]
    m.adj_dtype = dtype_code(adj_dtype)
    m.keep_prob = float(keep_prob)
    m.yeta = float(yeta if yeta is not None else 0.0)
    for i, L in enumerate(layers):
        s = m.layers[i]
        s.kind = KIND_CODES[L['kind']]
        k = L['kind']
        if k == 'GraphConvolution':
            s.input_dim = int(L.get('input_dim') or 0)
            s.output_dim = int(L['output_dim'])
            s.act = ACT_CODES[L['act']]
            s.sparse_inputs = int(bool(L['sparse_inputs']))
        elif k == 'Dense':
            s.input_dim = int(L['input_dim'])
            s.output_dim = int(L['output_dim'])
            s.act = ACT_CODES[L['act']]
        elif k == 'Padding':
            s.output_dim = int(L['max_in_dims'])
            s.padding_value = float(L.get('padding_value', 0))
        elif k == 'Attention':
            s.input_dim = int(L['input_dim'])
        elif k == 'NTN':
            s.input_dim = int(L['input_dim'])
            s.output_dim = int(L['feature_map_dim'])
            s.act = ACT_CODES[L['inneract']]
        s.bias = int(bool(L.get('bias', False)))
        s.dropout = int(bool(L.get('dropout', False)))
    return m


def validate(m: SgModel):
    """Returns (n_params, path): path 1 = fused kernel (sg_fast), 2 = fused capacity-32
    kernel (sg_fast32, config C4), 3 = graph-store path (sg_web_*, config C5),
    0 = generic kernel."""
    n = ctypes.c_int64(0)
    p = ctypes.c_int32(0)
    check(lib().sg_model_validate(ctypes.byref(m), ctypes.byref(n), ctypes.byref(p)),
          'sg_model_validate')
    return int(n.value), int(p.value)


def record_bytes(n_max: int, dtype='f32') -> int:
    return int(lib().sg_record_bytes_ex(int(n_max), dtype_code(dtype)))


def _ptr(t) -> Optional[int]:
    return None if t is None else int(t.data_ptr())


def _stream(stream) -> Optional[int]:
    if stream is None:
        import torch
        return int(torch.cuda.current_stream().cuda_stream)
    return int(stream)


def workspace_bytes(m: SgModel, n_pairs: int) -> int:
    b = int(lib().sg_workspace_bytes(ctypes.byref(m), int(n_pairs)))
    if b < 0:
        raise SiameseHipError('sg_workspace_bytes: unsupported model')
    return b


def pack_pairs(store_adj, store_types, store_n, n_max, pair_idx, labels, records, status=None,
               stream=None, dtype='f32'):
    n_graphs = int(store_n.shape[0])
    n_pairs = int(pair_idx.shape[0])
    check(lib().sg_pack_pairs_ex(_ptr(store_adj), _ptr(store_types), _ptr(store_n), n_graphs,
                                 int(n_max), dtype_code(dtype), _ptr(pair_idx), _ptr(labels),
                                 n_pairs, _ptr(records), _ptr(status), _stream(stream)),
          'sg_pack_pairs_ex')


def label_stats(records, n_pairs, n_max, stats_out, workspace, stream=None, dtype='f32'):
    check(lib().sg_label_stats_ex(_ptr(records), int(n_pairs), int(n_max), dtype_code(dtype),
                                  _ptr(stats_out), _ptr(workspace), _stream(stream)),
          'sg_label_stats_ex')


def pair_order_workspace_bytes(m: SgModel, n_pairs: int) -> int:
    b = int(lib().sg_pair_order_workspace_bytes(ctypes.byref(m), int(n_pairs)))
    if b < 0:
        raise SiameseHipError('sg_pair_order_workspace_bytes: bad arguments')
    return b


def pair_order(m: SgModel, records, n_pairs, order_out, workspace, stream=None):
    """Class-sorted processing order of the records (include/siamese_hip.h)."""
    check(lib().sg_pair_order(ctypes.byref(m), _ptr(records), int(n_pairs), _ptr(order_out),
                              _ptr(workspace), _stream(stream)), 'sg_pair_order')


def pair_order_cls(m: SgModel, records, n_pairs, order_out, class_start, workspace,
                   stream=None):
    """sg_pair_order plus the class table (int32 [FAST_CLASSES_P1]) of the fused path."""
    check(lib().sg_pair_order_cls(ctypes.byref(m), _ptr(records), int(n_pairs), _ptr(order_out),
                                  _ptr(class_start), _ptr(workspace), _stream(stream)),
          'sg_pair_order_cls')


def forward(m: SgModel, records, n_pairs, pair_offset, params, seed, s_out, workspace=None,
            stream=None, order=None, class_start=None):
    if class_start is not None:
        check(lib().sg_forward_cls(ctypes.byref(m), _ptr(records), _ptr(order),
                                   _ptr(class_start), int(n_pairs), int(pair_offset),
                                   _ptr(params), int(seed) & 0xFFFFFFFFFFFFFFFF, _ptr(s_out),
                                   _ptr(workspace), _stream(stream)), 'sg_forward_cls')
        return
    check(lib().sg_forward_ex(ctypes.byref(m), _ptr(records), _ptr(order), int(n_pairs),
                              int(pair_offset), _ptr(params), int(seed) & 0xFFFFFFFFFFFFFFFF,
                              _ptr(s_out), _ptr(workspace), _stream(stream)), 'sg_forward_ex')


def fwd_bwd(m: SgModel, records, n_pairs, pair_offset, batch_total, params, seed, y_stats,
            add_label_term, s_out, grad_out, loss_out, workspace, stream=None, order=None,
            class_start=None):
    if class_start is not None:
        check(lib().sg_fwd_bwd_cls(ctypes.byref(m), _ptr(records), _ptr(order),
                                   _ptr(class_start), int(n_pairs), int(pair_offset),
                                   int(batch_total), _ptr(params),
                                   int(seed) & 0xFFFFFFFFFFFFFFFF, _ptr(y_stats),
                                   int(add_label_term), _ptr(s_out), _ptr(grad_out),
                                   _ptr(loss_out), _ptr(workspace), _stream(stream)),
              'sg_fwd_bwd_cls')
        return
    check(lib().sg_fwd_bwd_ex(ctypes.byref(m), _ptr(records), _ptr(order), int(n_pairs),
                              int(pair_offset), int(batch_total), _ptr(params),
                              int(seed) & 0xFFFFFFFFFFFFFFFF, _ptr(y_stats), int(add_label_term),
                              _ptr(s_out), _ptr(grad_out), _ptr(loss_out), _ptr(workspace),
                              _stream(stream)), 'sg_fwd_bwd_ex')


def train_step(m: SgModel, records, n_pairs, pair_offset, batch_total, params, seed, y_stats,
               add_label_term, s_out, grad_out, loss_out, workspace, adam_m, adam_v, lr, beta1,
               beta2, eps, weight_decay, beta_powers, reg_loss=None, stream=None, order=None,
               class_start=None):
    """sg_train_step: fwd_bwd (class-scheduled when class_start is given) + adam_tf."""
    a = SgAdamArgs(_ptr(adam_m), _ptr(adam_v), float(lr), float(beta1), float(beta2), float(eps),
                   float(weight_decay), _ptr(beta_powers), _ptr(reg_loss))
    check(lib().sg_train_step(ctypes.byref(m), _ptr(records), _ptr(order), _ptr(class_start),
                              int(n_pairs), int(pair_offset), int(batch_total), _ptr(params),
                              int(seed) & 0xFFFFFFFFFFFFFFFF, _ptr(y_stats), int(add_label_term),
                              _ptr(s_out), _ptr(grad_out), _ptr(loss_out), _ptr(workspace),
                              ctypes.byref(a), _stream(stream)), 'sg_train_step')


def train_step_dseed(m: SgModel, records, n_pairs, pair_offset, batch_total, params, seed_dev,
                     y_stats, add_label_term, s_out, grad_out, loss_out, workspace, adam_m,
                     adam_v, lr, beta1, beta2, eps, weight_decay, beta_powers, reg_loss=None,
                     stream=None, order=None):
    """sg_train_step_dseed: train_step with the dropout seed read from device memory."""
    a = SgAdamArgs(_ptr(adam_m), _ptr(adam_v), float(lr), float(beta1), float(beta2), float(eps),
                   float(weight_decay), _ptr(beta_powers), _ptr(reg_loss))
    check(lib().sg_train_step_dseed(ctypes.byref(m), _ptr(records), _ptr(order), int(n_pairs),
                                    int(pair_offset), int(batch_total), _ptr(params),
                                    _ptr(seed_dev), _ptr(y_stats), int(add_label_term),
                                    _ptr(s_out), _ptr(grad_out), _ptr(loss_out), _ptr(workspace),
                                    ctypes.byref(a), _stream(stream)), 'sg_train_step_dseed')


def fwd_bwd_dseed(m: SgModel, records, n_pairs, pair_offset, batch_total, params, seed_dev,
                  y_stats, add_label_term, s_out, grad_out, loss_out, workspace, stream=None,
                  order=None):
    """fwd_bwd with the dropout seed read from the device (int64 tensor [1])."""
    check(lib().sg_fwd_bwd_dseed(ctypes.byref(m), _ptr(records), _ptr(order), int(n_pairs),
                                 int(pair_offset), int(batch_total), _ptr(params), _ptr(seed_dev),
                                 _ptr(y_stats), int(add_label_term), _ptr(s_out), _ptr(grad_out),
                                 _ptr(loss_out), _ptr(workspace), _stream(stream)),
          'sg_fwd_bwd_dseed')


def pair_source(store_dev, n_max, pair_idx=None, grid_base=0, labels=None, status=None):
    """sg_pair_source_t over a device dense store (adj, types, n) = GraphStore.to_device();
    pair_idx int32 [n, 2] or None for the all-pairs grid from grid_base.  The struct
    holds raw pointers: keep the tensors alive while it is in use."""
    adj, types, n = store_dev
    return SgPairSource(_ptr(adj), _ptr(types), _ptr(n), int(n.numel()), int(n_max),
                        _ptr(pair_idx), int(grid_base), _ptr(labels), _ptr(status))


def pair_order_src(m: SgModel, src: SgPairSource, n_pairs, order_out, workspace, stream=None):
    check(lib().sg_pair_order_src(ctypes.byref(m), ctypes.byref(src), int(n_pairs),
                                  _ptr(order_out), _ptr(workspace), _stream(stream)),
          'sg_pair_order_src')


def forward_src(m: SgModel, src: SgPairSource, n_pairs, pair_offset, params, seed, s_out,
                workspace=None, stream=None, order=None):
    check(lib().sg_forward_src(ctypes.byref(m), ctypes.byref(src), _ptr(order), int(n_pairs),
                               int(pair_offset), _ptr(params), int(seed) & 0xFFFFFFFFFFFFFFFF,
                               _ptr(s_out), _ptr(workspace), _stream(stream)), 'sg_forward_src')


def fwd_bwd_src(m: SgModel, src: SgPairSource, n_pairs, pair_offset, batch_total, params, seed,
                y_stats, add_label_term, s_out, grad_out, loss_out, workspace, stream=None,
                order=None):
    check(lib().sg_fwd_bwd_src(ctypes.byref(m), ctypes.byref(src), _ptr(order), int(n_pairs),
                               int(pair_offset), int(batch_total), _ptr(params),
                               int(seed) & 0xFFFFFFFFFFFFFFFF, _ptr(y_stats), int(add_label_term),
                               _ptr(s_out), _ptr(grad_out), _ptr(loss_out), _ptr(workspace),
                               _stream(stream)), 'sg_fwd_bwd_src')


def seed_advance(seed_dev, delta=1, stream=None):
    check(lib().sg_seed_advance(_ptr(seed_dev), int(delta) & 0xFFFFFFFFFFFFFFFF,
                                _stream(stream)), 'sg_seed_advance')


def feed_step(feed: SgFeed, pairs_out, records, labels_out, y_stats_out, status_out=None,
              stream=None):
    check(lib().sg_feed_step(ctypes.byref(feed), _ptr(pairs_out), _ptr(records),
                             _ptr(labels_out), _ptr(y_stats_out), _ptr(status_out),
                             _stream(stream)), 'sg_feed_step')


def sampler_random(state, sigma, n, count, pairs_out, stream=None):
    check(lib().sg_sampler_random(_ptr(state), _ptr(sigma), int(n), int(count), _ptr(pairs_out),
                                  _stream(stream)), 'sg_sampler_random')


def sampler_density(state, dens_order, bins, bin_size, item_table, count, pairs_out,
                    stream=None):
    check(lib().sg_sampler_density(_ptr(state), _ptr(dens_order), _ptr(bins),
                                   int(bins.numel()), int(bin_size), _ptr(item_table),
                                   int(count), _ptr(pairs_out), _stream(stream)),
          'sg_sampler_density')


def adam_tf(params, m, v, grad, lr, beta1, beta2, eps, weight_decay, beta_powers, reg_loss=None,
            stream=None):
    check(lib().sg_adam_tf(_ptr(params), _ptr(m), _ptr(v), _ptr(grad), int(params.numel()),
                           float(lr), float(beta1), float(beta2), float(eps), float(weight_decay),
                           _ptr(beta_powers), _ptr(reg_loss), _stream(stream)), 'sg_adam_tf')


def adam_tf_ex(params, m, v, grad, lr, beta1, beta2, eps, weight_decay, beta_powers, reg_loss,
               workspace, stream=None):
    check(lib().sg_adam_tf_ex(_ptr(params), _ptr(m), _ptr(v), _ptr(grad), int(params.numel()),
                              float(lr), float(beta1), float(beta2), float(eps),
                              float(weight_decay), _ptr(beta_powers), _ptr(reg_loss),
                              _ptr(workspace), _stream(stream)), 'sg_adam_tf_ex')


def adam_workspace_bytes(n: int) -> int:
    return int(lib().sg_adam_workspace_bytes(int(n)))


def csr_struct(n_graphs, n_max, node_off, types, row_ptr, col, val, max_nnz=0) -> SgCsrStore:
    s = SgCsrStore()
    s.max_nnz = int(max_nnz)
    s.n_graphs = int(n_graphs)
    s.n_max = int(n_max)
    s.node_off, s.types, s.row_ptr = _ptr(node_off), _ptr(types), _ptr(row_ptr)
    s.col, s.val = _ptr(col), _ptr(val)
    return s


def web_workspace_bytes(m: SgModel, chunk: int, n_pairs: int = -1) -> int:
    """Workspace of sg_web_* calls in chunks of `chunk`; n_pairs >= 0: calls of at most
    n_pairs pairs (one pipeline slot when n_pairs <= chunk, sg_web_workspace_bytes_ex)."""
    if n_pairs >= 0:
        b = int(lib().sg_web_workspace_bytes_ex(ctypes.byref(m), int(chunk), int(n_pairs)))
    else:
        b = int(lib().sg_web_workspace_bytes(ctypes.byref(m), int(chunk)))
    if b < 0:
        raise SiameseHipError('sg_web_workspace_bytes: model is not on the graph-store path')
    return b


def web_forward(m: SgModel, store: SgCsrStore, pairs, n_pairs, pair_offset, params, seed, s_out,
                workspace, chunk, stream=None):
    check(lib().sg_web_forward(ctypes.byref(m), ctypes.byref(store), _ptr(pairs), int(n_pairs),
                               int(pair_offset), _ptr(params), int(seed) & 0xFFFFFFFFFFFFFFFF,
                               _ptr(s_out), _ptr(workspace), int(chunk), _stream(stream)),
          'sg_web_forward')


def web_fwd_bwd(m: SgModel, store: SgCsrStore, pairs, labels, n_pairs, pair_offset, batch_total,
                params, seed, y_stats, add_label_term, s_out, grad_out, loss_out, workspace, chunk,
                stream=None):
    check(lib().sg_web_fwd_bwd(ctypes.byref(m), ctypes.byref(store), _ptr(pairs), _ptr(labels),
                               int(n_pairs), int(pair_offset), int(batch_total), _ptr(params),
                               int(seed) & 0xFFFFFFFFFFFFFFFF, _ptr(y_stats), int(add_label_term),
                               _ptr(s_out), _ptr(grad_out), _ptr(loss_out), _ptr(workspace),
                               int(chunk), _stream(stream)), 'sg_web_fwd_bwd')


def web_release():
    """sg_web_release: destroy the graph-store pipeline's auxiliary streams and events
    (teardown; no sg_web_* call may be in flight)."""
    rc = int(lib().sg_web_release())
    if rc != 0:
        raise SiameseHipError('sg_web_release failed ({})'.format(rc))
