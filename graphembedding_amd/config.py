"""Hyper-parameters with the names and defaults of model/Siamese/config.py:4-123.

`FLAGS` is a plain mutable namespace (the reference used tf.app.flags); the
layer stack is the same `Name:key=value,...` string grammar (config.py:44-66),
parsed by graphembedding_amd.layers_factory.create_layers.
"""
from __future__ import annotations

import argparse
import copy
from typing import Any, Dict, Optional

DEFAULTS: Dict[str, Any] = dict(
    # data (config.py:7-33)
    dataset='aids80nef',
    valid_percentage=0.25,
    node_feat_name='type',
    node_feat_encoder='onehot',
    edge_feat_name='valence',
    edge_feat_processor=None,
    dist_metric='ged',
    dist_algo='astar',
    sampler='random',
    sample_num=-1,
    sampler_duplicate_removal=False,
    # model (config.py:36-87)
    model='siamese_gcntn_mse',
    num_layers=5,
    layer_0='GraphConvolution:output_dim=32,act=relu,dropout=True,bias=True,sparse_inputs=True',
    layer_1='GraphConvolution:input_dim=32,output_dim=16,act=identity,dropout=True,bias=True,'
            'sparse_inputs=False',
    layer_2='Dense:input_dim=16,output_dim=1,dropout=True,act=relu,bias=True',
    layer_3='Padding:max_in_dims=10,padding_value=0',
    layer_4='NTN:input_dim=10,feature_map_dim=10,inneract=relu,dropout=True,bias=True',
    batch_size=5,
    dist_norm=True,
    sim_kernel='gaussian',
    yeta=0.6,
    final_act='sim_kernel',
    loss_func='mse',
    delta=0.1,
    gamma=0.1,
    num_neg=5,
    graph_loss=None,
    dropout=0.1,
    weight_decay=5e-4,
    learning_rate=0.01,
    # train / test (config.py:110-121)
    iters=20,
    early_stopping=None,
    log=True,
    plot_results=False,
    # ---- build-only knobs (no reference counterpart) ----
    loss_mode='broadcast',     # 'broadcast' = reference B×B quirk (A2) | 'aligned'
    ntn_mode='reference',      # 'reference' = (ΣU)·Σ relu(m) quirk (A1) | 'intended'
    label_stream='compat',     # 'compat' = labels from a later sampler draw (A3) | 'aligned'
    test_matrix='full',        # 'full' = sim_mat[i][j] | 'compat_diag' = sim_mat[i][i] (A5)
    # one-hot type -> column map: 'set' = Python set iteration order as graphs.py:101-104
    # (PYTHONHASHSEED-dependent for string types, quirk A7) | 'sorted' = sorted by str, the
    # same in every process (tests, multi-rank runs)
    node_feat_order='set',
    # test_time_mat: 'batched' = one launch for all m x n pairs, every entry the launch time
    # / (m n) (a deviation from the reference, recorded on the result); 'per_pair' = one
    # timed single-pair launch per entry, as train.py:57-69 times each sess.run
    test_time='batched',
    n_max=None,                # record node capacity (default: Padding max_in_dims or data max)
    record_dtype='f32',        # storage of Â in pair records: 'f32' | 'bf16' (config C3); fp32 math
    seed=123,                  # dropout RNG base seed (the reference's TF RNG was unseeded)
    param_seed=0,              # glorot init seed
)


class Flags:
    """tf.app.flags-like namespace: attribute access + flag_values_dict()."""

    def __init__(self, **overrides):
        self.__dict__['_values'] = copy.deepcopy(DEFAULTS)
        for k, v in overrides.items():
            setattr(self, k, v)

    def __getattr__(self, k):
        try:
            return self.__dict__['_values'][k]
        except KeyError:
            raise AttributeError(k)

    def __setattr__(self, k, v):
        self.__dict__['_values'][k] = v

    def flag_values_dict(self) -> Dict[str, Any]:
        return dict(self.__dict__['_values'])

    def copy(self, **overrides) -> 'Flags':
        f = Flags()
        f.__dict__['_values'] = copy.deepcopy(self.__dict__['_values'])
        for k, v in overrides.items():
            setattr(f, k, v)
        return f


FLAGS = Flags()


def reset_flag(flags: Flags, name: str, value) -> None:
    """tuning.py:192-194 equivalent."""
    setattr(flags, name, value)


def parse_args(argv=None, flags: Optional[Flags] = None) -> Flags:
    """--name=value overrides for every flag (absl-style command line)."""
    flags = flags or FLAGS
    p = argparse.ArgumentParser(allow_abbrev=False)
    for k, v in DEFAULTS.items():
        if isinstance(v, bool):
            p.add_argument('--' + k, type=lambda s: s.lower() in ('1', 'true', 'yes'), default=None)
        elif isinstance(v, int):
            p.add_argument('--' + k, type=int, default=None)
        elif isinstance(v, float):
            p.add_argument('--' + k, type=float, default=None)
        else:
            p.add_argument('--' + k, type=str, default=None)
    ns, _ = p.parse_known_args(argv)
    for k, v in vars(ns).items():
        if v is not None:
            setattr(flags, k, v)
    return flags


def check_flags(flags: Optional[Flags] = None) -> None:
    """model/Siamese/utils_siamese.py:13-19."""
    f = flags or FLAGS
    assert 0 < f.valid_percentage < 1
    assert f.sample_num >= -1
    assert f.yeta >= 0
    assert f.num_layers >= 2
    assert f.batch_size >= 1
