"""Layer-string grammar of model/Siamese/layers_factory.py:8-127.

`create_layers(flags, input_dim)` turns FLAGS.layer_0..layer_{num_layers-1}
into plain layer dicts (the format of graphembedding_amd._lib.make_model and of
the oracle), raising the same RuntimeErrors as the reference for malformed
specs.  `Attention` is accepted as a build option: the reference defines the
class (layers.py:143-160) but its factory cannot create it (quirk A14).
"""
from __future__ import annotations

from math import exp
from typing import List

import numpy as np


def parse_as_bool(b: str) -> bool:
    if b == 'True':
        return True
    if b == 'False':
        return False
    raise RuntimeError('Unknown bool string {}'.format(b))


def _parse(spec: str):
    sp = spec.split(':')
    name = sp[0]
    info = {}
    if len(sp) > 1:
        assert len(sp) == 2
        for item in sp[1].split(','):
            ssp = item.split('=')
            info[ssp[0]] = ssp[1]
    return name, info


_ACTS = ('relu', 'identity', 'sigmoid', 'tanh')


def _check_act(a: str) -> str:
    if a not in _ACTS:
        raise RuntimeError('Unknown activation function {}'.format(a))
    return a


def create_layers(flags, input_dim: int) -> List[dict]:
    layers = []
    for i in range(flags.num_layers):
        name, info = _parse(flags.flag_values_dict()['layer_{}'.format(i)])
        if name == 'GraphConvolution':
            if not 5 <= len(info) <= 6:
                raise RuntimeError('GraphConvolution layer must have 3-4 specs')
            din = info.get('input_dim')
            if not din:
                if i != 0:
                    raise RuntimeError('The input dim for layer {} must be specified'.format(i))
                din = input_dim
            layers.append(dict(kind='GraphConvolution', input_dim=int(din),
                               output_dim=int(info['output_dim']),
                               dropout=parse_as_bool(info['dropout']),
                               sparse_inputs=parse_as_bool(info['sparse_inputs']),
                               act=_check_act(info['act']), bias=parse_as_bool(info['bias'])))
        elif name == 'Average':
            if len(info) != 0:
                raise RuntimeError('Average layer must have 0 specs')
            layers.append(dict(kind='Average'))
        elif name == 'Attention':
            if len(info) != 1:
                raise RuntimeError('Attention layer must have 1 spec (input_dim)')
            layers.append(dict(kind='Attention', input_dim=int(info['input_dim'])))
        elif name == 'NTN':
            if len(info) != 5:
                raise RuntimeError('Average layer must have 0 specs')  # sic, layers_factory.py:63
            layers.append(dict(kind='NTN', input_dim=int(info['input_dim']),
                               feature_map_dim=int(info['feature_map_dim']),
                               dropout=parse_as_bool(info['dropout']),
                               inneract=_check_act(info['inneract']),
                               bias=parse_as_bool(info['bias'])))
        elif name == 'Dot':
            if len(info) != 0:
                raise RuntimeError('Dot layer must have 0 specs')
            layers.append(dict(kind='Dot'))
        elif name == 'Dense':
            if len(info) != 5:
                raise RuntimeError('Dot layer must have 5 specs')  # sic, layers_factory.py:80
            layers.append(dict(kind='Dense', input_dim=int(info['input_dim']),
                               output_dim=int(info['output_dim']),
                               dropout=parse_as_bool(info['dropout']),
                               act=_check_act(info['act']), bias=parse_as_bool(info['bias'])))
        elif name == 'Padding':
            if len(info) != 2:
                raise RuntimeError('Padding layer must have 2 specs')
            layers.append(dict(kind='Padding', max_in_dims=int(info['max_in_dims']),
                               padding_value=int(info['padding_value'])))
        else:
            raise RuntimeError('Unknown layer {}'.format(name))
    return layers


def padding_dims(layers: List[dict]):
    for L in layers:
        if L['kind'] == 'Padding':
            return L['max_in_dims']
    return None


# numpy activations used by apply_final_act_np (layers_factory.py:101-127)
def relu_np(x):
    return np.maximum(x, 0)


def identity_np(x):
    return x


def sigmoid_np(x):
    return 1 / (1 + exp(-x))


def create_activation(act, sim_kernel=None, use_tf=False):
    if use_tf:
        raise RuntimeError('TensorFlow activations are not part of this build')
    if act == 'relu':
        return relu_np
    if act == 'identity':
        return identity_np
    if act == 'sigmoid':
        return sigmoid_np
    if act == 'tanh':
        return np.tanh
    if act == 'sim_kernel':
        return sim_kernel.dist_to_sim_np
    raise RuntimeError('Unknown activation function {}'.format(act))
