"""Paths, natural sort and pickle caches (src/utils.py:15-35, 45-75, 148-160,
203-234).  Pickles are written by this package only; foreign pickles (e.g. a
user's GED distance map) are read through `safe_load`, a restricted unpickler
that only materialises plain containers and numbers.
"""
from __future__ import annotations

import io
import os
import pickle
import re

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def get_root_path():
    return os.environ.get('SG_ROOT_PATH', _ROOT)


def get_data_path():
    return os.environ.get('SG_DATA_PATH', os.path.join(get_root_path(), 'data'))


def get_save_path():
    return os.environ.get('SG_SAVE_PATH', os.path.join(get_root_path(), 'save'))


def get_result_path():
    return os.environ.get('SG_RESULT_PATH', os.path.join(get_root_path(), 'result'))


def create_dir_if_not_exists(d):
    os.makedirs(d, exist_ok=True)


def get_train_str(train):
    return 'train' if train else 'test'


def get_file_base_id(file):
    return int(file.split('/')[-1].split('.')[0])


def sorted_nicely(l):
    def tryint(s):
        try:
            return int(s)
        except ValueError:
            return s

    def alphanum_key(s):
        return [tryint(c) for c in re.split('([0-9]+)', s)]

    return sorted(l, key=alphanum_key)


def proc_filepath(filepath):
    if type(filepath) is not str:
        raise RuntimeError('Did you pass a file path to this function?')
    ext = '.pickle'
    if ext not in filepath:
        filepath += ext
    return filepath


def save(filepath, obj):
    filepath = proc_filepath(filepath)
    create_dir_if_not_exists(os.path.dirname(filepath) or '.')
    with open(filepath, 'wb') as handle:
        pickle.dump(obj, handle, protocol=pickle.HIGHEST_PROTOCOL)


def load(filepath):
    """Load a cache pickle written by this package (returns None if absent)."""
    filepath = proc_filepath(filepath)
    if os.path.isfile(filepath):
        with open(filepath, 'rb') as handle:
            return pickle.load(handle)
    return None


class _SafeUnpickler(pickle.Unpickler):
    _ALLOWED = {('collections', 'OrderedDict'), ('builtins', 'dict'), ('builtins', 'list'),
                ('builtins', 'tuple'), ('builtins', 'set'), ('builtins', 'frozenset'),
                ('builtins', 'int'), ('builtins', 'float'), ('builtins', 'str')}

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError('refusing to load {}.{}'.format(module, name))


def safe_load(filepath):
    """Load a foreign pickle holding only containers / numbers (e.g. the
    reference's gid-pair distance map, dist_calculator.py:8-20)."""
    filepath = proc_filepath(filepath)
    if not os.path.isfile(filepath):
        return None
    with open(filepath, 'rb') as f:
        return _SafeUnpickler(io.BytesIO(f.read())).load()


def load_data(data, train):
    """src/utils.py:15-35 plus the synthetic stand-ins of BASELINE.md §3."""
    from . import data as D
    if data == 'syn':
        return D.SynData(train)
    elif data == 'aids10knef':
        return D.AIDS10kNEFData(train)
    elif data == 'aids10k':
        return D.AIDS10kData(train)
    elif data == 'aids700nef':
        return D.AIDS700nefData(train)
    elif data == 'aids80nef':
        return D.AIDS80nefData(train)
    elif data.startswith('syn_'):
        return D.SyntheticAIDSData(data, train)
    else:
        raise RuntimeError('Not recognized data %s' % data)
