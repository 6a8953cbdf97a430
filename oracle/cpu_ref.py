"""TEST INFRASTRUCTURE ONLY — ctypes front of oracle/_build/libsiamese_cpu.so
(the C restatement in siamese_cpu.c) and the bounded CPU-baseline timing that
bench.py reports as "cpu_baseline" ("kind": "port")."""
from __future__ import annotations

import ctypes
import os
import subprocess
import time

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, '_build', 'libsiamese_cpu.so')
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.isfile(_SO):
            subprocess.run(['make', '-s', '-C', _HERE], check=True)
        L = ctypes.CDLL(_SO)
        vp = ctypes.c_void_p
        L.sgc_n_params.argtypes = [ctypes.c_int, ctypes.c_int]
        L.sgc_n_params.restype = ctypes.c_int64
        L.sgc_fwd_bwd.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                  vp, ctypes.c_uint64, ctypes.c_float, ctypes.c_float,
                                  ctypes.c_float, vp, vp, vp, ctypes.c_int]
        L.sgc_fwd_bwd.restype = ctypes.c_int
        L.sgc_fwd_bwd_f64acc.argtypes = L.sgc_fwd_bwd.argtypes
        L.sgc_fwd_bwd_f64acc.restype = ctypes.c_int
        _lib = L
    return _lib


def fwd_bwd_records(words: np.ndarray, n_max: int, d_in: int, params: np.ndarray, seed: int,
                    keep: float, yeta: float, ybar: float, pair_offset: int = 0,
                    threads: int = 1, f64_acc: bool = False):
    """Default-stack fwd+bwd over host records (uint32 [P][W]).
    Returns (s [P], grad_mse [n_params], loss ½Σ(ŷ-ȳ)²).  f64_acc: the same float32
    per-pair arithmetic with the gradient summed in double (the full-batch checker)."""
    L = lib()
    words = np.ascontiguousarray(words, dtype=np.uint32)
    P = words.shape[0]
    params = np.ascontiguousarray(params, dtype=np.float32)
    npar = int(L.sgc_n_params(d_in, n_max))
    assert params.size == npar, (params.size, npar)
    s = np.zeros(P, np.float32)
    g = np.zeros(npar, np.float32)
    loss = ctypes.c_double(0.0)
    fn = L.sgc_fwd_bwd_f64acc if f64_acc else L.sgc_fwd_bwd
    rc = fn(words.ctypes.data, P, int(pair_offset), int(n_max), int(d_in),
                       params.ctypes.data, int(seed) & 0xFFFFFFFFFFFFFFFF, float(keep),
                       float(yeta), float(ybar), s.ctypes.data, g.ctypes.data,
                       ctypes.addressof(loss), int(threads))
    if rc != 0:
        raise RuntimeError('sgc_fwd_bwd failed')
    return s, g, float(loss.value)


def adam_step(params: np.ndarray, grad_mse: np.ndarray, st, flags) -> np.ndarray:
    """The step's ApplyAdam (models.py:28-36, TF form) with weight decay on every variable
    (models.py:67-74, quirk A10), as the timed GPU step runs it after fwd+bwd."""
    from oracle import siamese_oracle as O
    g = grad_mse.astype(np.float64) + flags.weight_decay * params.astype(np.float64)
    return O.adam_tf_step(params.astype(np.float64), g, st,
                          lr=flags.learning_rate).astype(np.float32)


def default_threads() -> int:
    env = os.environ.get('OMP_NUM_THREADS')
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return max(1, len(os.sched_getaffinity(0)))
    except AttributeError:
        return max(1, os.cpu_count() or 1)


def time_allpairs_sample(gs, labels, flags, n_sample: int = 0, target_s: float = 12.0,
                         threads: int = 0):
    """Time fwd+bwd of the C restatement on the all-pairs stream of `gs`.
    n_sample > 0: the first n_sample pairs once.  n_sample == 0 (auto): about
    target_s seconds of work — whole all-pairs passes repeated when one pass is
    shorter than that, else a prefix of the stream."""
    from graphembedding_amd.model_mse import glorot_flat
    from graphembedding_amd.layers_factory import create_layers
    G = len(gs.graphs)
    total = G * G
    threads = threads if threads and threads > 0 else default_threads()
    layers = create_layers(flags, gs.d_in)
    params = glorot_flat(layers, gs.d_in, flags.param_seed)
    ybar = float(labels.astype(np.float64).mean())
    cache = {}

    def words_for(n):
        if n not in cache:
            p = np.arange(n, dtype=np.int64)
            pairs = np.stack([p // G, p % G], axis=1)
            cache[n] = gs.store.pack_host(pairs, labels.reshape(-1)[:n])
        return cache[n]

    def run(n, reps=1):
        from oracle import siamese_oracle as O
        w = words_for(n)
        p = params.copy()
        st = O.adam_init(p.size)
        t0 = time.perf_counter()
        for r in range(reps):   # one training step: fwd+bwd, then Adam, like the GPU step
            _, g, _ = fwd_bwd_records(w, gs.n_max, gs.d_in, p, 1 + r, 1.0 - flags.dropout,
                                      flags.yeta, ybar, threads=threads)
            p = adam_step(p, g, st, flags)
        return time.perf_counter() - t0

    reps = 1
    if n_sample <= 0:
        probe = min(total, 20000)
        rate = probe / max(run(probe), 1e-6)
        want = rate * target_s
        if want >= total:
            n_sample, reps = total, max(1, int(round(want / total)))
        else:
            n_sample = max(probe, int(want))
    n_sample = min(n_sample, total)
    dt = run(n_sample, reps)
    what = ('{} full all-pairs passes ({} pairs each)'.format(reps, n_sample) if reps > 1
            else 'first {} pairs of the all-pairs stream'.format(n_sample))
    return {'value': n_sample * reps / dt, 'unit': 'graph-pairs/s', 'cores': threads,
            'kind': 'port',
            'sample': '{}, one training step each (fwd+bwd: loss + grads, then TF Adam with '
                      'weight decay), C restatement oracle/siamese_cpu.c, fp32, OpenMP {} '
                      'threads, {:.1f} s'.format(what, threads, dt)}


def time_web_sample(gs, labels, flags, n_sample: int = 32, target_s: float = 12.0,
                    threads: int = 0, seed: int = 0):
    """Config C5 (Web-sized graphs): time the C restatement on a seeded random
    sample of n_sample pairs of the all-pairs stream, packed as dense records at
    capacity n_max = D (the port has no sparse path), repeated for ~target_s."""
    from graphembedding_amd.model_mse import glorot_flat
    from graphembedding_amd.layers_factory import create_layers
    from graphembedding_amd.packer import GraphStore
    G = len(gs.graphs)
    threads = threads if threads and threads > 0 else default_threads()
    layers = create_layers(flags, gs.d_in)
    params = glorot_flat(layers, gs.d_in, flags.param_seed)
    ybar = float(labels.astype(np.float64).mean())
    rng = np.random.default_rng(seed)
    p = rng.choice(G * G, size=n_sample, replace=False)
    pairs = np.stack([p // G, p % G], axis=1)
    uniq, inv = np.unique(pairs.reshape(-1), return_inverse=True)
    store = GraphStore([gs.mgs[i] for i in uniq], gs.n_max, gs.d_in)
    words = store.pack_host(inv.reshape(-1, 2), labels.reshape(-1)[p])
    from oracle import siamese_oracle as O
    st = O.adam_init(params.size)
    t0 = time.perf_counter()
    reps = 0
    while True:
        _, g, _ = fwd_bwd_records(words, gs.n_max, gs.d_in, params, 1 + reps,
                                  1.0 - flags.dropout, flags.yeta, ybar, threads=threads)
        params = adam_step(params, g, st, flags)
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= target_s:
            break
    return {'value': n_sample * reps / dt, 'unit': 'graph-pairs/s', 'cores': threads,
            'kind': 'port',
            'sample': '{} x {} random pairs of the all-pairs stream (seed {}), fwd+bwd (loss + '
                      'grads) + TF Adam per pass, C restatement oracle/siamese_cpu.c on dense capacity-{} '
                      'records, fp32, OpenMP {} threads, {:.1f} s'.format(
                          reps, n_sample, seed, gs.n_max, threads, dt)}
