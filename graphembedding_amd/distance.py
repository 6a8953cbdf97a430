"""Graph distances (src/distance.py).

Only `normalized_dist` (distance.py:59-60) is on the hot path.  `ged` and `mcs`
shell out to the Java graph-matching-toolkit / the `chorus` library in the
reference (distance.py:10-56); those solvers are out of scope here and raise
unless a cached distance exists (see dist_calculator.DistCalculator).
"""
from __future__ import annotations


def normalized_dist(d, g1, g2):
    return 2 * d / (g1.number_of_nodes() + g2.number_of_nodes())


def ged(g1, g2, algo, debug=False, timeit=False):
    raise RuntimeError(
        'GED ground truth needs the external Java graph-matching-toolkit '
        '(reference src/distance.py:23-56); it is out of scope of this build. '
        'Provide a cached gid-pair distance map instead.')


def mcs(g1, g2):
    raise RuntimeError('MCS needs the external chorus library (reference src/distance.py:10-20).')
