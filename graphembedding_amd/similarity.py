"""Distance → similarity kernels (src/similarity.py:5-76), same interface.

`dist_to_sim_tf` of the reference becomes `dist_to_sim_torch` (same math on a
torch tensor); the name `dist_to_sim_tf` is kept as an alias so callers that
only need the value keep working.
"""
from __future__ import annotations

import numpy as np


def format_float(f):
    """src/utils.py:285-291."""
    if f < 1e-2:
        return '{:.2e}'.format(f)
    return '{:.2f}'.format(f)


class SimilarityKernel(object):
    def name(self):
        return ''

    def shortname(self):
        return ''

    def name_suffix(self):
        return ''

    def dist_to_sim_np(self, dist, max_dist):
        raise NotImplementedError()

    def dist_to_sim_torch(self, dist, max_dist):
        raise NotImplementedError()


class IdentityKernel:
    def dist_to_sim_np(self, dist, *unused):
        return self._d_to_s(dist)

    def dist_to_sim_torch(self, dist, *unused):
        return self._d_to_s(dist)

    dist_to_sim_tf = dist_to_sim_torch

    def _d_to_s(self, dist):
        return dist


class GaussianKernel(SimilarityKernel):
    def __init__(self, yeta):
        self.yeta = yeta

    def name(self):
        return 'Gaussian_yeta={}'.format(format_float(self.yeta))

    def shortname(self):
        return 'g_{:.2e}'.format(self.yeta)

    def dist_to_sim_np(self, dist, *unused):
        return np.exp(-self.yeta * np.square(dist))

    def dist_to_sim_torch(self, dist, *unused):
        import torch
        return torch.exp(-self.yeta * torch.square(dist))

    dist_to_sim_tf = dist_to_sim_torch


class BinaryKernel(SimilarityKernel):
    def __init__(self, threshold):
        self.threshold = threshold


def create_sim_kernel(kernel_name, yeta=None):
    if kernel_name == 'identity':
        return IdentityKernel()
    elif kernel_name == 'gaussian':
        return GaussianKernel(yeta)
    else:
        raise RuntimeError('Unknown sim kernel {}'.format(kernel_name))
