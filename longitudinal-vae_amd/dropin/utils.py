"""utils.py surface (reference utils.py:9-211): subject samplers, the Hensman loader and the GP
posterior prediction, backed by lvae_amd.  Samplers keep the reference constructors; the
reference's unseeded np.random.shuffle (utils.py:53, 76) is kept as the default (seed=None)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lvae_amd import samplers as _s  # noqa: E402
from lvae_amd.data import DeviceBatchLoader  # noqa: E402
from lvae_amd.predict import batch_predict_varying_T  # noqa: E402,F401


class SubjectSampler:
    """SubjectSampler(data_source, P, T) (utils.py:40-59): row indices of a shuffled subject order."""

    def __init__(self, data_source, P, T, seed=None):
        self.data_source = data_source
        self._s = _s.SubjectSampler(P, T, seed)

    def __iter__(self):
        return iter(self._s)

    def __len__(self):
        return len(self.data_source)


class VaryingLengthSubjectSampler:
    """VaryingLengthSubjectSampler(data_source, id_covariate) (utils.py:61-87): yields (row, subject)
    pairs over a shuffled subject order; subjects are contiguous runs of the id column."""

    def __init__(self, data_source, id_covariate, seed=None):
        self.data_source = data_source
        if hasattr(data_source, "labels"):
            ids = data_source.labels[:, id_covariate].cpu().numpy()
        else:
            ids = np.array([float(data_source[i]["label"][id_covariate]) for i in range(len(data_source))])
        self._s = _s.VaryingLengthSubjectSampler(ids, seed)
        self.P = len(self._s)

    def __iter__(self):
        return iter(self._s)

    def __len__(self):
        return self.P


class VaryingLengthBatchSampler:
    """VaryingLengthBatchSampler(sampler, batch_size) (utils.py:89-113): index batches of
    batch_size whole subjects."""

    def __init__(self, sampler, batch_size):
        self.sampler, self.batch_size = sampler, batch_size

    def __iter__(self):
        return iter(_s.varying_length_batches(self.sampler._s, self.batch_size))

    def __len__(self):
        return (len(self.sampler) + self.batch_size - 1) // self.batch_size


class HensmanDataLoader(DeviceBatchLoader):
    """HensmanDataLoader(dataset, batch_sampler, num_workers) (utils.py:24-38): device batches in
    the batch sampler's order (no worker processes: the dataset is device-resident)."""

    def __init__(self, dataset, batch_sampler, num_workers=0):
        super().__init__(dataset, batch_sampler)


__all__ = ["SubjectSampler", "VaryingLengthSubjectSampler", "VaryingLengthBatchSampler", "HensmanDataLoader",
           "batch_predict_varying_T"]
