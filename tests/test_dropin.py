"""The drop-in flat modules expose the reference's import surface (training.py:9-13,
LVAE.py:15-22, validation.py:5-6, model_test.py:9) backed by lvae_amd (no compute here)."""
import importlib
import os
import sys

import numpy as np

from conftest import ROOT

DROPIN = os.path.join(ROOT, "longitudinal-vae_amd", "dropin")

SURFACE = {
    "elbo_functions": ["KL_closed", "elbo", "deviance_upper_bound", "minibatch_KLD_upper_bound",
                       "minibatch_KLD_upper_bound_iter"],
    "kernel_gen": ["generate_kernel", "generate_kernel_approx", "generate_kernel_batched"],
    "GP_model": ["Likelihoods", "BinKernel", "CatKernel", "RbfKernel", "ScaleKernel", "AdditiveKernel",
                 "ProductKernel", "generate_kernel_batched"],
    "utils": ["SubjectSampler", "VaryingLengthSubjectSampler", "VaryingLengthBatchSampler", "HensmanDataLoader",
              "batch_predict_varying_T"],
    "dataset_def": ["HealthMNISTDatasetConv"],
}


def _import(name):
    sys.path.insert(0, DROPIN)
    try:
        sys.modules.pop(name, None)
        return importlib.import_module(name)
    finally:
        sys.path.remove(DROPIN)


def test_surface():
    for mod, names in SURFACE.items():
        m = _import(mod)
        assert m.__file__.startswith(DROPIN), m.__file__
        for n in names:
            assert hasattr(m, n), f"{mod}.{n}"
        sys.modules.pop(mod, None)


def test_reference_sampler_semantics():
    u = _import("utils")
    data = list(range(12))
    s = u.SubjectSampler(data, 3, 4, seed=1)
    rows = list(s)
    assert len(s) == 12 and sorted(rows) == data
    for k in range(3):  # whole subjects, contiguous, time-ordered
        blk = rows[4 * k: 4 * k + 4]
        assert blk == list(range(blk[0], blk[0] + 4)) and blk[0] % 4 == 0

    class DS:
        def __init__(self, ids):
            self.ids = ids

        def __len__(self):
            return len(self.ids)

        def __getitem__(self, i):
            return {"label": np.array([0.0, 0.0, self.ids[i]])}

    ids = [0, 0, 0, 1, 1, 2, 2, 2, 2, 3]
    vs = u.VaryingLengthSubjectSampler(DS(ids), 2, seed=3)
    batches = list(u.VaryingLengthBatchSampler(vs, 2))
    assert len(vs) == 4 and len(batches) == 2
    got = sorted(i for b in batches for i in b)
    assert got == list(range(10))
    for b in batches:
        assert len({ids[i] for i in b}) == 2
    sys.modules.pop("utils", None)
