"""Synthetic Health-MNIST-shaped inputs (no network: the MNIST jpgs are unavailable offline).

Covariate rules follow Health_MNIST_generate.py:89-154 and the label permutation of
dataset_def.py:210-213 -- columns (time_age, disease_time, subject, gender, disease, location),
NaN -> 0; subject-contiguous rows (T per subject), as the Hensman reshape [P_b, T, Q] requires
(elbo_functions.py:168).
"""
import numpy as np
import torch


def health_mnist_covariates(P, T, seed=0):
    rng = np.random.default_rng(seed)
    sick = rng.binomial(1, 0.5, size=P)
    loc = rng.binomial(1, 0.5, size=P)
    p = np.repeat(np.arange(P), T)
    t = np.tile(np.arange(T), P)
    X = np.zeros((P * T, 6))
    X[:, 0] = t
    X[:, 1] = np.where(sick[p] == 1, t - 9, 0.0)
    X[:, 2] = p
    X[:, 3] = (p >= P // 2).astype(np.float64)
    X[:, 4] = sick[p]
    X[:, 5] = loc[p]
    return X


def health_mnist_batch(P, T, seed=0, device="cpu", dtype=torch.float32):
    """(images [N,1,36,36] uniform [0,1), mask [N,1,36,36] Bernoulli(0.75), covariates [N,6] f64)."""
    g = torch.Generator().manual_seed(seed)
    N = P * T
    img = torch.rand(N, 1, 36, 36, generator=g, dtype=dtype)
    mask = (torch.rand(N, 1, 36, 36, generator=g) < 0.75).to(dtype)
    X = torch.tensor(health_mnist_covariates(P, T, seed), dtype=torch.float64)
    return img.to(device), mask.to(device), X.to(device)
