"""Calibrate the gate of the diag(K^-1) refinement on the CPU: for the -m gpu suite's KL draws (headline
workload, high-cond, small-noise), an fp32 LAPACK Cholesky inverse stands in for the GPU's x3 f16 one.
Printed per dim: cond(K), the dlogv error of the fp32 inverse (the tests' max-abs relative measure), the
relative size of the alpha refinement step ||a - a0|| / ||a|| (what the GPU already computes), and the
dlogv error after one fp64 Newton step on the diagonal: d' = 2 diag X - diag(X K X).

    python scripts/refine_calib.py"""
import os
import sys

import numpy as np
import scipy.linalg.lapack as lp
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "longitudinal-vae_amd"))
from oracle import lvae_oracle as O  # noqa: E402
import lvae_amd as la  # noqa: E402
from lvae_amd.data import health_mnist_covariates  # noqa: E402

CFG = dict(cat_kernel=[2], bin_kernel=[], sqexp_kernel=[0],
           cat_int_kernel=[{'cont_covariate': 0, 'cat_covariate': 2},
                           {'cont_covariate': 0, 'cat_covariate': 3},
                           {'cont_covariate': 1, 'cat_covariate': 4}],
           bin_int_kernel=[], covariate_missing_val=[])


def hypers(L, rng, scale=(0.3, 1.5), ell=(1.0, 4.0)):
    k = la.generate_kernel(**CFG, latent_dim=L)
    return np.stack([np.log(rng.uniform(*scale, L)) if "scale" in n else np.log(rng.uniform(*ell, L))
                     for n, _ in k.named_parameters()], 1)


def case(name, P, L, raw, noise, seed):
    X = torch.tensor(health_mnist_covariates(P, 16, seed=seed))
    gen = torch.Generator().manual_seed(seed)
    mu = torch.randn(P * 16, L, generator=gen, dtype=torch.float64).numpy()
    lv = 0.1 * torch.randn(P * 16, L, generator=gen, dtype=torch.float64).numpy()
    spec = O.spec_full(**CFG)
    for l in range(L):
        K = O.gram(spec, O.constrain(torch.tensor(raw[l])), X, X).numpy() + float(noise[l]) * np.eye(P * 16)
        ev = np.linalg.eigvalsh(K)
        Ki = np.linalg.inv(K)
        c32, info = lp.spotrf(K.astype(np.float32), lower=1)
        X32, info2 = lp.spotri(c32, lower=1)
        X32 = np.tril(X32) + np.tril(X32, -1).T
        X64 = X32.astype(np.float64)
        v = np.exp(lv[:, l])
        ref = 0.5 * (v * np.diag(Ki) - 1)
        d32 = np.diag(X64)
        e32 = np.abs(0.5 * (v * d32 - 1) - ref).max() / np.abs(ref).max()
        a = Ki @ mu[:, l]
        a0 = X64 @ mu[:, l]
        est = np.linalg.norm(a0 - a) / np.linalg.norm(a)
        estc = np.diag(K).max() * np.diag(X64).max()
        dref = 2 * d32 - np.einsum("ij,ij->j", X64, K @ X64)
        e_ref = np.abs(0.5 * (v * dref - 1) - ref).max() / np.abs(ref).max()
        print(f"{name} dim {l}: cond {ev[-1] / ev[0]:.2e}  dlogv err fp32 {e32:.2e}  alpha step {est:.2e}  "
              f"ratio {e32 / est:.2f}  refined {e_ref:.2e}  maxKii*maxXii {estc:.2e} ({estc / (ev[-1] / ev[0]):.2f} cond)", flush=True)


def main():
    k = la.generate_kernel(**CFG, latent_dim=2)
    raw = torch.stack([p.detach().double().reshape(-1) for _, p in k.named_parameters()], 1).numpy()
    print("bench init raw params", raw[0])
    case("bench_init", 256, 1, raw[:1], np.ones(1), 16)
    rng = np.random.default_rng(16)
    raw = hypers(16, rng)
    noise = rng.uniform(0.5, 1.0, 16)
    case("headline", 256, 16, raw, noise, 16)
    rng = np.random.default_rng(17)
    raw = hypers(8, rng, scale=(0.2, 3.0), ell=(0.5, 6.0))
    noise = rng.uniform(0.05, 1.0, 8)
    case("high_cond", 256, 8, raw, noise, 17)
    for nz in (1e-3, 1e-4):
        rng = np.random.default_rng(int(1 / nz))
        raw = hypers(2, rng)
        case(f"small_noise {nz}", 64, 2, raw, np.full(2, nz), 3)


if __name__ == "__main__":
    main()
