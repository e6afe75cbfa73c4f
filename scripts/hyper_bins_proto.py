"""CPU prototype (fp64) of the binned hyper-parameter gradient of the exact KL: d KL / d theta_p =
sum_ij G_ij dK_ij/dtheta_p, G = (K^-1 - S - alpha alpha^T) / 2, S = K^-1 V K^-1, evaluated WITHOUT S:
  far components (no gate on the big covariate): bins b = (small gate values, integer distance value);
      sum_ij X_ij F(b_i, b_j) = sum_bb' F[b][b'] (Phi^T X Phi)[b][b'], and Phi^T S Phi = H V H^T with
      H = Phi^T K^-1 (bin sums of K^-1's rows), Phi^T K^-1 Phi = H Phi, Phi^T alpha alpha^T Phi = a a^T;
  near components (gated by the big covariate, e.g. the subject): only pairs inside a run of equal big values
      (contiguous), S's run blocks = X_run V X_run^T from the run's rows of K^-1.
Checked against autograd of the oracle's KL_closed."""
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "longitudinal-vae_amd"))
from oracle import lvae_oracle as O  # noqa: E402
from lvae_amd.data import health_mnist_covariates  # noqa: E402

CFG = dict(cat_kernel=[2], bin_kernel=[], sqexp_kernel=[0],
           cat_int_kernel=[{'cont_covariate': 0, 'cat_covariate': 2}, {'cont_covariate': 0, 'cat_covariate': 3},
                           {'cont_covariate': 1, 'cat_covariate': 4}], bin_int_kernel=[], covariate_missing_val=[])


def main(P=12, T=16, seed=0):
    torch.manual_seed(seed)
    X = torch.tensor(health_mnist_covariates(P, T, seed=seed))
    N = X.shape[0]
    spec = O.spec_full(**CFG)
    rng = np.random.default_rng(seed)
    params = torch.tensor(rng.uniform(0.5, 2.5, O.n_params(spec)), requires_grad=True)
    mu = torch.randn(N, dtype=torch.float64)
    lv = 0.3 * torch.randn(N, dtype=torch.float64)
    kl = O.kl_closed(spec, params, X, 1.0, mu, lv)
    kl.backward()
    ref = params.grad.clone()

    with torch.no_grad():
        K = O.gram(spec, params, X, X) + torch.eye(N, dtype=torch.float64)
        Ki = torch.linalg.inv(K)
        v = torch.exp(lv)
        al = Ki @ mu
        x = X.numpy()
        big = 2  # the subject covariate
        # runs of the big covariate (sorted: contiguous)
        starts = [0] + [i for i in range(1, N) if x[i, big] != x[i - 1, big]] + [N]
        got = torch.zeros_like(ref)
        j = 0
        for comp in spec:
            s = params[j].item()
            js = j
            j += 1
            gates = [f for f in comp if f[0] in ("cat", "bin")]
            cont = [f for f in comp if f[0] in ("rbf", "per")]
            jl = None
            if cont:
                jl = j
                j += 1
            ell = params[jl].item() if cont else None

            def phi_and_dphi(dd):  # factor and d factor / d ell at distance dd (array)
                if not cont:
                    return np.ones_like(dd), np.zeros_like(dd)
                ph = np.exp(-dd ** 2 / (2 * ell ** 2))
                return ph, ph * dd ** 2 / ell ** 3

            near = any(f[0] == "cat" and f[1] == big for f in gates)
            if near:
                # pairs inside runs only: sum over runs of (K^-1 - S - aa^T)_ij dK_ij
                ts = tl = 0.0
                for a, b in zip(starts[:-1], starts[1:]):
                    idx = np.arange(a, b)
                    Xr = Ki[a:b, :]
                    Srun = (Xr * v) @ Xr.T
                    G = 0.5 * (Ki[a:b, a:b] - Srun - torch.outer(al[a:b], al[a:b])).numpy()
                    gate = np.ones((b - a, b - a))
                    for kind, d in gates:
                        xi, xj = x[idx, d][:, None], x[idx, d][None, :]
                        gate *= (xi == xj) if kind == "cat" else (xi + xj == 2)
                    dd = (x[idx, cont[0][1]][:, None] - x[idx, cont[0][1]][None, :]) if cont else np.zeros_like(gate)
                    ph, dph = phi_and_dphi(dd)
                    ts += (G * gate * ph).sum()
                    tl += (G * gate * s * dph).sum()
                got[js] = ts
                if cont:
                    got[jl] = tl
            else:
                # far: bins b = (small gate values..., distance-dim value)
                keys = [tuple(int(x[i, d]) for _, d in gates) + ((int(x[i, cont[0][1]]),) if cont else ()) for i in range(N)]
                uniq = sorted(set(keys))
                bix = {k: q for q, k in enumerate(uniq)}
                nb = len(uniq)
                Phi = torch.zeros(N, nb, dtype=torch.float64)
                for i, k in enumerate(keys):
                    Phi[i, bix[k]] = 1.0
                H = Phi.T @ Ki                      # bin sums of K^-1's rows
                Mk = H @ Phi                        # Phi^T K^-1 Phi
                Ms = (H * v) @ H.T                  # Phi^T S Phi
                aa = Phi.T @ al
                Ma = torch.outer(aa, aa)
                Gb = 0.5 * (Mk - Ms - Ma).numpy()
                # F over bin pairs
                kb = np.array(uniq, dtype=float)
                gate = np.ones((nb, nb))
                for q, (kind, d) in enumerate(gates):
                    xi, xj = kb[:, q][:, None], kb[:, q][None, :]
                    gate *= (xi == xj) if kind == "cat" else (xi + xj == 2)
                dd = (kb[:, -1][:, None] - kb[:, -1][None, :]) if cont else np.zeros((nb, nb))
                ph, dph = phi_and_dphi(dd)
                got[js] = (Gb * gate * ph).sum()
                if cont:
                    got[jl] = (Gb * gate * s * dph).sum()
    err = float((got - ref).abs().max() / ref.abs().max())
    print("autograd", ref.numpy())
    print("binned  ", got.numpy())
    print(f"max rel err {err:.3e}")
    assert err < 1e-10


if __name__ == "__main__":
    main()
