"""Exact-KL forward + backward alone (no ConvVAE beside it) at the headline shape, for kernel-level
timing of the Gram fill / adjoint under rocprofv3 --kernel-trace --stats.
usage: python scripts/gram_micro.py [iters]"""
import os
import sys
import torch
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "longitudinal-vae_amd"))
sys.path.insert(0, ROOT)
import lvae_amd as la  # noqa: E402
from lvae_amd.data import health_mnist_covariates  # noqa: E402
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda:0")
cfg = dict(cat_kernel=[2], bin_kernel=[], sqexp_kernel=[0],
           cat_int_kernel=[{'cont_covariate': 0, 'cat_covariate': 2}, {'cont_covariate': 0, 'cat_covariate': 3},
                           {'cont_covariate': 1, 'cat_covariate': 4}], bin_int_kernel=[], covariate_missing_val=[])
P, T, L = 256, 16, 16
X = torch.tensor(health_mnist_covariates(P, T, seed=0)).to(dev)
g = torch.Generator().manual_seed(0)
mu = torch.randn(P * T, L, generator=g, dtype=torch.float64).to(dev).requires_grad_()
lv = (0.1 * torch.randn(P * T, L, generator=g, dtype=torch.float64)).to(dev).requires_grad_()
k = la.generate_kernel(**cfg, latent_dim=L).to(dev)
lik = la.GaussianLikelihood(L, noise=1.0).to(dev)
for it in range(iters):
    for p in list(k.parameters()) + list(lik.parameters()):
        p.grad = None
    kl = la.KL_closed_batched(k, X, lik, mu, lv)
    kl.sum().backward()
torch.cuda.synchronize()
print(la._lib.LIB_PATH, [round(v, 4) for v in kl[:3].tolist()], float(mu.grad.abs().sum()))
# the hyper-parameter gradients of the last iteration, in full (old / new library bit-identity check)
print("hyper-grads", [repr(float(p.grad.double().sum())) for p in list(k.parameters()) + list(lik.parameters())
                      if p.grad is not None])
