"""The N x N factor / solve entry points (potrf.hip: lvae_potrf_*, lvae_trsm_*, lvae_potrs_*) against the
oracle's LAPACK restatement of the reference's calls (elbo_functions.py:26-29: torch.cholesky,
torch.cholesky_solve, 2 sum log diag L), through lvae_amd.linalg.

Tolerances: fp64 paths 1e-11 relative to the result's max (LAPACK-grade backward error at cond <= 1e4);
the fp32 potrf is the exact KL's f16 3-product-split factorisation, ~2^-22 of each 256-block's max per
product: 2e-5 of max |L|; fp32 solves compute in fp64 from fp32 operands: 1e-5 of the result's max.
"""
import numpy as np
import pytest
import torch

from oracle import lvae_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
CFG = dict(cat_kernel=[2], bin_kernel=[], sqexp_kernel=[0],
           cat_int_kernel=[{'cont_covariate': 0, 'cat_covariate': 2},
                           {'cont_covariate': 0, 'cat_covariate': 3},
                           {'cont_covariate': 1, 'cat_covariate': 4}],
           bin_int_kernel=[], covariate_missing_val=[])


def rel(a, b):
    a = a.detach().cpu().double()
    b = b.detach().cpu().double()
    return float((a - b).abs().max() / max(b.abs().max(), 1e-300))


def spd(L, n, seed, cond=1e3):
    g = torch.Generator().manual_seed(seed)
    Q, _ = torch.linalg.qr(torch.randn(L, n, n, generator=g, dtype=torch.float64))
    ev = torch.logspace(0, np.log10(cond), n, dtype=torch.float64)
    return (Q * ev) @ Q.transpose(-1, -2)


def health_mnist_K(P, L, seed):
    """the exact KL's K = Gram + noise I on Health-MNIST covariates (the C2 shape at P = 64, L = 8)"""
    from lvae_amd.data import health_mnist_covariates
    X = torch.tensor(health_mnist_covariates(P, 16, seed=seed))
    spec = O.spec_full(**CFG)
    rng = np.random.default_rng(seed)
    Ks = []
    for _ in range(L):
        params = torch.tensor(rng.uniform(0.5, 3.0, O.n_params(spec)))
        Ks.append(O.gram(spec, params, X, X) + torch.eye(X.shape[0], dtype=torch.float64))
    return torch.stack(Ks)


@pytest.mark.parametrize("n,L", [(1, 2), (63, 3), (64, 1), (65, 2), (200, 3), (1024, 2)])
def test_potrf_f64_vs_oracle(hip, n, L):
    import lvae_amd.linalg as LA
    A = spd(L, n, seed=n)
    Lr, ldr = O.potrf(A)
    Lg, ldg, info = LA.cholesky_ex(A.to(DEV))
    assert int(info.abs().sum()) == 0
    assert rel(Lg, Lr) < 1e-11
    assert rel(ldg, ldr) < 1e-12
    assert torch.equal(torch.triu(Lg.cpu(), 1), torch.zeros_like(Lr))  # torch.cholesky's zero upper part


def test_potrf_f64_many_workgroups(hip):
    """n = 2048, L = 16: the first pass launches 31 x 16 panel workgroups, more than are resident at once
    (the former fused diagonal + panel launch raced on A_kk exactly when its workgroups did not all
    start together; the tests above all fit in one wave of workgroups)."""
    import lvae_amd.linalg as LA
    n, L = 2048, 16
    g = torch.Generator().manual_seed(5)
    B = torch.randn(L, n, n, generator=g, dtype=torch.float64)
    A = B @ B.transpose(-1, -2) / n + torch.eye(n, dtype=torch.float64)
    Lr, ldr = O.potrf(A)
    Lg, ldg, info = LA.cholesky_ex(A.to(DEV))
    assert int(info.abs().sum()) == 0
    assert rel(Lg, Lr) < 1e-11
    assert rel(ldg, ldr) < 1e-12


def test_potrf_f64_in_place(hip):
    """Lout == A: the factor overwrites A's lower triangle (upper zeroed)."""
    n, L = 300, 2
    A = spd(L, n, seed=3)
    Ad = A.to(DEV).contiguous()
    ld = torch.empty(L, dtype=torch.float64, device=DEV)
    info = torch.empty(L, dtype=torch.int32, device=DEV)
    from lvae_amd import _lib
    rc = hip.lvae_potrf_f64(n, L, _lib.ptr(Ad), n, n * n, _lib.ptr(Ad), n, n * n, _lib.ptr(ld), _lib.ptr(info),
                            _lib.stream_ptr())
    assert rc == 0
    assert rel(Ad, O.potrf(A)[0]) < 1e-11


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_potrf_not_pd_raises(hip, dtype):
    """info = the first non-positive leading minor (LAPACK / torch.cholesky's error), per batch element."""
    import lvae_amd.linalg as LA
    n = 600
    A = spd(2, n, seed=7)
    A[1, 437, 437] = -5.0  # leading minor 438 fails (the earlier ones are untouched)
    _, _, info = LA.cholesky_ex(A.to(DEV, dtype))
    info = info.cpu()
    assert int(info[0]) == 0 and int(info[1]) == 438
    with pytest.raises(torch.linalg.LinAlgError):
        LA.cholesky(A.to(DEV, dtype))


@pytest.mark.parametrize("n,L", [(100, 2), (256, 1), (1000, 2), (1024, 3)])
def test_potrf_f32_vs_oracle(hip, n, L):
    """fp32 through the exact KL's own blocked factorisation (chol_inv.hip, f16 x3 split)."""
    import lvae_amd.linalg as LA
    A = spd(L, n, seed=n + 1, cond=1e2)
    Lr, ldr = O.potrf(A)
    Lg, ldg, info = LA.cholesky_ex(A.to(DEV, torch.float32))
    assert int(info.abs().sum()) == 0
    assert Lg.dtype == torch.float32
    assert rel(Lg, Lr) < 2e-5
    assert rel(ldg, ldr) < 1e-5
    assert torch.equal(torch.triu(Lg.cpu(), 1), torch.zeros(L, n, n, dtype=torch.float32))


def test_potrf_f32_c2_shape(hip):
    """C2 (N = 1024, L = 8): the HIP factor of the exact KL's own K against LAPACK fp64 (BASELINE configs[1])."""
    import lvae_amd.linalg as LA
    K = health_mnist_K(64, 8, seed=2)
    Lr, ldr = O.potrf(K)
    Lg, ldg, info = LA.cholesky_ex(K.to(DEV, torch.float32))
    assert int(info.abs().sum()) == 0
    assert rel(Lg, Lr) < 2e-5
    assert rel(ldg, ldr) < 1e-5
    Lg64, ldg64, info = LA.cholesky_ex(K.to(DEV))
    assert rel(Lg64, Lr) < 1e-11 and rel(ldg64, ldr) < 1e-12


@pytest.mark.parametrize("n,nrhs", [(64, 1), (65, 5), (300, 64), (1024, 100)])
def test_potrs_f64_vs_oracle(hip, n, nrhs):
    import lvae_amd.linalg as LA
    L = 2
    A = spd(L, n, seed=nrhs)
    g = torch.Generator().manual_seed(nrhs)
    B = torch.randn(L, n, nrhs, generator=g, dtype=torch.float64)
    Lr, _ = O.potrf(A)
    Xr = O.potrs(B, Lr)
    Xg = LA.cholesky_solve(B.to(DEV), Lr.to(DEV))
    assert rel(Xg, Xr) < 1e-11
    # triangular solves, both orientations
    Yr = torch.linalg.solve_triangular(Lr, B, upper=False)
    assert rel(LA.solve_triangular(Lr.to(DEV), B.to(DEV)), Yr) < 1e-11
    Zr = torch.linalg.solve_triangular(Lr.transpose(-1, -2), B, upper=True)
    assert rel(LA.solve_triangular(Lr.to(DEV), B.to(DEV), transpose=True), Zr) < 1e-11


def test_potrs_f32_vs_oracle(hip):
    import lvae_amd.linalg as LA
    n, nrhs, L = 500, 7, 2
    A = spd(L, n, seed=11, cond=1e2)
    Lr, _ = O.potrf(A)
    B = torch.randn(L, n, nrhs, generator=torch.Generator().manual_seed(1), dtype=torch.float64)
    Xr = O.potrs(B.float().double(), Lr.float().double())
    Xg = LA.cholesky_solve(B.to(DEV, torch.float32), Lr.to(DEV, torch.float32))
    assert Xg.dtype == torch.float32
    assert rel(Xg, Xr) < 1e-5


def test_kl_closed_through_linalg_matches_oracle(hip):
    """The reference's KL_closed (elbo_functions.py:21-33) written with lvae_amd.linalg in place of
    torch.cholesky / cholesky_solve, in fp64, against the oracle's KL at 1e-11."""
    import lvae_amd.linalg as LA
    P, L = 16, 3
    K = health_mnist_K(P, L, seed=4)
    n = K.shape[-1]
    g = torch.Generator().manual_seed(4)
    mu = torch.randn(L, n, generator=g, dtype=torch.float64)
    lv = 0.1 * torch.randn(L, n, generator=g, dtype=torch.float64)
    Kd = K.to(DEV)
    LK1, logdet11 = LA.cholesky_logdet(Kd)
    iK1 = LA.cholesky_solve(torch.eye(n, dtype=torch.float64, device=DEV).expand(L, n, n), LK1)
    mud, v1 = mu.to(DEV), torch.exp(lv).to(DEV)
    qf1 = (mud * (iK1 @ mud.unsqueeze(-1)).squeeze(-1)).sum(-1)
    tr1 = (v1 * torch.diagonal(iK1, dim1=-2, dim2=-1)).sum(-1)
    kld = 0.5 * (tr1 + qf1 - n + logdet11 - lv.to(DEV).sum(-1))
    Lr, ldr = O.potrf(K)
    iKr = O.potrs(torch.eye(n, dtype=torch.float64).expand(L, n, n), Lr)
    ref = 0.5 * ((torch.exp(lv) * torch.diagonal(iKr, dim1=-2, dim2=-1)).sum(-1)
                 + (mu * (iKr @ mu.unsqueeze(-1)).squeeze(-1)).sum(-1) - n + ldr - lv.sum(-1))
    assert rel(kld, ref) < 1e-11
