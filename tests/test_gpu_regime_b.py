"""HIP exact-KL path (Regime B) against the oracle and the reference's golden vectors.

Tolerance (north star): ELBO / KL terms within 1e-4 relative in fp32; gradients within 1e-4
relative to their max-norm.  Everything runs through the C ABI (liblvae_hip.so).
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import lvae_oracle as O

pytestmark = pytest.mark.gpu

CFG = dict(cat_kernel=[2], bin_kernel=[], sqexp_kernel=[0],
           cat_int_kernel=[{'cont_covariate': 0, 'cat_covariate': 2},
                           {'cont_covariate': 0, 'cat_covariate': 3},
                           {'cont_covariate': 1, 'cat_covariate': 4}],
           bin_int_kernel=[], covariate_missing_val=[])
DEV = "cuda"


def rel(a, b):
    a = a.detach().cpu().double().numpy() if isinstance(a, torch.Tensor) else np.asarray(a, np.float64)
    b = b.detach().cpu().double().numpy() if isinstance(b, torch.Tensor) else np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def set_raw(module, raw_rows):
    """raw_rows: [L, P] raw parameters in named_parameters order."""
    ps = [p for _, p in module.named_parameters()]
    with torch.no_grad():
        for j, p in enumerate(ps):
            p.copy_(torch.as_tensor(raw_rows[:, j], dtype=p.dtype))


@pytest.mark.parametrize("name", ["kl_closed_n64.npz", "kl_closed_n256.npz", "kl_closed_n96_noise.npz"])
def test_kl_closed_golden(hip, name):
    import lvae_amd as la
    g = golden(name)
    L = int(g["L"])
    k = la.generate_kernel(**CFG, latent_dim=L).double()
    set_raw(k, g["raw"])
    k = k.to(DEV)
    lik = la.GaussianLikelihood(L, noise=float(g["noise"][0])).to(DEV)
    X = torch.tensor(g["X"], device=DEV)
    mu = torch.tensor(g["mu"], device=DEV, requires_grad=True)
    lv = torch.tensor(g["logv"], device=DEV, requires_grad=True)
    kl = la.KL_closed_batched(k, X, lik, mu, lv)
    kl.sum().backward()
    assert rel(kl, g["kl"]) < 1e-4
    assert rel(mu.grad, g["dmu"]) < 1e-4
    assert rel(lv.grad, g["dlogv"]) < 1e-4
    draw = torch.stack([p.grad for _, p in k.named_parameters()], 1)
    assert rel(draw, g["draw"]) < 1e-4


def test_kl_closed_single_dim_api(hip):
    """Drop-in signature KL_closed(covar_module, train_x, likelihoods, data, mu, log_var)."""
    import lvae_amd as la
    g = golden("kl_closed_n64.npz")
    k = la.generate_kernel(**CFG).double()
    set_raw(k, g["raw"][:1])
    k = k.to(DEV)
    lik = la.GaussianLikelihood(1, noise=1.0).to(DEV)
    X = torch.tensor(g["X"], device=DEV)
    kl = la.KL_closed(k, X, lik, X, torch.tensor(g["mu"][:, 0], device=DEV), torch.tensor(g["logv"][:, 0], device=DEV))
    assert abs(kl.item() - g["kl"][0]) < 1e-4 * abs(g["kl"][0])


@pytest.mark.parametrize("P,L", [(64, 2), (13, 3), (9, 1)])  # N = 1024, 208 (padded), 144 (padded)
def test_kl_closed_vs_oracle(hip, P, L):
    import lvae_amd as la
    from lvae_amd.data import health_mnist_covariates
    T = 16
    X = torch.tensor(health_mnist_covariates(P, T, seed=P))
    gen = torch.Generator().manual_seed(P)
    mu = torch.randn(P * T, L, generator=gen, dtype=torch.float64)
    lv = 0.1 * torch.randn(P * T, L, generator=gen, dtype=torch.float64)
    k = la.generate_kernel(**CFG, latent_dim=L).double()
    rng = np.random.default_rng(P)
    raw = np.stack([np.log(rng.uniform(0.3, 1.5, L)) if "scale" in n else np.log(rng.uniform(1, 4, L))
                    for n, _ in k.named_parameters()], 1)
    set_raw(k, raw)
    kd = k.to(DEV)
    lik = la.GaussianLikelihood(L, noise=1.0).to(DEV)
    mu_d, lv_d = mu.to(DEV).requires_grad_(), lv.to(DEV).requires_grad_()
    kl = la.KL_closed_batched(kd, X.to(DEV), lik, mu_d, lv_d)
    (kl * torch.arange(1, L + 1, device=DEV)).sum().backward()
    spec = O.spec_full(**CFG)
    for l in range(L):
        r = torch.tensor(raw[l], requires_grad=True)
        m_, v_ = mu[:, l].clone().requires_grad_(), lv[:, l].clone().requires_grad_()
        ref = O.kl_closed(spec, O.constrain(r), X, 1.0, m_, v_)
        ((l + 1) * ref).backward()
        assert rel(kl[l], ref) < 1e-4
        assert rel(mu_d.grad[:, l], m_.grad) < 1e-4
        assert rel(lv_d.grad[:, l], v_.grad) < 1e-4
        draw = torch.stack([p.grad[l] for _, p in kd.named_parameters()])
        assert rel(draw, r.grad) < 1e-4


def test_potrf_potri(hip):
    """Blocked MFMA block-LDL^T + inverse on random SPD matrices vs fp64 torch on the host:
    Lt Dt Lt^T reconstructs A, log|A| and A^-1 match (np = 384: three 128-blocks)."""
    import lvae_amd as la
    lib = hip
    L, n, nb = 2, 384, 128
    gen = torch.Generator().manual_seed(1)
    Xm = torch.randn(L, n, n, generator=gen, dtype=torch.float64) / n ** 0.5
    A = Xm @ Xm.transpose(1, 2) + torch.eye(n, dtype=torch.float64)
    Ad = torch.tril(A).float().to(DEV).contiguous()  # only the lower triangle is read
    W = torch.zeros_like(Ad)
    Ai = torch.zeros_like(Ad)
    logdet = torch.zeros(L, dtype=torch.float64, device=DEV)
    info = torch.zeros(L, dtype=torch.int32, device=DEV)
    P = la._lib
    P.check(lib.lvae_potrf_f32(n, L, P.ptr(Ad), P.ptr(W), P.ptr(logdet), P.ptr(info), P.stream_ptr()), "potrf")
    torch.cuda.synchronize()
    Wc = W.cpu().double()
    Lt = torch.eye(n, dtype=torch.float64).repeat(L, 1, 1)
    Dt = torch.zeros(L, n, n, dtype=torch.float64)
    for I in range(n // nb):
        sl = slice(I * nb, (I + 1) * nb)
        Dt[:, sl, sl] = torch.linalg.inv(Wc[:, sl, sl])
        for J in range(I):
            sj = slice(J * nb, (J + 1) * nb)
            Lt[:, sl, sj] = Wc[:, sl, sj]
    assert int(info.abs().sum()) == 0
    assert rel(Lt @ Dt @ Lt.transpose(1, 2), A) < 1e-5
    assert rel(logdet.cpu(), torch.logdet(A)) < 1e-5
    P.check(lib.lvae_potri_f32(n, L, P.ptr(Ad), P.ptr(W), P.ptr(Ai), P.stream_ptr()), "potri")
    torch.cuda.synchronize()
    assert rel(Ai.cpu(), torch.linalg.inv(A)) < 1e-4


def test_not_positive_definite_raises(hip):
    import lvae_amd as la
    from lvae_amd.data import health_mnist_covariates
    X = torch.tensor(health_mnist_covariates(4, 16), device=DEV)
    k = la.generate_kernel(**CFG, latent_dim=1).double().to(DEV)
    lik = la.GaussianLikelihood(1, noise=1.0).to(DEV)
    with torch.no_grad():
        lik._log_noise.fill_(-30.0)       # noise ~ 1e-7: rank-deficient Gram -> fp32 pivot failure
        for _, p in k.named_parameters():
            p.fill_(5.0)
    mu = torch.zeros(64, 1, dtype=torch.float64, device=DEV)
    with pytest.raises(torch.linalg.LinAlgError):
        la.KL_closed_batched(k, X, lik, mu, mu.clone())


def test_gram_batched_semantics(hip):
    """covar(x1, x2).evaluate() shapes/values of the Hensman call sites (elbo_functions.py:171-174)."""
    import lvae_amd as la
    L, P_b, T, M = 3, 2, 16, 20
    from lvae_amd.data import health_mnist_covariates
    X = torch.tensor(health_mnist_covariates(P_b, T, 3))
    Z = torch.stack([X[:M]] * L)
    k0, k1 = la.generate_kernel_batched(L, **CFG, id_covariate=2)
    k0 = k0.double()
    rng = np.random.default_rng(0)
    set_raw(k0, np.log(rng.uniform(0.5, 3.0, (L, len(list(k0.parameters()))))))
    s0, s1 = O.spec_split(**CFG, id_covariate=2)
    _, p0 = la.kernel_spec_and_params(k0)
    p0c = p0.detach()
    k0 = k0.to(DEV)
    xst = X.reshape(P_b, T, 6)
    sx = torch.stack([xst] * L, 1)
    for a, b, shape in [(X, Z, (L, P_b * T, M)), (Z, Z, (L, M, M)), (sx, sx, (P_b, L, T, T))]:
        got = k0(a.to(DEV), b.to(DEV)).evaluate()
        ref = O.gram(s0, p0c, a, b)
        assert tuple(got.shape) == shape
        assert rel(got, ref) < 1e-13
    # adjoint
    G = torch.randn(L, P_b * T, M, dtype=torch.float64)
    k0.zero_grad()
    (k0(X.to(DEV), Z.to(DEV)).evaluate() * G.to(DEV)).sum().backward()
    raw = torch.stack([p.detach().cpu() for _, p in k0.named_parameters()], 1).requires_grad_()
    (O.gram(s0, O.constrain(raw), X, Z) * G).sum().backward()
    got = torch.stack([p.grad.cpu() for _, p in k0.named_parameters()], 1)
    assert rel(got, raw.grad) < 1e-12


@pytest.mark.parametrize("n", [128, 384, 640, 1024])
def test_spd_inverse_recursive(hip, n):
    """Recursive Schur-complement inverse (the Regime B path) vs fp64 torch: A^-1 and log|A|; odd
    tile counts exercise the uneven split.  The upper triangle of A is never read."""
    import lvae_amd as la
    L = 2
    gen = torch.Generator().manual_seed(n)
    Xm = torch.randn(L, n, n, generator=gen, dtype=torch.float64) / n ** 0.5
    A = Xm @ Xm.transpose(1, 2) + torch.eye(n, dtype=torch.float64)
    Ad = (torch.tril(A) + 7.0 * torch.triu(torch.ones(n, n, dtype=torch.float64), 1)).float().to(DEV).contiguous()
    W = torch.zeros_like(Ad)
    Ai = torch.zeros_like(Ad)
    logdet = torch.zeros(L, dtype=torch.float64, device=DEV)
    info = torch.zeros(L, dtype=torch.int32, device=DEV)
    P = la._lib
    P.check(hip.lvae_spd_inverse_f32(n, L, P.ptr(Ad), P.ptr(W), P.ptr(Ai), P.ptr(logdet), P.ptr(info),
                                     P.stream_ptr()), "spd_inverse")
    torch.cuda.synchronize()
    assert int(info.abs().sum()) == 0
    assert rel(Ai.cpu(), torch.linalg.inv(A)) < 1e-5
    assert rel(logdet.cpu(), torch.logdet(A)) < 1e-6


@pytest.mark.parametrize("n,L", [(256, 3), (512, 2), (768, 2), (1280, 2), (4096, 1)])
def test_spd_sweep(hip, n, L):
    """Block symmetric sweep (the default Regime B inverse) vs fp64 torch: A^-1 (both triangles
    written) and log|A|.  nt = n / 256 = 1, 2, 3, 5, 16 pivot blocks; the upper triangle of A is
    garbage (never read) and A's scale is uneven (diagonal 0.5 .. 50) as the unit-diagonal pivot
    scaling must handle."""
    import lvae_amd as la
    gen = torch.Generator().manual_seed(n + L)
    Xm = torch.randn(L, n, n, generator=gen, dtype=torch.float64) / n ** 0.5
    A = Xm @ Xm.transpose(1, 2) + torch.eye(n, dtype=torch.float64)
    s = torch.exp(torch.rand(L, n, 1, generator=gen, dtype=torch.float64) * 4.6 - 0.7) ** 0.5
    A = s * A * s.transpose(1, 2)
    Ad = (torch.tril(A) + 7.0 * torch.triu(torch.ones(n, n, dtype=torch.float64), 1)).float().to(DEV).contiguous()
    scr = torch.full((hip.lvae_spd_sweep_scratch_size(n, L) // 4,), float("nan"), device=DEV)
    Ai = torch.full_like(Ad, float("nan"))
    logdet = torch.zeros(L, dtype=torch.float64, device=DEV)
    info = torch.zeros(L, dtype=torch.int32, device=DEV)
    P = la._lib
    P.check(hip.lvae_spd_sweep_f32(n, L, P.ptr(Ad), P.ptr(scr), P.ptr(Ai), P.ptr(logdet), P.ptr(info),
                                   P.stream_ptr()), "spd_sweep")
    torch.cuda.synchronize()
    assert int(info.abs().sum()) == 0
    ref = torch.linalg.inv(A)
    got = Ai.cpu().double()
    assert torch.isfinite(got).all()
    err = rel(got, ref)
    print(f"spd_sweep n={n} L={L}: rel err {err:.3e}")
    assert err < 1e-4
    assert rel(logdet.cpu(), torch.logdet(A)) < 1e-6


def test_spd_sweep_not_pd(hip):
    """A non-SPD pivot is reported LAPACK-style with the global column (block 1, local column 10)."""
    import lvae_amd as la
    n, L = 512, 2
    A = torch.eye(n, dtype=torch.float64).repeat(L, 1, 1)
    A[1, 256 + 10, 256 + 10] = -1.0
    Ad = A.float().to(DEV).contiguous()
    scr = torch.zeros(hip.lvae_spd_sweep_scratch_size(n, L) // 4, device=DEV)
    Ai = torch.zeros_like(Ad)
    logdet = torch.zeros(L, dtype=torch.float64, device=DEV)
    info = torch.zeros(L, dtype=torch.int32, device=DEV)
    P = la._lib
    P.check(hip.lvae_spd_sweep_f32(n, L, P.ptr(Ad), P.ptr(scr), P.ptr(Ai), P.ptr(logdet), P.ptr(info),
                                   P.stream_ptr()), "spd_sweep")
    torch.cuda.synchronize()
    assert info.cpu().tolist() == [0, 256 + 10 + 1]
    assert abs(float(logdet[0])) < 1e-6


def test_kl_closed_vs_oracle_full_size(hip):
    """The headline size N = 4096 (P = 256 subjects x T = 16), one latent dim, vs the fp64 oracle
    (north-star tolerance 1e-4 on the KL and every gradient)."""
    import lvae_amd as la
    from lvae_amd.data import health_mnist_covariates
    P, T, L = 256, 16, 1
    X = torch.tensor(health_mnist_covariates(P, T, seed=5))
    gen = torch.Generator().manual_seed(5)
    mu = torch.randn(P * T, L, generator=gen, dtype=torch.float64)
    lv = 0.1 * torch.randn(P * T, L, generator=gen, dtype=torch.float64)
    k = la.generate_kernel(**CFG, latent_dim=L).double()
    raw = torch.stack([p.detach() for _, p in k.named_parameters()], 1)
    kd = k.to(DEV)
    lik = la.GaussianLikelihood(L, noise=1.0).to(DEV)
    mu_d, lv_d = mu.to(DEV).requires_grad_(), lv.to(DEV).requires_grad_()
    kl = la.KL_closed_batched(kd, X.to(DEV), lik, mu_d, lv_d)
    kl.sum().backward()
    r = raw[0].clone().requires_grad_()
    m_, v_ = mu[:, 0].clone().requires_grad_(), lv[:, 0].clone().requires_grad_()
    ref = O.kl_closed(O.spec_full(**CFG), O.constrain(r), X, 1.0, m_, v_)
    ref.backward()
    assert rel(kl[0], ref) < 1e-4
    assert rel(mu_d.grad[:, 0], m_.grad) < 1e-4
    assert rel(lv_d.grad[:, 0], v_.grad) < 1e-4
    assert rel(torch.stack([p.grad[0] for _, p in kd.named_parameters()]), r.grad) < 1e-4


def test_relu_maxpool2_matches_torch(hip):
    """Fused encoder relu + 2x2 max pool vs torch (values bit-exact, gradient routing identical)."""
    from lvae_amd.vae import relu_maxpool2
    import torch.nn.functional as F
    gen = torch.Generator(device=DEV).manual_seed(0)
    x = torch.randn(7, 16, 36, 36, device=DEV, generator=gen)
    x[0, 0, :4, :4] = -1.0       # all-negative windows
    x[1, 1, 2:4, 2:4] = 0.5      # ties: the first maximum in scan order takes the gradient
    xa = x.clone().requires_grad_()
    xb = x.clone().requires_grad_()
    ya = relu_maxpool2(xa)
    yb = F.max_pool2d(F.relu(xb), 2, 2)
    assert torch.equal(ya, yb)
    g = torch.randn(ya.shape, device=DEV, generator=gen)
    ya.backward(g)
    yb.backward(g)
    assert torch.equal(xa.grad, xb.grad)
