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


@pytest.mark.parametrize("P,L", [(64, 2), (64, 8), (13, 3), (9, 1)])  # N = 1024 (64-8: C2), 208 / 144 (padded)
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
    from lvae_amd.elbo import kl_closed_refine_log
    with kl_closed_refine_log() as rlog:
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


def test_kl_closed_prefactor_matches(hip):
    """KL_closed_batched with the Gram + inverse launched ahead on another stream
    (kl_closed_prefactor -> lvae_kl_closed_factor_f32, then lvae_kl_closed_reduce_f32) equals the
    one-call forward bit for bit, values and every gradient."""
    import lvae_amd as la
    from lvae_amd.data import health_mnist_covariates
    P, T, L = 40, 16, 3
    X = torch.tensor(health_mnist_covariates(P, T, seed=5), device=DEV)
    k = la.generate_kernel(**CFG, latent_dim=L).double()
    set_raw(k, _random_hypers(k, L, np.random.default_rng(5)))
    k = k.to(DEV)
    lik = la.GaussianLikelihood(L, noise=1.0).to(DEV)
    gen = torch.Generator().manual_seed(5)
    mu0 = torch.randn(P * T, L, generator=gen, dtype=torch.float64).to(DEV)
    lv0 = (0.1 * torch.randn(P * T, L, generator=gen, dtype=torch.float64)).to(DEV)
    out = []
    for pre in (False, True):
        k.zero_grad()
        mu, lv = mu0.clone().requires_grad_(), lv0.clone().requires_grad_()
        f = la.kl_closed_prefactor(k, X, lik, L, torch.cuda.Stream()) if pre else None
        kl = la.KL_closed_batched(k, X, lik, mu, lv, factor=f)
        (kl * torch.arange(1, L + 1, device=DEV)).sum().backward()
        out.append([kl.detach(), mu.grad, lv.grad] + [p.grad.clone() for _, p in k.named_parameters()])
    for a, b in zip(*out):
        assert torch.equal(a, b)


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


# (the rounds 1-2 block sweep, spd_sweep.hip, is retired and no longer built: csrc/retired/)
INV_KINDS = ["chol"]


def _spd_inverse(hip, kind, n, L, Ad):
    """A^-1 (both triangles), log|A|, info of the [L, n, n] fp32 lower triangles Ad through the C ABI:
    kind 'chol' (blocked Cholesky + trtri + lauum, chol_inv.hip, the KL's inverse)."""
    import lvae_amd as la
    P = la._lib
    size, fn = hip.lvae_spd_inv_chol_scratch_size, hip.lvae_spd_inv_chol_f32
    scr = torch.full((size(n, L) // 4,), float("nan"), device=DEV)
    Ai = torch.full_like(Ad, float("nan"))
    logdet = torch.zeros(L, dtype=torch.float64, device=DEV)
    info = torch.zeros(L, dtype=torch.int32, device=DEV)
    P.check(fn(n, L, P.ptr(Ad), P.ptr(scr), P.ptr(Ai), P.ptr(logdet), P.ptr(info), P.stream_ptr()), kind)
    torch.cuda.synchronize()
    return Ai, logdet, info


@pytest.mark.parametrize("kind", INV_KINDS)
@pytest.mark.parametrize("n,L", [(256, 3), (512, 2), (768, 2), (1280, 2), (4096, 1), (256, 9), (512, 9), (768, 10),
                                 (1280, 9)])
def test_spd_inverse(hip, kind, n, L):
    """The two blocked SPD inverses vs fp64 torch: A^-1 (both triangles written) and log|A|.
    nt = n / 256 = 1, 2, 3, 5, 16 blocks (3 and 5: trtri's recursive doubling with a ragged last
    group), under both host schedules (L <= 8: pivots back to back, each updating its own block; L > 8:
    the whole chain on the side stream); the upper triangle of A is garbage (never read) and A's scale
    is uneven (diagonal 0.5 .. 50)."""
    gen = torch.Generator().manual_seed(n + L)
    Xm = torch.randn(L, n, n, generator=gen, dtype=torch.float64) / n ** 0.5
    A = Xm @ Xm.transpose(1, 2) + torch.eye(n, dtype=torch.float64)
    s = torch.exp(torch.rand(L, n, 1, generator=gen, dtype=torch.float64) * 4.6 - 0.7) ** 0.5
    A = s * A * s.transpose(1, 2)
    Ad = (torch.tril(A) + 7.0 * torch.triu(torch.ones(n, n, dtype=torch.float64), 1)).float().to(DEV).contiguous()
    Ai, logdet, info = _spd_inverse(hip, kind, n, L, Ad)
    assert int(info.abs().sum()) == 0
    ref = torch.linalg.inv(A)
    got = Ai.cpu().double()
    assert torch.isfinite(got).all()
    err = rel(got, ref)
    print(f"{kind} n={n} L={L}: rel err {err:.3e}")
    assert err < 1e-4
    assert rel(logdet.cpu(), torch.logdet(A)) < 1e-6


@pytest.mark.parametrize("kind", INV_KINDS)
def test_spd_inverse_not_pd(hip, kind):
    """A non-SPD pivot is reported LAPACK-style with the global column (block 1, local column 10)."""
    n, L = 512, 2
    A = torch.eye(n, dtype=torch.float64).repeat(L, 1, 1)
    A[1, 256 + 10, 256 + 10] = -1.0
    Ad = A.float().to(DEV).contiguous()
    _, logdet, info = _spd_inverse(hip, kind, n, L, Ad)
    assert info.cpu().tolist() == [0, 256 + 10 + 1]
    assert abs(float(logdet[0])) < 1e-6


def test_spd_inverse_ill_conditioned(hip):
    """Why the KL uses the Cholesky form: on exact-KL covariances with small likelihood noise (the
    sample config's kernel, N = 1024, noise 1e-3 / 1e-4: cond(K) 1e4 .. 1e5) the blocked Cholesky
    inverse keeps |I - K X| at fp32-Cholesky level (LAPACK spotri: ~cond 2^-24), while the block sweep
    (Gauss-Jordan) loses ~two more digits.  Errors printed against cond."""
    import lvae_amd as la
    from lvae_amd.data import health_mnist_covariates
    P, T, L = 64, 16, 2
    X = torch.tensor(health_mnist_covariates(P, T, seed=3))
    spec = O.spec_full(**CFG)
    k = la.generate_kernel(**CFG, latent_dim=L)
    for noise in (1e-3, 1e-4):
        raw = _random_hypers(k, L, np.random.default_rng(int(1 / noise)))
        K = torch.stack([O.gram(spec, O.constrain(torch.tensor(raw[l])), X, X) for l in range(L)])
        K = K + noise * torch.eye(P * T, dtype=torch.float64)
        res = {}
        for kind in INV_KINDS:
            Ai, logdet, info = _spd_inverse(hip, kind, P * T, L, K.float().to(DEV).contiguous())
            assert int(info.abs().sum()) == 0
            Xi = Ai.cpu().double()
            res[kind] = [float(torch.linalg.matrix_norm(torch.eye(P * T, dtype=torch.float64) - K[l] @ Xi[l], 2))
                         for l in range(L)]
            ld_err = float((logdet.cpu() - torch.logdet(K)).abs().max())
            print(f"noise {noise} {kind}: |I - K X|_2 per dim {res[kind]}, |dlog|K|| {ld_err:.2e}")
        conds = [float(torch.linalg.cond(K[l])) for l in range(L)]
        for l in range(L):
            assert res["chol"][l] < max(1e-3, 2 * conds[l] * 2.0 ** -22), (noise, l, conds[l])
            if "sweep" in res:
                assert res["chol"][l] < 0.2 * res["sweep"][l] or res["sweep"][l] < 1e-2


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
    from lvae_amd.elbo import kl_closed_refine_log
    with kl_closed_refine_log() as rlog:
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


@pytest.mark.parametrize("n,c,hw", [(5, 16, 36), (37, 32, 18)])
def test_relu_maxpool2_bias_kernels_match_torch(hip, n, c, hw):
    """The bias-folded relu + pool kernels on a given conv output y0 vs torch's y0 + b -> relu ->
    max_pool2d: pooled values and the routed gradient bit-exact, the bias gradient to fp32
    summation order."""
    import torch.nn.functional as F
    from lvae_amd import _lib
    gen = torch.Generator(device=DEV).manual_seed(1)
    y0 = torch.randn(n, c, hw, hw, device=DEV, generator=gen)
    y0[0, 0, :4, :4] = -5.0      # all-negative windows
    y0[1, 1, 2:4, 2:4] = 0.25    # ties
    b = torch.randn(c, device=DEV, generator=gen)
    y = torch.empty(n, c, hw // 2, hw // 2, device=DEV)
    idx = torch.empty(n, c, hw // 2, hw // 2, dtype=torch.uint8, device=DEV)
    _lib.check(hip.lvae_relu_maxpool2_bias_fwd_f32(_lib.ptr(y0), _lib.ptr(b), n, c, hw, hw, _lib.ptr(y), _lib.ptr(idx),
                                                    _lib.stream_ptr()), "fwd")
    yr = y0.clone().requires_grad_()
    br = b.clone().requires_grad_()
    ref = F.max_pool2d(F.relu(yr + br.view(1, -1, 1, 1)), 2, 2)
    assert torch.equal(y, ref)
    g = torch.randn(y.shape, device=DEV, generator=gen)
    ref.backward(g)
    gx = torch.empty_like(y0)
    db = torch.empty(c, device=DEV)
    ws = torch.empty(hip.lvae_relu_maxpool2_bias_workspace_size(n, c) // 4 + 1, device=DEV)
    _lib.check(hip.lvae_relu_maxpool2_bias_bwd_f32(_lib.ptr(g), _lib.ptr(y), _lib.ptr(idx), n, c, hw, hw, _lib.ptr(gx),
                                                    _lib.ptr(db), _lib.ptr(ws), _lib.stream_ptr()), "bwd")
    assert torch.equal(gx, yr.grad)
    assert float((db - br.grad).abs().max() / br.grad.abs().max()) < 1e-5


@pytest.mark.parametrize("n,cin,cout,hw,xgrad", [(5, 1, 16, 36, True), (37, 16, 32, 18, True), (37, 1, 16, 36, False),
                                               (3, 1, 4, 8, False), (520, 16, 32, 18, True), (600, 1, 16, 36, False),
                                               (2050, 16, 32, 18, True), (2051, 1, 16, 36, False)])
def test_conv_relu_maxpool2_bias_matches_torch(hip, n, cin, cout, hw, xgrad):
    """Encoder conv with its bias folded into the fused relu + pool pass (bias gradient from its
    backward, weight / input gradients from aten.convolution_backward; for the first conv, whose
    input needs no gradient, weight and bias gradients straight from the pooled gradient; below 512
    images the MIOpen weight gradient) vs the same conv + relu + 2x2 pool in fp64 on the GPU: values
    and input gradients to 1e-5, the weight / bias gradients (sums over n (hw/2)^2 terms of both
    signs) to 5e-5 of their max.  The fp64 reference routes each window's gradient through the argmax
    and the relu decision the HIP forward took (a window whose top two fp32 values nearly tie, or whose
    max is within fp32 rounding of 0, may go either way; at 2050 images a few of the 5e6 windows do,
    and routing them by fp64's own decisions moved the input gradient by 1e-3..2e-2 of its max); that
    the chosen values are the windows' relu-max to fp32 rounding is asserted against fp64 max_pool2d."""
    from lvae_amd import _lib
    from lvae_amd.vae import conv_relu_maxpool2
    import copy
    import torch.nn.functional as F
    gen = torch.Generator(device=DEV).manual_seed(1)
    conv = torch.nn.Conv2d(cin, cout, 3, 1, 1).to(DEV)
    conv64 = copy.deepcopy(conv).double()
    x = torch.randn(n, cin, hw, hw, device=DEV, generator=gen)
    xr = x.clone().requires_grad_(xgrad)
    y = conv_relu_maxpool2(conv, xr)
    g = torch.randn(y.shape, device=DEV, generator=gen)
    got = [y] + list(torch.autograd.grad(y, ([xr] if xgrad else []) + [conv.weight, conv.bias], g))
    # the argmax the forward chose (the same HIP kernels the module runs, called directly)
    ho = hw // 2
    y2 = torch.empty(n, cout, ho, ho, device=DEV)
    idx = torch.empty(n, cout, ho, ho, dtype=torch.uint8, device=DEV)
    w, b = conv.weight.detach().contiguous(), conv.bias.detach().contiguous()
    if cin == 1:
        rc = hip.lvae_conv1_relu_maxpool2_fwd_f32(_lib.ptr(x), _lib.ptr(w), _lib.ptr(b), n, cout, hw, hw,
                                                  _lib.ptr(y2), _lib.ptr(idx), _lib.stream_ptr())
    elif cin == 16 and hw == 18 and cout % 16 == 0:  # (the second conv's fused forward)
        rc = hip.lvae_conv3x3_relu_maxpool2_fwd_f32(_lib.ptr(x), _lib.ptr(w), _lib.ptr(b), n, cin, cout, hw, hw,
                                                    _lib.ptr(y2), _lib.ptr(idx), _lib.stream_ptr())
    else:
        y0 = F.conv2d(x, w, None, 1, 1).contiguous()
        rc = hip.lvae_relu_maxpool2_bias_fwd_f32(_lib.ptr(y0), _lib.ptr(b), n, cout, hw, hw, _lib.ptr(y2),
                                                 _lib.ptr(idx), _lib.stream_ptr())
    assert rc == 0 and torch.equal(y2, y.detach())
    x64 = x.double().requires_grad_(xgrad)
    z64 = conv64(x64)
    win = z64.view(n, cout, ho, 2, ho, 2).permute(0, 1, 2, 4, 3, 5).reshape(n, cout, ho, ho, 4)
    # relu at the HIP forward's decision too (a pre-activation within fp32 rounding of 0 may fall on
    # either side)
    y64 = win.gather(-1, idx.long().unsqueeze(-1)).squeeze(-1) * (y.detach() > 0).double()  # k = 2 dy + dx
    assert rel(y64, F.max_pool2d(F.relu(z64), 2, 2)) < 1e-5
    ref = [y64] + list(torch.autograd.grad(y64, ([x64] if xgrad else []) + [conv64.weight, conv64.bias], g.double()))
    tols = [1e-5] + ([1e-5] if xgrad else []) + [5e-5, 5e-5]
    errs = [rel(a, r) for a, r in zip(got, ref)]
    assert all(e < tol for e, tol in zip(errs, tols)), errs


@pytest.mark.parametrize("n,c", [(1, 32), (5, 16), (2047, 32), (2050, 32), (4096, 32), (4, 48)])
def test_conv3x3_relu_maxpool2_fused_vs_fp64(hip, n, c):
    """lvae_conv3x3_relu_maxpool2_fwd_f32 (the second encoder conv + bias + relu + 2x2 pool in one pass, VAE.py:48-50)
    vs fp64 conv2d on the same inputs: y within 1e-5 of its max of the fp64 relu-max; idx the fp64 argmax wherever
    the window's top two fp64 values are apart by more than fp32 rounding (a near-tie may go either way); the
    one-image-per-block (< 2048 images) and three-images-per-block grids, ragged last blocks.  Unsupported shapes
    return -3."""
    from lvae_amd import _lib
    import torch.nn.functional as F
    gen = torch.Generator(device=DEV).manual_seed(n + c)
    cin, hw, ho = 16, 18, 9
    x = torch.randn(n, cin, hw, hw, device=DEV, generator=gen).clamp_min(0.0)  # (post-relu inputs, like the model's)
    w = torch.randn(c, cin, 3, 3, device=DEV, generator=gen) * 0.1
    b = torch.randn(c, device=DEV, generator=gen) * 0.1
    y = torch.full((n, c, ho, ho), float("nan"), device=DEV)
    idx = torch.full((n, c, ho, ho), 255, dtype=torch.uint8, device=DEV)
    rc = hip.lvae_conv3x3_relu_maxpool2_fwd_f32(_lib.ptr(x), _lib.ptr(w), _lib.ptr(b), n, cin, c, hw, hw, _lib.ptr(y),
                                                _lib.ptr(idx), _lib.stream_ptr())
    assert rc == 0
    z64 = F.conv2d(x.double(), w.double(), b.double(), padding=1)
    win = z64.view(n, c, ho, 2, ho, 2).permute(0, 1, 2, 4, 3, 5).reshape(n, c, ho, ho, 4)
    ref = F.max_pool2d(F.relu(z64), 2, 2)
    assert rel(y, ref) < 1e-5
    top2 = win.topk(2, dim=-1).values
    clear = (top2[..., 0] - top2[..., 1]) > 1e-5 * float(z64.abs().max())
    assert int(idx.max()) <= 3
    assert torch.equal(idx.long()[clear], win.argmax(-1)[clear])
    assert hip.lvae_conv3x3_relu_maxpool2_fwd_f32(_lib.ptr(x), _lib.ptr(w), _lib.ptr(b), n, 8, c, hw, hw, _lib.ptr(y),
                                                  _lib.ptr(idx), _lib.stream_ptr()) == -3
    assert hip.lvae_conv3x3_relu_maxpool2_fwd_f32(_lib.ptr(x), _lib.ptr(w), _lib.ptr(b), n, cin, 24, hw, hw,
                                                  _lib.ptr(y), _lib.ptr(idx), _lib.stream_ptr()) == -3


@pytest.mark.parametrize("n,c,hw", [(3, 4, 8), (37, 32, 18), (2, 8, 30), (513, 32, 18), (4, 20, 12)])
def test_conv3x3_pool_dgrad_vs_fp64(hip, n, c, hw):
    """lvae_conv3x3_pool_dgrad_f32 (the second encoder conv's input gradient from the pooled gradient, the
    routed gradient formed in LDS) vs fp64 conv2d backward-data of the routed gradient (routed by the same
    argmax / relu decisions), to 1e-5 of its max; ties of the window max (idx = first maximum) and
    windows with y = 0 included.  Unsupported shapes return -3 (Cin != 16) / -4 (LDS)."""
    from lvae_amd import _lib
    import torch.nn.functional as F
    gen = torch.Generator(device=DEV).manual_seed(5)
    cin, ho = 16, hw // 2
    w = torch.randn(c, cin, 3, 3, device=DEV, generator=gen)
    gy = torch.randn(n, c, ho, ho, device=DEV, generator=gen)
    y = torch.randn(n, c, ho, ho, device=DEV, generator=gen).clamp_min(0.0)  # ~half the windows relu'd off
    idx = torch.randint(0, 4, (n, c, ho, ho), device=DEV, generator=gen, dtype=torch.int32).to(torch.uint8)
    gx = torch.full((n, cin, hw, hw), float("nan"), device=DEV)
    rc = hip.lvae_conv3x3_pool_dgrad_f32(_lib.ptr(gy), _lib.ptr(y), _lib.ptr(idx), _lib.ptr(w), n, c, cin, hw, hw,
                                         _lib.ptr(gx), _lib.stream_ptr())
    assert rc == 0
    g = torch.where(y > 0, gy, torch.zeros_like(gy)).double()
    g0 = torch.zeros(n, c, ho, ho, 4, dtype=torch.float64, device=DEV)
    g0.scatter_(-1, idx.long().unsqueeze(-1), g.unsqueeze(-1))
    g0 = g0.view(n, c, ho, ho, 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(n, c, hw, hw)  # k = 2 dy + dx
    ref = torch.nn.grad.conv2d_input((n, cin, hw, hw), w.double(), g0, padding=1)
    assert rel(gx, ref) < 1e-5
    assert hip.lvae_conv3x3_pool_dgrad_f32(_lib.ptr(gy), _lib.ptr(y), _lib.ptr(idx), _lib.ptr(w), n, c, 5, hw, hw,
                                           _lib.ptr(gx), _lib.stream_ptr()) == -3
    assert hip.lvae_conv3x3_pool_dgrad_f32(_lib.ptr(gy), _lib.ptr(y), _lib.ptr(idx), _lib.ptr(w), n, 64, cin, 34, 34,
                                           _lib.ptr(gx), _lib.stream_ptr()) == -4


@pytest.mark.parametrize("n,cin,hw", [(5, 16, 18), (37, 16, 18), (3, 5, 7), (2051, 16, 18)])
def test_deconv_sigmoid_matches_torch(hip, n, cin, hw):
    """Decoder output layer sigmoid(ConvTranspose2d(cin, 1, 4, 2, 1)(z)) as one HIP pass each way vs
    torch (MIOpen transposed conv + sigmoid): output and all three gradients to fp32 rounding."""
    from lvae_amd.vae import deconv_sigmoid
    gen = torch.Generator(device=DEV).manual_seed(3)
    dc = torch.nn.ConvTranspose2d(cin, 1, 4, 2, 1).to(DEV)
    z = torch.randn(n, cin, hw, hw, device=DEV, generator=gen)
    g = None
    outs = []
    for fused in (True, False):
        zr = z.clone().requires_grad_()
        y = deconv_sigmoid(dc, zr) if fused else torch.sigmoid(dc(zr))
        if g is None:
            g = torch.randn(y.shape, device=DEV, generator=gen)
        outs.append([y] + list(torch.autograd.grad(y, [zr, dc.weight, dc.bias], g)))
    assert outs[0][0].shape == (n, 1, 2 * hw, 2 * hw)
    # output and input gradient: a few fp32 roundings; weight / bias gradients: sums over n (2hw)^2
    # terms of both signs in a different order than MIOpen's -> 1e-4 of their max
    for a, b, tol in zip(*outs, (1e-5, 1e-5, 1e-4, 1e-4)):
        assert float((a - b).abs().max() / b.abs().max()) < tol


def _random_hypers(k, L, rng, scale=(0.3, 1.5), ell=(1.0, 4.0)):
    """[L, P] raw parameters: per-dim random scales and lengthscales (named_parameters order)."""
    return np.stack([np.log(rng.uniform(*scale, L)) if "scale" in n else np.log(rng.uniform(*ell, L))
                     for n, _ in k.named_parameters()], 1)


def _kl_vs_oracle(P, L, raw, noise, seed, oracle_dev="cpu", dims_cpu=None, cfg=CFG, return_per_dim=False):
    """HIP KL_closed_batched (values + all gradients) vs the fp64 oracle, per latent dim.
    oracle_dev="cuda": the oracle's fp64 formula evaluated by PyTorch on the GPU (large N);
    dims_cpu: dims additionally checked with the CPU oracle.  Returns the max relative errors."""
    import lvae_amd as la
    from lvae_amd.data import health_mnist_covariates
    T = 16
    X = torch.tensor(health_mnist_covariates(P, T, seed=seed))
    gen = torch.Generator().manual_seed(seed)
    mu = torch.randn(P * T, L, generator=gen, dtype=torch.float64)
    lv = 0.1 * torch.randn(P * T, L, generator=gen, dtype=torch.float64)
    k = la.generate_kernel(**cfg, latent_dim=L).double()
    set_raw(k, raw)
    kd = k.to(DEV)
    lik = la.GaussianLikelihood(L, noise=1.0).to(DEV)
    lik.noise = torch.as_tensor(noise, dtype=torch.float64)
    mu_d, lv_d = mu.to(DEV).requires_grad_(), lv.to(DEV).requires_grad_()
    from lvae_amd.elbo import kl_closed_refine_log
    with kl_closed_refine_log() as rlog:
        kl = la.KL_closed_batched(kd, X.to(DEV), lik, mu_d, lv_d)
    w = torch.arange(1, L + 1, device=DEV, dtype=torch.float64)
    (kl * w).sum().backward()
    draw = torch.stack([p.grad for _, p in kd.named_parameters()], 1)  # [L, P]
    assert torch.isfinite(kl).all() and torch.isfinite(mu_d.grad).all() and torch.isfinite(draw).all()
    spec = O.spec_full(**cfg)
    nz = torch.as_tensor(noise, dtype=torch.float64).expand(L)
    worst = dict(kl=0.0, dmu=0.0, dlogv=0.0, draw=0.0)
    per_dim = {}
    for dev, dims in ((oracle_dev, range(L)), ("cpu", dims_cpu or [])):
        for l in dims:
            r = torch.tensor(raw[l], device=dev, requires_grad=True)
            m_ = mu[:, l].to(dev).clone().requires_grad_()
            v_ = lv[:, l].to(dev).clone().requires_grad_()
            ref = O.kl_closed(spec, O.constrain(r), X.to(dev), float(nz[l]), m_, v_)
            ((l + 1) * ref).backward()
            errs = dict(kl=rel(kl[l], ref), dmu=rel(mu_d.grad[:, l], m_.grad), dlogv=rel(lv_d.grad[:, l], v_.grad),
                        draw=rel(draw[l], r.grad))
            for key, e in errs.items():
                worst[key] = max(worst[key], e)
            per_dim.setdefault(l, {}).update({f"{dev}:{k}": v for k, v in errs.items()})
            if rlog:  # the fp64 diag(K^-1) refinement's gate (kl_refine.hip)
                per_dim[l]["est"] = float(rlog[0][0][l])
                per_dim[l]["refined"] = int(rlog[0][1][l])
            # the KL error split: tr(K^-1 V) = sum (2 dlogv / w + 1) on both sides (w = l + 1)
            v64 = torch.exp(lv[:, l]).to(dev)
            tr_hip = float((2 * lv_d.grad[:, l].to(dev).double() / (l + 1) + 1).sum())
            tr_ref = float((2 * v_.grad / (l + 1) + 1).sum())
            dkl = float(kl[l]) - float(ref)
            per_dim[l]["trace_err"] = abs(0.5 * (tr_hip - tr_ref)) / abs(float(ref))
            per_dim[l]["rest_err"] = abs(dkl - 0.5 * (tr_hip - tr_ref)) / abs(float(ref))
            del v64
    if return_per_dim:
        return worst, per_dim
    return worst


def _cond(spec, raw, X, noise, dev=DEV):
    K = O.gram(spec, O.constrain(torch.tensor(raw, device=dev)), X.to(dev), X.to(dev))
    ev = torch.linalg.eigvalsh(K + noise * torch.eye(X.shape[0], dtype=torch.float64, device=dev))
    return float(ev[-1] / ev[0])


def test_kl_closed_headline_workload(hip):
    """The bench's own workload: N = 4096 (P = 256 x T = 16), L = 16 batched, every dim with its own
    random scales (0.3..1.5), lengthscales (1..4) and noise (0.5..1) around the sample config's init
    (cond(K) up to ~1e4) -- KL and every gradient vs the fp64 oracle within the north-star 1e-4.  All
    16 dims against the oracle formula run in fp64 on the GPU, dims 0 and 15 also on the CPU oracle."""
    import lvae_amd as la
    from lvae_amd.data import health_mnist_covariates
    L, P = 16, 256
    rng = np.random.default_rng(16)
    k = la.generate_kernel(**CFG, latent_dim=L)
    raw = _random_hypers(k, L, rng, scale=(0.3, 1.5), ell=(1.0, 4.0))
    noise = torch.tensor(rng.uniform(0.5, 1.0, L))
    worst, per = _kl_vs_oracle(P, L, raw, noise, seed=16, oracle_dev="cuda", dims_cpu=[0, 15], return_per_dim=True)
    X = torch.tensor(health_mnist_covariates(P, 16, seed=16))
    spec = O.spec_full(**CFG)
    for l in range(L):
        print(f"dim {l}: cond(K) {_cond(spec, raw[l], X, float(noise[l])):.2e}", per[l])
    print("headline workload max rel errors:", worst)
    for key, e in worst.items():
        assert e < 1e-4, (key, e)


def test_kl_closed_high_cond(hip):
    """Wider hyper-parameter draws at N = 4096 (scales 0.2..3, lengthscales 0.5..6, noise 0.05..1:
    cond(K) up to ~1e5).  The KL, dmu = K^-1 mu (the blocked Cholesky inverse + one fp64 refinement step
    of K^-1 mu) and dlogv (diag K^-1: refined in fp64 where the gate flags the dim, kl_refine.hip) within
    the north-star 1e-4; the hyper-parameter gradients (through K^-1 and S = K^-1 V K^-1, not refined)
    within 1e-4 as well.  Printed per dim: cond(K), the gate's estimate and whether it refined."""
    import lvae_amd as la
    from lvae_amd.data import health_mnist_covariates
    L, P = 8, 256
    rng = np.random.default_rng(17)
    k = la.generate_kernel(**CFG, latent_dim=L)
    raw = _random_hypers(k, L, rng, scale=(0.2, 3.0), ell=(0.5, 6.0))
    noise = torch.tensor(rng.uniform(0.05, 1.0, L))
    worst, per = _kl_vs_oracle(P, L, raw, noise, seed=17, oracle_dev="cuda", return_per_dim=True)
    X = torch.tensor(health_mnist_covariates(P, 16, seed=17))
    spec = O.spec_full(**CFG)
    for l in range(L):
        cond = _cond(spec, raw[l], X, float(noise[l]))
        print(f"dim {l}: cond(K) {cond:.2e}", per[l])
        for key in ("kl", "dmu", "dlogv", "draw"):
            assert per[l][f"cuda:{key}"] < 1e-4, (l, key)


@pytest.mark.parametrize("case", ["headline", "high_cond"])
def test_kl_closed_early_route(hip, monkeypatch, case):
    """The opt-in early reduce (LVAE_KL_EARLY=1, kl_closed.hip): a0 = Y^T (Y mu), diag K^-1 = the row sums of
    squares of Y^T and a = a0 + Y^T (Y r) from the Y / Y^T planes before any lauum; the refinement gate on that
    diagonal, and for the flagged dims their K^-1 alone (ci_lauum_flagged_f32) for the fp64 diag refinement; lauum
    in the backward.  The headline workload and the high-cond draws of the tests above (some dims flagged), every
    value and gradient within the north-star 1e-4 of the fp64 oracle."""
    import lvae_amd as la
    monkeypatch.setenv("LVAE_KL_EARLY", "1")
    L, P = (16, 256) if case == "headline" else (8, 256)
    rng = np.random.default_rng(16 if case == "headline" else 17)
    k = la.generate_kernel(**CFG, latent_dim=L)
    if case == "headline":
        raw = _random_hypers(k, L, rng, scale=(0.3, 1.5), ell=(1.0, 4.0))
        noise = torch.tensor(rng.uniform(0.5, 1.0, L))
    else:
        raw = _random_hypers(k, L, rng, scale=(0.2, 3.0), ell=(0.5, 6.0))
        noise = torch.tensor(rng.uniform(0.05, 1.0, L))
    worst, per = _kl_vs_oracle(P, L, raw, noise, seed=16 if case == "headline" else 17, oracle_dev="cuda",
                               return_per_dim=True)
    print(f"early route, {case}:", worst, "refined dims:", [l for l in range(L) if per[l]["refined"]])
    for key, e in worst.items():
        assert e < 1e-4, (key, e)


@pytest.mark.parametrize("noise", [1e-3, 1e-4])
def test_kl_closed_small_noise(hip, noise):
    """Small likelihood noise (N = 1024: cond(K) 1e3..1.3e5; K^-1 entries ~1/noise, which the
    per-block split scales keep inside fp16's range).  KL, dmu, dlogv (diag K^-1 refined in fp64 for the
    gated dims, kl_refine.hip) and draw within the north-star 1e-4 of the fp64 oracle.  Printed: the KL
    error split into the trace term tr(K^-1 V) (recovered from dlogv = (v diag K^-1 - 1) / 2) and the
    rest (log|K| and mu^T K^-1 mu, the latter refined in fp64), and the refinement gate per dim."""
    import lvae_amd as la
    from lvae_amd.data import health_mnist_covariates
    L, P, T = 2, 64, 16
    rng = np.random.default_rng(int(1 / noise))
    k = la.generate_kernel(**CFG, latent_dim=L)
    raw = _random_hypers(k, L, rng)
    X = torch.tensor(health_mnist_covariates(P, T, seed=3))
    spec = O.spec_full(**CFG)
    conds = []
    for l in range(L):
        K = O.gram(spec, O.constrain(torch.tensor(raw[l])), X, X) + noise * torch.eye(P * T, dtype=torch.float64)
        ev = torch.linalg.eigvalsh(K)
        conds.append(float(ev[-1] / ev[0]))
    worst, per = _kl_vs_oracle(P, L, raw, noise, seed=3, return_per_dim=True)
    print(f"noise {noise}: cond(K) {max(conds):.3e}, errors {worst}")
    for l in range(L):
        print(f"  dim {l}: cond {conds[l]:.2e}, trace-term error / |KL| {per[l]['trace_err']:.2e}, "
              f"rest (log|K| + mu^T K^-1 mu) {per[l]['rest_err']:.2e}, gate est {per[l].get('est', 0):.2e} "
              f"refined {per[l].get('refined')}")
    for key, e in worst.items():
        assert e < 1e-4, (key, e)


@pytest.mark.parametrize("mode", ["0", "1"])
def test_kl_refine_forced(hip, monkeypatch, mode):
    """The fp64 diag(K^-1) refinement (kl_refine.hip) switched off / forced on for every dim, on a
    ragged N (P = 67 subjects: n = 1072, not a multiple of the 128-wide refinement tiles) with one
    small-noise dim (cond ~1e5) and one well-conditioned dim: the gate's state reports the mode, the
    refined run holds dlogv within 1e-5 of the fp64 oracle on both dims (the Newton step squares the
    fp32 inverse's error), the unrefined one leaves the small-noise dim's dlogv at the fp32 level."""
    import lvae_amd as la
    monkeypatch.setenv("LVAE_KL_REFINE", mode)
    L, P = 2, 67
    rng = np.random.default_rng(5)
    k = la.generate_kernel(**CFG, latent_dim=L)
    raw = _random_hypers(k, L, rng)
    worst, per = _kl_vs_oracle(P, L, raw, torch.tensor([1e-3, 0.7]), seed=5, return_per_dim=True)
    print(f"LVAE_KL_REFINE={mode}:", {l: per[l] for l in range(L)})
    for l in range(L):
        assert per[l]["refined"] == int(mode), l
        assert per[l]["cpu:kl"] < 1e-4 and per[l]["cpu:dmu"] < 1e-4, l
    if mode == "1":
        assert worst["dlogv"] < 1e-5 and worst["kl"] < 1e-5, worst
    else:
        assert per[1]["est"] == 0.0


def test_kl_closed_c5_refined(hip, monkeypatch):
    """The fp64 diag(K^-1) refinement (kl_refine.hip) forced on at the C5 size (N = 16384, one dim: the
    fp64 K is 2 GiB, 128-wide tiles of K X over 16384^2) against the GPU-evaluated fp64 oracle: every
    value and gradient within 1e-4, dlogv far below the unrefined dim's 1.4e-5."""
    import lvae_amd as la
    monkeypatch.setenv("LVAE_KL_REFINE", "1")
    P, L = 1024, 1
    rng = np.random.default_rng(1025)
    k = la.generate_kernel(**CFG, latent_dim=L)
    raw = _random_hypers(k, L, rng)
    worst, per = _kl_vs_oracle(P, L, raw, 1.0, seed=1025, oracle_dev="cuda", return_per_dim=True)
    print("C5 refined:", per[0])
    assert per[0]["refined"] == 1
    for key, e in worst.items():
        assert e < 1e-4, (key, e)
    assert worst["dlogv"] < 1e-6, worst


@pytest.mark.parametrize("L", [1, 4])
def test_kl_closed_c5(hip, L):
    """C5 shape (N = 16384: P = 1024 x T = 16), the reference kernel set: one latent dim, and L = 4 --
    one rank's share of C5's L = 32 on 8 GPUs (training.py:515-575 loops KL_closed over every dim;
    here the 4 dims go through ONE batched launch sequence at np = 16384, as a rank of the sharded
    step runs them).  KL and all gradients of every dim vs the oracle's fp64 formula evaluated on the
    GPU (a CPU fp64 inverse at this size takes minutes); bound 1e-4."""
    import lvae_amd as la
    P = 1024
    rng = np.random.default_rng(1024 + L)
    k = la.generate_kernel(**CFG, latent_dim=L)
    raw = _random_hypers(k, L, rng)
    worst, per = _kl_vs_oracle(P, L, raw, 1.0, seed=1024 + L, oracle_dev="cuda", return_per_dim=True)
    for l in range(L):
        print(f"C5 L={L} dim {l}:", per[l])
    print(f"C5 L={L} max rel errors:", worst)
    for key, e in worst.items():
        assert e < 1e-4, (key, e)


C5_CFG_EXT = "RBF(time) + Cat(subject) + Per(time) + Lin(disease_time)"


def _c5_kernel(L):
    """The C5 stress kernel (BASELINE configs[4]): the sample config's R = 5 components plus the
    periodic and linear extensions -- PARITY UNPINNED (no reference kernel; checked against the
    oracle's own restatement only)."""
    import lvae_amd as la
    from lvae_amd.kernels import AdditiveKernel, LinearKernel, PeriodicKernel, ScaleKernel
    base = la.generate_kernel(**CFG, latent_dim=L)
    return AdditiveKernel(list(base.kernels) + [ScaleKernel(PeriodicKernel(0, L, 1.5, 6.0), L),
                                                ScaleKernel(LinearKernel(1), L, scale=0.05)])


def _c5_spec():
    return O.spec_full(**CFG) + [[("per", 0)], [("lin", 1)]]


@pytest.mark.parametrize("P,L,dev", [(16, 2, "cpu"), (64, 2, "cpu"), (1024, 1, "cuda"), (1024, 4, "cuda")])
def test_kl_closed_periodic_linear(hip, P, L, dev):
    """Periodic + linear extension kernels (parity unpinned: the reference has neither) through the
    exact KL: values and gradients (incl. period / lengthscale of the periodic factor) vs the oracle
    restatement; N = 16384 (C5) on the GPU-evaluated fp64 oracle, one dim and one rank's share of
    C5 (L = 4, the C5 stress kernel of BASELINE configs[4])."""
    import lvae_amd as la
    from lvae_amd.data import health_mnist_covariates
    T = 16
    X = torch.tensor(health_mnist_covariates(P, T, seed=P))
    gen = torch.Generator().manual_seed(P)
    mu = torch.randn(P * T, L, generator=gen, dtype=torch.float64)
    lv = 0.1 * torch.randn(P * T, L, generator=gen, dtype=torch.float64)
    k = _c5_kernel(L).double()
    rng = np.random.default_rng(P)
    with torch.no_grad():
        for _, p in k.named_parameters():
            p.add_(torch.tensor(rng.uniform(-0.3, 0.3, L)))
    raw = torch.stack([p.detach().clone() for _, p in k.named_parameters()], 1)
    kd = k.to(DEV)
    lik = la.GaussianLikelihood(L, noise=1.0).to(DEV)
    mu_d, lv_d = mu.to(DEV).requires_grad_(), lv.to(DEV).requires_grad_()
    from lvae_amd.elbo import kl_closed_refine_log
    with kl_closed_refine_log() as rlog:
        kl = la.KL_closed_batched(kd, X.to(DEV), lik, mu_d, lv_d)
    kl.sum().backward()
    spec = _c5_spec()
    for l in range(L):
        r = raw[l].to(dev).clone().requires_grad_()
        m_, v_ = mu[:, l].to(dev).clone().requires_grad_(), lv[:, l].to(dev).clone().requires_grad_()
        ref = O.kl_closed(spec, O.constrain(r), X.to(dev), 1.0, m_, v_)
        ref.backward()
        assert rel(kl[l], ref) < 1e-4
        assert rel(mu_d.grad[:, l], m_.grad) < 1e-4
        assert rel(lv_d.grad[:, l], v_.grad) < 1e-4
        assert rel(torch.stack([p.grad[l] for _, p in kd.named_parameters()]), r.grad) < 1e-4


CFG_GATES = dict(cat_kernel=[2], bin_kernel=[4], sqexp_kernel=[0],
                 cat_int_kernel=[{'cont_covariate': 0, 'cat_covariate': 3}],
                 bin_int_kernel=[{'cont_covariate': 1, 'bin_covariate': 4}],
                 covariate_missing_val=[{'covariate': 1, 'mask': 5}])


@pytest.mark.parametrize("case", ["integer", "half_time", "wide_window", "gates_masks", "c5"])
def test_kl_closed_resid_paths(hip, case):
    """The fp64 residual r = mu - K a0 behind the K^-1 mu refinement (elbo_functions.py:27-30) on both
    of its paths: integer-coded covariates go through the binned O(N W) kernels (kl_resid_bins.hip:
    "integer", Bin gates and a missing-value mask in "gates_masks", the periodic / linear C5 factors in
    "c5"), the rest through the tiled O(N^2) kernel (times shifted by 0.5: "half_time"; a time window
    of 76 > 64 values: "wide_window").  dmu = K^-1 mu is the refined quantity: within 1e-8 of the fp64
    oracle (the refinement reaches ~1e-10 here; a residual that missed terms leaves the fp32-equivalent
    inverse's ~1e-5), and the KL within 1e-6.  The same cases select the Gram fill / adjoint paths
    (gram.hip covariate flag): tables for "integer" / "gates_masks", fp32 covariates for "wide_window"
    and "c5" (a linear factor), fp64 covariates for "half_time" -- dlogv and draw within 1e-4."""
    import lvae_amd as la
    from lvae_amd.data import health_mnist_covariates
    P, T, L = 64, 16, 2
    cfg = CFG_GATES if case == "gates_masks" else CFG
    X = torch.tensor(health_mnist_covariates(P, T, seed=7))
    if case == "half_time":
        X[:, 0] += 0.5
    elif case == "wide_window":
        X[:, 0] *= 5.0
    gen = torch.Generator().manual_seed(7)
    mu = torch.randn(P * T, L, generator=gen, dtype=torch.float64)
    lv = 0.1 * torch.randn(P * T, L, generator=gen, dtype=torch.float64)
    rng = np.random.default_rng(7)
    if case == "c5":  # around its own init (the linear factor's scale 0.05 keeps cond(K) moderate)
        k = _c5_kernel(L).double()
        with torch.no_grad():
            for _, p in k.named_parameters():
                p.add_(torch.tensor(rng.uniform(-0.3, 0.3, L)))
    else:
        k = la.generate_kernel(**cfg, latent_dim=L).double()
        set_raw(k, _random_hypers(k, L, rng))
    raw = torch.stack([p.detach().clone() for _, p in k.named_parameters()], 1)
    kd = k.to(DEV)
    lik = la.GaussianLikelihood(L, noise=1.0).to(DEV)
    mu_d, lv_d = mu.to(DEV).requires_grad_(), lv.to(DEV).requires_grad_()
    from lvae_amd.elbo import kl_closed_refine_log
    with kl_closed_refine_log() as rlog:
        kl = la.KL_closed_batched(kd, X.to(DEV), lik, mu_d, lv_d)
    kl.sum().backward()
    spec = _c5_spec() if case == "c5" else O.spec_full(**cfg)
    for l in range(L):
        r = raw[l].clone().requires_grad_()
        m_, v_ = mu[:, l].clone().requires_grad_(), lv[:, l].clone().requires_grad_()
        ref = O.kl_closed(spec, O.constrain(r), X, 1.0, m_, v_)
        ref.backward()
        e_kl, e_mu = rel(kl[l], ref), rel(mu_d.grad[:, l], m_.grad)
        e_lv = rel(lv_d.grad[:, l], v_.grad)
        e_raw = rel(torch.stack([p.grad[l] for _, p in kd.named_parameters()]), r.grad)
        print(f"{case} dim {l}: kl {e_kl:.2e} dmu {e_mu:.2e} dlogv {e_lv:.2e} draw {e_raw:.2e}")
        assert e_kl < 1e-6 and e_mu < 1e-8, (case, l, e_kl, e_mu)
        assert e_lv < 1e-4 and e_raw < 1e-4, (case, l, e_lv, e_raw)


def test_closed_step_vs_oracle(hip):
    """One full standard_training step with type_KL='closed' (training.py:484-592): ConvVAE forward /
    backward over all N = 1024 images, the exact KL of L = 4 dims, the step composition
    recon + weight * KL / L -- net, recon and KL terms plus the raw kernel-parameter and network
    gradients vs oracle.closed_step (fp32 conv vs fp64 reference: 1e-4)."""
    import lvae_amd as la
    from lvae_amd.steps import ClosedStep
    from lvae_amd.vae import ConvVAE
    from lvae_amd.data import health_mnist_batch
    L, P, T = 4, 64, 16
    img, mask, X = health_mnist_batch(P, T, seed=8, dtype=torch.float64)
    ref_vae = O.ConvVAE(L).double()
    ref_vae.load_state_dict(O.vae_weights(ref_vae, 21))
    vae = ConvVAE(L, 1296, p_input=0.0, p=0.0).double()
    vae.load_state_dict(ref_vae.state_dict())
    vae = vae.float().to(DEV)
    k = la.generate_kernel(**CFG, latent_dim=L)
    rng = np.random.default_rng(8)
    set_raw(k, _random_hypers(k, L, rng))
    raw = torch.stack([p.detach().clone() for _, p in k.named_parameters()], 1).requires_grad_()
    kd = k.to(DEV)
    lik = la.GaussianLikelihood(L, noise=1.0).to(DEV)
    eps = torch.randn(P * T, L, generator=torch.Generator().manual_seed(1), dtype=torch.float64)
    loss, recon, gp = O.closed_step(ref_vae, O.spec_full(**CFG), raw, torch.ones(L, dtype=torch.float64), img, mask,
                                    X, eps, 0.15)
    opt = torch.optim.SGD(list(vae.parameters()) + list(kd.parameters()), lr=0.0)
    step = ClosedStep(vae, kd, lik, opt, weight=0.15, loss_function="mse")
    net, rl, _, g = step(img.float().to(DEV), mask.float().to(DEV), X.to(DEV), eps.float().to(DEV))
    assert rel(net, loss) < 1e-4
    assert rel(rl, recon) < 1e-4
    assert rel(g, gp) < 1e-4
    assert rel(torch.stack([p.grad for _, p in kd.named_parameters()], 1), raw.grad) < 1e-4
    for (name, p), (_, q) in zip(vae.named_parameters(), ref_vae.named_parameters()):
        if q.grad is not None:  # (_log_vy has no gradient under loss='mse')
            assert rel(p.grad, q.grad) < 1e-3, name


def test_closed_step_headline_vs_oracle(hip):
    """The bench's whole step at the headline shape (BASELINE configs[2]: N = 4096 images, L = 16; training.py:
    499-575): ClosedStep -- the HIP ConvVAE kernels and MIOpen / hipBLASLt in fp32, the exact KL of all 16 dims --
    against oracle.closed_step in fp64 on the GPU (the reference's ConvVAE in fp64 over all 4096 images and the
    oracle's KL formula: fp64 Gram, Cholesky, cholesky_solve per dim, autograd through both).
    Bounds: net, recon and KL terms and the raw kernel-parameter gradients 1e-4 (north star; measured r6: 9e-9
    and 4.7e-7).  The network gradients: 2e-4 of each tensor's max, twice the largest measured (r6: fc4.weight
    9.9e-5, fc3.weight 9.6e-5, the encoder convs 2-3e-5; profiles/r6_pytest_gpu.log) -- fp32 layers against
    fp64 over sums of 4096 images, where a relu / 2x2 max-pool decision that sits within fp32 rounding of a tie
    can flip and reroute one pooled gradient (test_conv_relu_maxpool_fused's docstring).
    """
    import lvae_amd as la
    from lvae_amd.steps import ClosedStep
    from lvae_amd.vae import ConvVAE
    from lvae_amd.data import health_mnist_batch
    L, P, T = 16, 256, 16
    img, mask, X = health_mnist_batch(P, T, seed=31, dtype=torch.float64)
    ref_vae = O.ConvVAE(L).double()
    ref_vae.load_state_dict(O.vae_weights(ref_vae, 31))
    vae = ConvVAE(L, 1296, p_input=0.0, p=0.0).double()
    vae.load_state_dict(ref_vae.state_dict())
    vae = vae.float().to(DEV)
    ref_vae = ref_vae.to(DEV)
    k = la.generate_kernel(**CFG, latent_dim=L)
    rng = np.random.default_rng(31)
    set_raw(k, _random_hypers(k, L, rng))
    raw = torch.stack([p.detach().clone() for _, p in k.named_parameters()], 1).to(DEV).requires_grad_()
    kd = k.to(DEV)
    lik = la.GaussianLikelihood(L, noise=1.0).to(DEV)
    eps = torch.randn(P * T, L, generator=torch.Generator().manual_seed(31), dtype=torch.float64)
    loss, recon, gp = O.closed_step(ref_vae, O.spec_full(**CFG), raw, torch.ones(L, dtype=torch.float64, device=DEV),
                                    img.to(DEV), mask.to(DEV), X.to(DEV), eps.to(DEV), 0.15)
    opt = torch.optim.SGD(list(vae.parameters()) + list(kd.parameters()), lr=0.0)
    step = ClosedStep(vae, kd, lik, opt, weight=0.15, loss_function="mse")
    net, rl, _, g = step(img.float().to(DEV), mask.float().to(DEV), X.to(DEV), eps.float().to(DEV))
    torch.cuda.synchronize()
    errs = dict(net=rel(net, loss), recon=rel(rl, recon), kl=rel(g, gp),
                raw=rel(torch.stack([p.grad for _, p in kd.named_parameters()], 1), raw.grad))
    print("headline step:", errs)
    for key, e in errs.items():
        assert e < 1e-4, (key, e)
    for (name, p), (_, q) in zip(vae.named_parameters(), ref_vae.named_parameters()):
        if q.grad is None:  # (_log_vy has no gradient under loss='mse')
            continue
        e = rel(p.grad, q.grad)
        print(f"  {name}: {e:.2e}")
        assert e < 2e-4, (name, e)


def test_latent_sharded_closed_step_cuda_path(hip):
    """LatentShardedClosedStep's CUDA path (decoder + recon backward on a second stream beside the
    all-gather / KL / all-reduce, dLoss/dz joined into the encoder backward) in a world-1 gloo group
    on the GPU, against the oracle's whole-batch step: loss terms and every gradient."""
    import socket
    import torch.distributed as dist
    import lvae_amd as la
    from lvae_amd.distributed import LatentShardedClosedStep
    from lvae_amd.vae import ConvVAE
    from lvae_amd.data import health_mnist_batch
    L, P, T = 4, 32, 16
    img, mask, X = health_mnist_batch(P, T, seed=9, dtype=torch.float64)
    ref_vae = O.ConvVAE(L).double()
    ref_vae.load_state_dict(O.vae_weights(ref_vae, 22))
    vae = ConvVAE(L, 1296, p_input=0.0, p=0.0).double()
    vae.load_state_dict(ref_vae.state_dict())
    vae = vae.float().to(DEV)
    k = la.generate_kernel(**CFG, latent_dim=L)
    set_raw(k, _random_hypers(k, L, np.random.default_rng(9)))
    raw = torch.stack([p.detach().clone() for _, p in k.named_parameters()], 1).requires_grad_()
    kd = k.to(DEV)
    lik = la.GaussianLikelihood(L, noise=1.0).to(DEV)
    eps = torch.randn(P * T, L, generator=torch.Generator().manual_seed(2), dtype=torch.float64)
    loss, recon, gp = O.closed_step(ref_vae, O.spec_full(**CFG), raw, torch.ones(L, dtype=torch.float64), img, mask,
                                    X, eps, 0.15)
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        opt = torch.optim.SGD(list(vae.parameters()) + list(kd.parameters()), lr=0.0)
        step = LatentShardedClosedStep(vae, kd, lik, opt, weight=0.15, loss_function="mse")
        net, rl, _, g = step(img.float().to(DEV), mask.float().to(DEV), X.to(DEV), eps.float().to(DEV))
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
    assert rel(net, loss) < 1e-4
    assert rel(rl, recon) < 1e-4
    assert rel(g, gp) < 1e-4
    assert rel(torch.stack([p.grad for _, p in kd.named_parameters()], 1), raw.grad) < 1e-4
    for (name, p), (_, q) in zip(vae.named_parameters(), ref_vae.named_parameters()):
        if q.grad is not None:
            assert rel(p.grad, q.grad) < 1e-3, name


VAR_CFG = dict(cat_kernel=[2, 3], bin_kernel=[5], sqexp_kernel=[0],
               cat_int_kernel=[{'cont_covariate': 0, 'cat_covariate': 2},
                               {'cont_covariate': 1, 'cat_covariate': 4}],
               bin_int_kernel=[{'cont_covariate': 0, 'bin_covariate': 4}],
               covariate_missing_val=[{'covariate': 0, 'mask': 6}, {'covariate': 3, 'mask': 7}])


def test_kl_closed_kernel_variants_golden(hip):
    """Bin, bin x RBF and missing-value mask products (GP_model.py:146-236) through the HIP Gram,
    sweep and adjoint, against the reference's KL_closed (kernel_variants_kl.npz, N = 80)."""
    import lvae_amd as la
    g = golden("kernel_variants_kl.npz")
    L = int(g["L"])
    k0, k1 = la.generate_kernel_batched(L, **VAR_CFG, id_covariate=2)
    k = k0 + k1
    set_raw(k, g["raw"])
    k = k.to(DEV)
    lik = la.GaussianLikelihood(L, noise=float(g["noise"][0])).to(DEV)
    X = torch.tensor(g["X"], device=DEV)
    with torch.no_grad():
        K = k(X, X).evaluate()
    assert rel(K, g["gram"]) < 1e-13
    mu = torch.tensor(g["mu"], device=DEV, requires_grad=True)
    lv = torch.tensor(g["logv"], device=DEV, requires_grad=True)
    kl = la.KL_closed_batched(k, X, lik, mu, lv)
    kl.sum().backward()
    assert rel(kl, g["kl"]) < 1e-4
    assert rel(mu.grad, g["dmu"]) < 1e-4
    assert rel(lv.grad, g["dlogv"]) < 1e-4
    draw = torch.stack([p.grad for _, p in k.named_parameters()], 1)
    assert rel(draw, g["draw"]) < 1e-4


def test_closed_step_three_epochs_vs_reference(hip):
    """Three epochs of the reference's standard_training(type_KL='closed') (standard_training_closed
    .npz: full batch N = 64, L = 2, Adam, constrain_scales) replayed through lvae_amd.ClosedStep (the
    step the bench times) with an fp64 ConvVAE: per-step net / recon / GP loss and the final kernel
    and network parameters.  The KL is fp32-equivalent (north-star 1e-4); the parameters move by
    lr-sized Adam steps whose direction is insensitive to that, so they match to ~1e-6."""
    import lvae_amd as la
    from lvae_amd.steps import ClosedStep
    from lvae_amd.vae import ConvVAE
    g = golden("standard_training_closed.npz")
    L, epochs = int(g["L"]), int(g["epochs"])
    img = torch.tensor(g["pix"].astype(np.float64) / 255.0, device=DEV)
    mask = torch.tensor(g["msk"].astype(np.float64), device=DEV)
    X = torch.tensor(g["X"], device=DEV)
    ref_vae = O.ConvVAE(L).double()
    ref_vae.load_state_dict(O.vae_weights(ref_vae, int(g["seed"])))
    vae = ConvVAE(L, 1296, p_input=0.0, p=0.0).double()
    vae.load_state_dict(ref_vae.state_dict())
    vae = vae.to(DEV)
    k = la.generate_kernel(**CFG, latent_dim=L).double()
    set_raw(k, g["raw"])
    k = k.to(DEV)
    lik = la.GaussianLikelihood(L, noise=1.0).to(DEV)
    opt = torch.optim.Adam(list(k.parameters()) + list(vae.parameters()), lr=1e-3)
    step = ClosedStep(vae, k, lik, opt, weight=0.15)
    for s in range(epochs):
        net, recon, nll, gp = step(img, mask, X, torch.tensor(g["eps"][2 * s], device=DEV))
        assert rel(net, g["step_net"][s]) < 1e-4, s
        # step 0 is the same fp64 network on the same weights; later steps see weights moved by
        # Adam with the fp32-equivalent KL gradients
        assert rel(recon, g["step_recon"][s]) < (1e-12 if s == 0 else 1e-7), s
        assert rel(nll, g["step_nll"][s]) < (1e-12 if s == 0 else 1e-7), s
        assert rel(gp, g["step_gp"][s]) < 1e-4, s
    assert rel(torch.stack([p for _, p in k.named_parameters()], 1), g["raw_final"]) < 1e-5
    sd = dict(vae.named_parameters())
    for name in ("conv1.weight", "fc211.bias", "deconv2.weight", "_log_vy"):
        assert rel(sd[name], g["vae_" + name]) < 1e-5, name


def test_kl_factor_single_use_and_rank_share_rehearsal(hip):
    """(1) A KLFactor is consumed by its reduce (the backward overwrites its operands): a second
    KL_closed_batched(..., factor=) on it raises.  (2) The rank-share rehearsal (LatentShardedClosedStep
    with sim_world = 2: rank 0's dims and images, collectives replaced by local stand-ins -- bench.py
    --rank-share) returns the KL of its own dims over the stand-in all-gather (its rows tiled), which the
    batched KL of those rows reproduces."""
    import lvae_amd as la
    from lvae_amd.distributed import LatentShardedClosedStep
    from lvae_amd.elbo import kl_closed_prefactor
    from lvae_amd.vae import ConvVAE
    from lvae_amd.data import health_mnist_batch
    L, P, T = 4, 32, 16
    img, mask, X = health_mnist_batch(P, T, seed=5, device=DEV)
    k = la.generate_kernel(**CFG, latent_dim=L).to(DEV)
    lik = la.GaussianLikelihood(L, noise=1.0).to(DEV)
    mu = torch.randn(P * T, L, device=DEV, dtype=torch.float64)
    lv = 0.1 * torch.randn(P * T, L, device=DEV, dtype=torch.float64)
    f = kl_closed_prefactor(k, X, lik, L, torch.cuda.current_stream())
    kl1 = la.KL_closed_batched(k, X, lik, mu, lv, factor=f)
    kl0 = la.KL_closed_batched(k, X, lik, mu, lv)
    assert rel(kl1, kl0) < 1e-6
    with pytest.raises(RuntimeError, match="already used"):
        la.KL_closed_batched(k, X, lik, mu, lv, factor=f)
    # the rank-share rehearsal, rank 0 of 2
    torch.manual_seed(3)
    vae = ConvVAE(L, 1296, p_input=0.0, p=0.0).to(DEV)
    opt = torch.optim.SGD(list(vae.parameters()) + list(k.parameters()), lr=0.0)
    W, n = 2, P * T // 2
    eps = torch.randn(n, L, device=DEV, generator=torch.Generator(device=DEV).manual_seed(1))
    step = LatentShardedClosedStep(vae, k, lik, opt, weight=0.15, loss_function="mse", sim_world=W)
    net, rl, nl, gp = step(img[:n], mask[:n], X, eps)
    with torch.no_grad():
        m_, v_ = vae.encode(img[:n])
        full = torch.cat([m_, v_], 1).repeat(W, 1).double()
    spec, params = la.kernel_spec_and_params(k)
    from lvae_amd.elbo import _kl_closed_apply, _noise_vector
    with torch.no_grad():
        nz = _noise_vector(lik, L).to(params.device)
        ref = _kl_closed_apply(params[:L // W], nz[:L // W], full[:, :L // W], full[:, L:L + L // W], X, spec, None)
    assert torch.isfinite(torch.stack([net, rl, nl, gp])).all()
    assert rel(gp * L, ref.sum()) < 1e-6
