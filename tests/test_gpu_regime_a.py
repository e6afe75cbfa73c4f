"""HIP Hensman SVI path (Regime A, fp64) against the reference's golden vectors and the oracle.

K0zz carries a 1e-6 jitter (cond ~1e8), so fp64 results depend on the op order at the cond*eps
level.  Tolerances: KL 1e-8 relative; gradients 1e-6 relative to their max-norm, except
  * gradients flowing through B_p (k1 hyper-parameters, noise): they contain Xq = c (iK H iK - iK),
    a difference of two O(|iK|) terms; two fp64 evaluations of the reference formula (autograd
    through elbo_functions.py:144-216 vs the closed-form adjoint, both on the CPU) already differ by
    1.1e-5 relative here, so the bound is 1e-4;
  * grad_H = 1/2 (iK Q iK + iK - iH) at the benign init H = K0zz, where iK - iH cancels 5 orders of
    magnitude: compared at 1e-7 of max|iH| (cond(K0zz) * eps ~ 1e-8).
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
    with torch.no_grad():
        for j, (_, p) in enumerate(module.named_parameters()):
            p.copy_(torch.as_tensor(raw_rows[:, j], dtype=p.dtype))


def build(g):
    import lvae_amd as la
    L = int(g["L"])
    k0, k1 = la.generate_kernel_batched(L, **CFG, id_covariate=2)
    set_raw(k0, g["raw0"].T)
    set_raw(k1, g["raw1"].T)
    lik = la.GaussianLikelihood(L, noise=1.0).to(DEV)
    lik.noise = torch.tensor(g["noise"][:, 0], device=DEV)
    return k0.to(DEV), k1.to(DEV), lik


@pytest.mark.parametrize("name", ["hensman_ng.npz", "hensman_ng_benign.npz", "hensman_adam.npz"])
def test_hensman_golden(hip, name):
    import lvae_amd as la
    from lvae_amd.elbo import minibatch_KLD_upper_bound
    g = golden(name)
    k0, k1, lik = build(g)
    ng = bool(g["natural_gradient"])
    X = torch.tensor(g["X_all"][g["idx"]], device=DEV)
    mu = torch.tensor(g["mu"], device=DEV, requires_grad=True)
    lv = torch.tensor(g["logv"], device=DEV, requires_grad=True)
    m = torch.tensor(g["m"], device=DEV, requires_grad=not ng)
    H = torch.tensor(g["H"], device=DEV, requires_grad=not ng)
    kld, gm, gH = minibatch_KLD_upper_bound(k0, k1, lik, int(g["L"]), m, H, X, mu, lv, torch.tensor(g["Z"], device=DEV),
                                            int(g["P_tot"]), int(g["P_b"]), int(g["T"]), ng, float(g["eps"]))
    kld.backward()
    assert rel(kld, g["kld"]) < 1e-8
    assert rel(mu.grad, g["dmu"]) < 1e-6
    assert rel(lv.grad, g["dlogv"]) < 1e-6
    d0 = torch.stack([p.grad for _, p in k0.named_parameters()])
    d1 = torch.stack([p.grad for _, p in k1.named_parameters()])
    assert rel(d0, g["draw0"]) < 1e-6
    assert rel(d1, g["draw1"]) < 1e-4
    if ng:
        assert rel(gm, g["grad_m"]) < 1e-6
        scale = max(np.abs(g["grad_H"]).max(), np.abs(np.linalg.inv(g["H"])).max())
        assert np.abs(gH.cpu().numpy() - g["grad_H"]).max() < 1e-7 * scale
    else:
        assert rel(m.grad, g["dm"]) < 1e-6
        assert rel(H.grad, g["dH"]) < 1e-6


@pytest.mark.parametrize("name", ["hensman_ng.npz", "hensman_adam.npz"])
def test_hensman_prior_split_matches_one_call(hip, name):
    """HensmanPrior (part 1 ahead of the latents, lvae_hensman_fwd_part_f64; on the caller's stream or a
    second one) + the rest = the one-call forward, bit for bit: the same kernels on the same operands,
    values and every gradient."""
    import lvae_amd as la
    from lvae_amd.elbo import minibatch_KLD_upper_bound
    g = golden(name)
    ng = bool(g["natural_gradient"])
    args = dict(P_tot=int(g["P_tot"]), P_batch=int(g["P_b"]), T=int(g["T"]), natural_gradient=ng, eps=float(g["eps"]))
    out = []
    for split in (False, True, "stream"):
        k0, k1, lik = build(g)
        X = torch.tensor(g["X_all"][g["idx"]], device=DEV)
        Z = torch.tensor(g["Z"], device=DEV)
        mu = torch.tensor(g["mu"], device=DEV, requires_grad=True)
        lv = torch.tensor(g["logv"], device=DEV, requires_grad=True)
        m = torch.tensor(g["m"], device=DEV, requires_grad=not ng)
        H = torch.tensor(g["H"], device=DEV, requires_grad=not ng)
        L = int(g["L"])
        if split:
            st = torch.cuda.Stream() if split == "stream" else None
            prior = la.HensmanPrior(k0, k1, lik, L, m, H, X, Z, **args, stream=st)
            kld, gm, gH = minibatch_KLD_upper_bound(k0, k1, lik, L, m, H, X, mu, lv, Z, **args, prior=prior)
            with pytest.raises(RuntimeError):
                minibatch_KLD_upper_bound(k0, k1, lik, L, m, H, X, mu, lv, Z, **args, prior=prior)
        else:
            kld, gm, gH = minibatch_KLD_upper_bound(k0, k1, lik, L, m, H, X, mu, lv, Z, **args)
        kld.backward()
        grads = [mu.grad, lv.grad] + [p.grad for _, p in k0.named_parameters()] + \
                [p.grad for _, p in k1.named_parameters()] + [lik._log_noise.grad]
        grads += [gm, gH] if ng else [m.grad, H.grad]
        out.append([kld.detach()] + [t.detach().clone() for t in grads])
    assert rel(out[1][0], g["kld"]) < 1e-8
    for o in out[1:]:
        for a, b in zip(out[0], o):
            assert torch.equal(a, b)


@pytest.mark.parametrize("name", ["hensman_iter_ng.npz", "hensman_iter_adam.npz"])
def test_hensman_iter_varying_T_golden(hip, name):
    """minibatch_KLD_upper_bound_iter (elbo_functions.py:219-307) on subjects of 5..16 time points,
    rows in unsorted subject order: padded [P_b, T_max] layout + masked HIP bound vs the reference."""
    from lvae_amd.elbo import minibatch_KLD_upper_bound_iter
    g = golden(name)
    k0, k1, lik = build(g)
    ng = bool(g["natural_gradient"])
    X = torch.tensor(g["X_all"][g["idx"]], device=DEV)
    mu = torch.tensor(g["mu"], device=DEV, requires_grad=True)
    lv = torch.tensor(g["logv"], device=DEV, requires_grad=True)
    m = torch.tensor(g["m"], device=DEV, requires_grad=not ng)
    H = torch.tensor(g["H"], device=DEV, requires_grad=not ng)
    kld, gm, gH = minibatch_KLD_upper_bound_iter(k0, k1, lik, int(g["L"]), m, H, X, mu, lv,
                                                 torch.tensor(g["Z"], device=DEV), int(g["P_tot"]),
                                                 int(g["P_in_batch"]), int(g["N"]), ng, int(g["id_covariate"]),
                                                 float(g["eps"]))
    kld.backward()
    assert rel(kld, g["kld"]) < 1e-8
    assert rel(mu.grad, g["dmu"]) < 1e-6
    assert rel(lv.grad, g["dlogv"]) < 1e-6
    d0 = torch.stack([p.grad for _, p in k0.named_parameters()])
    d1 = torch.stack([p.grad for _, p in k1.named_parameters()])
    assert rel(d0, g["draw0"]) < 1e-6
    assert rel(d1, g["draw1"]) < 1e-4
    if ng:
        assert rel(gm, g["grad_m"]) < 1e-6
        assert rel(gH, g["grad_H"]) < 1e-6
    else:
        assert rel(m.grad, g["dm"]) < 1e-6
        assert rel(H.grad, g["dH"]) < 1e-6


def test_hensman_iter_uniform_T_matches_fixed(hip):
    """With every subject at T rows the _iter variant equals the reference's _iter output (and the
    fixed-T bound) on the same batch."""
    from lvae_amd.elbo import minibatch_KLD_upper_bound_iter
    g = golden("hensman_ng.npz")
    k0, k1, lik = build(g)
    X = torch.tensor(g["X_all"][g["idx"]], device=DEV)
    kld, gm, gH = minibatch_KLD_upper_bound_iter(k0, k1, lik, int(g["L"]), torch.tensor(g["m"], device=DEV),
                                                 torch.tensor(g["H"], device=DEV), X,
                                                 torch.tensor(g["mu"], device=DEV), torch.tensor(g["logv"], device=DEV),
                                                 torch.tensor(g["Z"], device=DEV), int(g["P_tot"]), int(g["P_b"]),
                                                 int(g["P_tot"]) * int(g["T"]), True, 2, float(g["eps"]))
    assert rel(kld, g["kld_iter"]) < 1e-8
    assert rel(gm, g["grad_m_iter"]) < 1e-6


def test_hensman_noise_gradient(hip):
    """A trainable noise (constrain_scales=False) gets d kld / d noise = sum_p tr(dB_p) (vs oracle)."""
    import lvae_amd as la
    from lvae_amd.elbo import minibatch_KLD_upper_bound
    g = golden("hensman_adam.npz")
    k0, k1, lik = build(g)
    L, M = int(g["L"]), int(g["M"])
    X = torch.tensor(g["X_all"][g["idx"]])
    Z = torch.tensor(g["Z"])
    args = (torch.tensor(g["m"]), torch.tensor(g["H"]))
    kld, _, _ = minibatch_KLD_upper_bound(k0, k1, lik, L, args[0].to(DEV), args[1].to(DEV), X.to(DEV),
                                          torch.tensor(g["mu"], device=DEV), torch.tensor(g["logv"], device=DEV),
                                          Z.to(DEV), int(g["P_tot"]), int(g["P_b"]), int(g["T"]), False, 1e-6)
    kld.backward()
    s0, s1 = O.spec_split(**CFG, id_covariate=2)
    nz = torch.tensor(g["noise"][:, 0], requires_grad=True)
    ref, _, _ = O.hensman_kld(s0, O.constrain(torch.tensor(g["raw0"].T.copy())), s1,
                              O.constrain(torch.tensor(g["raw1"].T.copy())), nz, args[0], args[1], X,
                              torch.tensor(g["mu"]), torch.tensor(g["logv"]), Z, int(g["P_tot"]), int(g["P_b"]),
                              int(g["T"]), False, 1e-6)
    ref.backward()
    # lik noise = exp(m + softplus(raw - m)) -> chain rule factor
    with torch.no_grad():
        raw = lik._log_noise.detach().cpu()
        dnoise_draw = torch.sigmoid(raw + 16.0) * torch.exp(-16.0 + torch.nn.functional.softplus(raw + 16.0))
    assert rel(lik._log_noise.grad.cpu(), nz.grad * dnoise_draw) < 1e-4


def test_natural_gradient_update(hip):
    from lvae_amd.elbo import natural_gradient_update
    g = golden("hensman_ng_benign.npz")
    m, H = torch.tensor(g["m"]), torch.tensor(g["H"])
    gm, gH = torch.tensor(g["grad_m"]), torch.tensor(g["grad_H"])
    m_ref, H_ref = O.natural_gradient_update(m, H, gm, gH, 0.01)
    m2, H2 = natural_gradient_update(m.to(DEV), H.to(DEV), gm.to(DEV), gH.to(DEV), 0.01)
    assert rel(H2, H_ref) < 1e-7
    assert rel(m2, m_ref) < 1e-7


def test_natural_gradient_update_reuses_forward_inverse(hip):
    """After the forward on H, the update reuses the workspace's H^-1 (no second inversion); the
    result equals the fresh-inversion path and the oracle.  A changed H disables the reuse."""
    from lvae_amd.elbo import minibatch_KLD_upper_bound, natural_gradient_update
    g = golden("hensman_ng.npz")
    k0, k1, lik = build(g)
    X = torch.tensor(g["X_all"][g["idx"]], device=DEV)
    m = torch.tensor(g["m"], device=DEV)
    H = torch.tensor(g["H"], device=DEV)
    with torch.no_grad():
        _, gm, gH = minibatch_KLD_upper_bound(k0, k1, lik, int(g["L"]), m, H, X, torch.tensor(g["mu"], device=DEV),
                                              torch.tensor(g["logv"], device=DEV), torch.tensor(g["Z"], device=DEV),
                                              int(g["P_tot"]), int(g["P_b"]), int(g["T"]), True, float(g["eps"]))
    assert getattr(gH, "_lvae_iH", None) is not None
    m_a, H_a = natural_gradient_update(m, H, gm, gH, 0.01)          # reuse path
    m_b, H_b = natural_gradient_update(m, H, gm, gH.clone(), 0.01)  # fresh inversion
    m_ref, H_ref = O.natural_gradient_update(m.cpu(), H.cpu(), gm.cpu(), gH.cpu(), 0.01)
    assert rel(H_a, H_b) < 1e-9 and rel(m_a, m_b) < 1e-7
    assert rel(H_a, H_ref) < 1e-7 and rel(m_a, m_ref) < 1e-6
    H.mul_(1.0)  # bumps H's version: the cached inverse must not be used any more
    m_c, H_c = natural_gradient_update(m, H, gm, gH, 0.01)
    assert rel(H_c, H_b) < 1e-12


def test_spd_inv_small_and_gemm(hip):
    import lvae_amd as la
    P = la._lib
    lib = hip
    gen = torch.Generator().manual_seed(3)
    for n, b in [(120, 3), (16, 7), (1, 2), (128, 1)]:
        X = torch.randn(b, n, n, generator=gen, dtype=torch.float64)
        A = X @ X.transpose(1, 2) + n * torch.eye(n, dtype=torch.float64)
        Ad = A.to(DEV)
        Ai = torch.empty_like(Ad)
        ld = torch.empty(b, dtype=torch.float64, device=DEV)
        info = torch.empty(b, dtype=torch.int32, device=DEV)
        P.check(lib.lvae_spd_inv_small_f64(n, b, P.ptr(Ad), n * n, P.ptr(Ai), n * n, P.ptr(ld), P.ptr(info),
                                           P.stream_ptr()), "spd_inv")
        assert int(info.abs().sum()) == 0
        assert rel(Ai, torch.linalg.inv(A)) < 1e-12
        assert rel(ld, torch.logdet(A)) < 1e-12
    # gemm: C = 0.5 A^T B + 2 C over a (2, 3) batch with broadcast B
    m_, n_, k_ = 37, 45, 70
    A = torch.randn(2, 3, k_, m_, generator=gen, dtype=torch.float64)
    B = torch.randn(n_, k_, generator=gen, dtype=torch.float64)
    C = torch.randn(2, 3, m_, n_, generator=gen, dtype=torch.float64)
    ref = 0.5 * A.transpose(-1, -2) @ B.T + 2 * C
    Ad, Bd, Cd = A.to(DEV), B.to(DEV), C.to(DEV)
    P.check(lib.lvae_gemm_small_f64(1, 1, m_, n_, k_, 0.5, P.ptr(Ad), m_, 3 * k_ * m_, k_ * m_, P.ptr(Bd), k_, 0, 0,
                                    2.0, P.ptr(Cd), n_, 3 * m_ * n_, m_ * n_, 2, 3, P.stream_ptr()), "gemm")
    assert rel(Cd, ref) < 1e-13
    # non-PD detection
    A = -torch.eye(4, dtype=torch.float64).unsqueeze(0).to(DEV)
    Ai = torch.empty_like(A)
    ld = torch.empty(1, dtype=torch.float64, device=DEV)
    info = torch.empty(1, dtype=torch.int32, device=DEV)
    lib.lvae_spd_inv_small_f64(4, 1, P.ptr(A), 16, P.ptr(Ai), 16, P.ptr(ld), P.ptr(info), P.stream_ptr())
    assert int(info[0]) == 1


def test_dp_contract_simulated_ranks(hip):
    """Two simulated ranks (sequential, one GPU): the mean of per-rank Adam gradients and the SUM of
    per-rank natural-gradient directions (ng_prior_share = 1/2) equal the union batch's."""
    import lvae_amd as la
    from lvae_amd.elbo import minibatch_KLD_upper_bound
    from lvae_amd.data import health_mnist_covariates
    L, M, T, P_tot = 3, 24, 16, 40
    X = torch.tensor(health_mnist_covariates(P_tot, T, seed=9), device=DEV)
    gen = torch.Generator().manual_seed(2)
    mu = torch.randn(P_tot * T, L, generator=gen, dtype=torch.float64).to(DEV)
    lv = (0.1 * torch.randn(P_tot * T, L, generator=gen, dtype=torch.float64)).to(DEV)
    N = P_tot * T
    z = torch.stack([torch.cat([X[0:M // 2], X[N // 2:N // 2 + M // 2]])] * L)
    k0, k1 = la.generate_kernel_batched(L, **CFG, id_covariate=2)
    k0, k1 = k0.to(DEV), k1.to(DEV)
    lik = la.GaussianLikelihood(L, noise=1.0, constrain=False).to(DEV)
    with torch.no_grad():
        H = k0(z, z).evaluate() + 1e-3 * torch.eye(M, dtype=torch.float64, device=DEV)
    m = torch.randn(L, M, 1, generator=gen, dtype=torch.float64).to(DEV)
    subjects = [5, 17, 2, 30, 11, 8]
    rows = lambda ss: torch.cat([torch.arange(s * T, (s + 1) * T) for s in ss]).to(DEV)

    def run(ss, share):
        for p in list(k0.parameters()) + list(k1.parameters()):
            p.grad = None
        r = rows(ss)
        kld, gm, gH = minibatch_KLD_upper_bound(k0, k1, lik, L, m, H, X[r], mu[r], lv[r], z, P_tot, len(ss), T,
                                                True, 1e-6, ng_prior_share=share)
        kld.backward()
        return (kld.detach(), gm, gH, [p.grad.clone() for p in list(k0.parameters()) + list(k1.parameters())])

    u = run(subjects, 1.0)
    a = run(subjects[:3], 0.5)
    b = run(subjects[3:], 0.5)
    assert rel((a[0] + b[0]) / 2, u[0]) < 1e-10
    for ga, gb, gu in zip(a[3], b[3], u[3]):
        assert rel((ga + gb) / 2, gu) < 1e-8
    assert rel(a[1] + b[1], u[1]) < 1e-8
    assert rel(a[2] + b[2], u[2]) < 1e-8


def test_hensman_step_vs_oracle(hip):
    """One full hensman_training batch (ConvVAE fwd/bwd, bound, Adam, natural-gradient update;
    training.py:91-135) against the oracle step: fp32 conv vs fp64 reference -> 1e-4."""
    import lvae_amd as la
    from lvae_amd.steps import HensmanStep
    from lvae_amd.vae import ConvVAE
    from lvae_amd.data import health_mnist_batch
    L, M, T, P_tot, P_b = 4, 40, 16, 32, 5
    img, mask, X = health_mnist_batch(P_tot, T, seed=4, dtype=torch.float64)
    N = P_tot * T
    z = torch.stack([torch.cat([X[0:M // 2], X[N // 2:N // 2 + M // 2]])] * L)
    ref_vae = O.ConvVAE(L).double()
    ref_vae.load_state_dict(O.vae_weights(ref_vae, 11))
    vae = ConvVAE(L, 1296, p_input=0.0, p=0.0).double()
    vae.load_state_dict(ref_vae.state_dict())
    vae = vae.float().to(DEV)
    s0, s1 = O.spec_split(**CFG, id_covariate=2)
    k0, k1 = la.generate_kernel_batched(L, **CFG, id_covariate=2)
    raw0 = torch.stack([p.detach().clone() for _, p in k0.named_parameters()], 1).requires_grad_()
    raw1 = torch.stack([p.detach().clone() for _, p in k1.named_parameters()], 1).requires_grad_()
    k0, k1 = k0.to(DEV), k1.to(DEV)
    lik = la.GaussianLikelihood(L, noise=1.0, constrain=False).to(DEV)
    with torch.no_grad():
        H = O.gram(s0, O.constrain(raw0), z, z) + 1e-6 * torch.eye(M, dtype=torch.float64)
    m = torch.zeros(L, M, 1, dtype=torch.float64)
    rows = torch.cat([torch.arange(s * T, (s + 1) * T) for s in [3, 9, 20, 1, 27]])
    eps = torch.randn(P_b * T, L, generator=torch.Generator().manual_seed(0), dtype=torch.float64)
    # oracle step (no optimiser: compare the losses and the natural-gradient update)
    loss, recon, kld, m_ref, H_ref = O.hensman_step(ref_vae, s0, raw0, s1, raw1, torch.ones(L), m, H, img[rows],
                                                    mask[rows], X[rows], z, eps, P_tot, T, 0.15, 0.01)
    opt = torch.optim.SGD(list(vae.parameters()) + list(k0.parameters()) + list(k1.parameters()), lr=0.0)
    step = HensmanStep(vae, k0, k1, lik, opt, m.to(DEV), H.to(DEV), z.to(DEV), P_tot, T)
    net, rl, _, kl = step(img[rows].float().to(DEV), mask[rows].float().to(DEV), X[rows].to(DEV),
                          eps.float().to(DEV))
    assert rel(net, loss) < 1e-4
    assert rel(rl, recon) < 1e-4
    assert rel(kl, kld) < 1e-4
    assert rel(step.m, m_ref) < 1e-4
    assert rel(step.H, H_ref) < 1e-4
    d0 = torch.stack([p.grad for _, p in k0.named_parameters()], 1)
    assert rel(d0, raw0.grad) < 1e-4


def test_batch_predict_varying_T_golden(hip):
    """utils.batch_predict_varying_T (utils.py:115-211) through lvae_predict_f64: 12 prediction
    subjects of 5..16 points, 4 test subjects (rows in unsorted subject order)."""
    from lvae_amd.predict import batch_predict_varying_T
    g = golden("predict_varying.npz")
    k0, k1, lik = build(g)
    X = g["X_all"]
    zp = batch_predict_varying_T(int(g["L"]), k0, k1, lik, torch.tensor(X[g["pidx"]], device=DEV),
                                 torch.tensor(X[g["tidx"]], device=DEV), torch.tensor(g["mu"], device=DEV),
                                 torch.tensor(g["Z"], device=DEV), int(g["id_covariate"]), float(g["eps"]))
    assert tuple(zp.shape) == g["Z_pred"].shape
    # Z_pred applies K0zz^-1 (cond ~1e8 with the 1e-6 jitter) and H^-1: the reference LU-solves
    # (torch.solve), the HIP path multiplies by the Cholesky-based inverse -> cond * eps ~ 1e-7
    assert rel(zp, g["Z_pred"]) < 1e-6


def test_gpapprox_elbo_and_dubo_golden(hip):
    """Full-batch GPapprox ELBO (elbo_functions.py:36-84) and DUBO (86-142) of one latent dim:
    values and autograd gradients (y / mu / log_v and raw kernel parameters) vs the reference."""
    import lvae_amd as la
    g = golden("gpapprox.npz")
    P, T = int(g["P"]), int(g["T"])
    X, Z = torch.tensor(g["X"], device=DEV), torch.tensor(g["Z"], device=DEV)

    def kernels():
        k0, k1 = la.generate_kernel_batched(1, **CFG, id_covariate=2)
        set_raw(k0, g["raw0"].T)
        set_raw(k1, g["raw1"].T)
        lik = la.GaussianLikelihood(1, noise=float(g["noise"])).to(DEV)
        return k0.to(DEV), k1.to(DEV), lik

    k0, k1, lik = kernels()
    y = torch.tensor(g["y"], device=DEV, requires_grad=True)
    el = la.elbo(k0, k1, lik, X, y, Z, P, T, float(g["eps"]))
    el.backward()
    assert rel(el, g["elbo"]) < 1e-9
    assert rel(y.grad, g["elbo_dy"]) < 1e-7
    assert rel(torch.cat([p.grad for _, p in k0.named_parameters()]), g["elbo_draw0"][:, 0]) < 1e-6
    assert rel(torch.cat([p.grad for _, p in k1.named_parameters()]), g["elbo_draw1"][:, 0]) < 1e-6
    k0, k1, lik = kernels()
    mu = torch.tensor(g["mu"], device=DEV, requires_grad=True)
    lv = torch.tensor(g["logv"], device=DEV, requires_grad=True)
    du = la.deviance_upper_bound(k0, k1, lik, X, mu, lv, Z, P, T, float(g["eps"]))
    du.backward()
    assert rel(du, g["dubo"]) < 1e-9
    assert rel(mu.grad, g["dubo_dmu"]) < 1e-7
    assert rel(lv.grad, g["dubo_dlogv"]) < 1e-7
    assert rel(torch.cat([p.grad for _, p in k0.named_parameters()]), g["dubo_draw0"][:, 0]) < 1e-6
    assert rel(torch.cat([p.grad for _, p in k1.named_parameters()]), g["dubo_draw1"][:, 0]) < 1e-6
    # validation_dubo with batched kernels == sum of per-dim DUBOs (here one dim)
    k0, k1, lik = kernels()
    vd = la.validation_dubo(1, k0, k1, lik, X, torch.tensor(g["mu"], device=DEV)[:, None],
                            torch.tensor(g["logv"], device=DEV)[:, None], Z[None], P, T, float(g["eps"]))
    assert rel(vd, g["dubo"]) < 1e-9


def _c4_problem(seed, benign):
    """C3/C4 Regime A shapes: L = 16, M = 120 (the hard-coded inducing rows of LVAE.py:199-203 at
    N >= 2060), P_b = 5 subjects x T = 16 of P_tot = 256 (N = 4096); random per-dim hyper-parameters;
    (m, H) the LVAE.py:222-226 draw (m ~ N(0,1), H = X X^T / 100) or the benign (0, K0zz)."""
    import lvae_amd as la
    from lvae_amd.data import health_mnist_covariates
    L, M, T, P_tot = 16, 120, 16, 256
    N = P_tot * T
    X = torch.tensor(health_mnist_covariates(P_tot, T, seed=seed))
    gen = torch.Generator().manual_seed(seed)
    mu = torch.randn(N, L, generator=gen, dtype=torch.float64)
    lv = 0.1 * torch.randn(N, L, generator=gen, dtype=torch.float64)
    z = torch.stack([torch.cat([X[0:M // 2], X[N // 2:N // 2 + M // 2]])] * L)
    k0, k1 = la.generate_kernel_batched(L, **CFG, id_covariate=2)
    rng = np.random.default_rng(seed)
    raw0 = np.log(rng.uniform(0.5, 2.0, (L, len(list(k0.parameters())))))
    raw1 = np.log(rng.uniform(0.5, 2.0, (L, len(list(k1.parameters())))))
    set_raw(k0, raw0)
    set_raw(k1, raw1)
    s0, s1 = O.spec_split(**CFG, id_covariate=2)
    if benign:
        m = torch.zeros(L, M, 1, dtype=torch.float64)
        H = O.gram(s0, O.constrain(torch.tensor(raw0)), z, z) + 1e-6 * torch.eye(M, dtype=torch.float64)
    else:
        m = torch.randn(L, M, 1, generator=gen, dtype=torch.float64)
        Xh = torch.randn(L, M, M, generator=gen, dtype=torch.float64) / 10
        H = Xh @ Xh.transpose(1, 2)
    lik = la.GaussianLikelihood(L, noise=1.0).to(DEV)
    return dict(L=L, M=M, T=T, P_tot=P_tot, X=X, mu=mu, lv=lv, z=z, k0=k0.to(DEV), k1=k1.to(DEV), lik=lik,
                raw0=raw0, raw1=raw1, s0=s0, s1=s1, m=m, H=H)


@pytest.mark.parametrize("benign", [False, True])
def test_hensman_c4_shapes_vs_oracle(hip, benign):
    """minibatch_KLD_upper_bound at the C3 / C4 Regime A shapes (L = 16, M = 120, P_b = 5, T = 16)
    vs the fp64 oracle: the bound, grad_m / grad_H and every autograd gradient.

    K0zz carries the 1e-6 jitter (cond ~1e8..1e10 at M = 120 with random hyper-parameters) and the
    k1 / noise gradients contain Xq = c (iK H iK - iK), a difference of O(|iK|^2) terms, so fp64
    itself determines them only to a few digits.  The test measures that: the oracle formula is
    evaluated twice in fp64 -- LAPACK on the CPU and rocSOLVER / rocBLAS on the GPU -- and each
    quantity must match within max(base, 10 x the two fp64 oracles' own spread); base = 1e-8 (bound),
    1e-6 (gradients), as the golden tests."""
    from lvae_amd.elbo import minibatch_KLD_upper_bound
    c = _c4_problem(41, benign)
    L, M, T, P_tot = c["L"], c["M"], c["T"], c["P_tot"]
    subjects = [7, 130, 64, 201, 12]
    rows = torch.cat([torch.arange(s * T, (s + 1) * T) for s in subjects])
    mu = c["mu"][rows].to(DEV).requires_grad_()
    lv = c["lv"][rows].to(DEV).requires_grad_()
    kld, gm, gH = minibatch_KLD_upper_bound(c["k0"], c["k1"], c["lik"], L, c["m"].to(DEV), c["H"].to(DEV),
                                            c["X"][rows].to(DEV), mu, lv, c["z"].to(DEV), P_tot, 5, T, True, 1e-6)
    kld.backward()
    hip_vals = dict(kld=kld, dmu=mu.grad, dlogv=lv.grad,
                    draw0=torch.stack([p.grad for _, p in c["k0"].named_parameters()], 1),
                    draw1=torch.stack([p.grad for _, p in c["k1"].named_parameters()], 1), gm=gm, gH=gH)

    def oracle(dev):
        r0 = torch.tensor(c["raw0"], device=dev, requires_grad=True)
        r1 = torch.tensor(c["raw1"], device=dev, requires_grad=True)
        mu_r = c["mu"][rows].to(dev).requires_grad_()
        lv_r = c["lv"][rows].to(dev).requires_grad_()
        ref, gm_r, gH_r = O.hensman_kld(c["s0"], O.constrain(r0), c["s1"], O.constrain(r1),
                                        torch.ones(L, dtype=torch.float64, device=dev), c["m"].to(dev),
                                        c["H"].to(dev), c["X"][rows].to(dev), mu_r, lv_r, c["z"].to(dev), P_tot, 5, T,
                                        True, 1e-6)
        ref.backward()
        return dict(kld=ref, dmu=mu_r.grad, dlogv=lv_r.grad, draw0=r0.grad, draw1=r1.grad, gm=gm_r, gH=gH_r)

    cpu, gpu = oracle("cpu"), oracle(DEV)
    base = dict(kld=1e-8, dmu=1e-6, dlogv=1e-6, draw0=1e-6, draw1=1e-6, gm=1e-6, gH=1e-6)
    for key, b in base.items():
        err, spread = rel(hip_vals[key], cpu[key]), rel(gpu[key], cpu[key])
        print(f"C4 Regime A {'benign' if benign else 'LVAE-init'} {key}: err {err:.2e}, fp64 oracle spread {spread:.2e}")
        assert err < max(b, 10 * spread), key


def test_dp_contract_c4_eight_ranks(hip):
    """The C4 data-parallel contract at its own shapes: 8 ranks x P_b = 5 subjects, simulated
    sequentially on one GPU with ng_prior_share = 1/8.  The mean over ranks of the bound and of the
    Adam gradients and the SUM of the natural-gradient directions equal one process with the 40-subject
    union batch; each rank's mu / logv gradient rows equal 8x the union's rows.
    The jitter is 1e-3 here (the reference's 1e-6 makes cond(K0zz) ~1e8..1e10, and then two fp64
    evaluations of one bound already differ in the 9th digit -- test_hensman_c4_shapes_vs_oracle);
    the identity itself holds for any jitter, and is checked to near round-off this way."""
    from lvae_amd.elbo import minibatch_KLD_upper_bound
    c = _c4_problem(43, False)
    L, T, P_tot, W, P_b = c["L"], c["T"], c["P_tot"], 8, 5
    perm = torch.randperm(P_tot, generator=torch.Generator().manual_seed(5))[:W * P_b].tolist()
    m, H, z = c["m"].to(DEV), c["H"].to(DEV), c["z"].to(DEV)
    params = list(c["k0"].parameters()) + list(c["k1"].parameters())

    def run(subjects, share):
        for p in params:
            p.grad = None
        rows = torch.cat([torch.arange(s * T, (s + 1) * T) for s in subjects])
        mu = c["mu"][rows].to(DEV).requires_grad_()
        kld, gm, gH = minibatch_KLD_upper_bound(c["k0"], c["k1"], c["lik"], L, m, H, c["X"][rows].to(DEV), mu,
                                                c["lv"][rows].to(DEV), z, P_tot, len(subjects), T, True, 1e-3,
                                                ng_prior_share=share)
        kld.backward()
        return kld.detach(), gm, gH, [p.grad.clone() for p in params], mu.grad.detach()

    u = run(perm, 1.0)
    ranks = [run(perm[r * P_b:(r + 1) * P_b], 1.0 / W) for r in range(W)]
    errs = dict(kld=rel(sum(r[0] for r in ranks) / W, u[0]),
                grads=max(rel(sum(r[3][i] for r in ranks) / W, u[3][i]) for i in range(len(params))),
                gm=rel(sum(r[1] for r in ranks), u[1]), gH=rel(sum(r[2] for r in ranks), u[2]),
                dmu=rel(torch.cat([r[4] for r in ranks]) / W, u[4]))
    print("8-rank DP contract errors:", errs)
    assert errs["kld"] < 1e-10 and errs["dmu"] < 1e-10
    assert errs["grads"] < 1e-8 and errs["gm"] < 1e-8 and errs["gH"] < 1e-8


def test_graphed_hensman_step_matches_eager(hip):
    """The HIP-graph replay of the Hensman step (GraphedStep: forward, backward, capturable Adam and
    the in-place natural-gradient update in one graph) reproduces the eager step, step after step,
    with a new batch gathered into the static inputs before every replay."""
    import lvae_amd as la
    from lvae_amd.data import health_mnist_batch
    from lvae_amd.steps import GraphedStep, HensmanStep
    from lvae_amd.vae import ConvVAE
    L, M, T, P, P_b = 4, 40, 16, 32, 5
    img, mask, X = health_mnist_batch(P, T, seed=6, device=DEV)
    N = P * T
    z = torch.stack([torch.cat([X[0:M // 2], X[N // 2:N // 2 + M // 2]])] * L)
    batches = [torch.cat([torch.arange(s * T, (s + 1) * T) for s in ss]).to(DEV)
               for ss in ([3, 9, 20, 1, 27], [4, 11, 30, 0, 7], [2, 5, 8, 13, 21], [6, 10, 12, 14, 15])]
    eps = torch.randn(P_b * T, L, generator=torch.Generator().manual_seed(0)).to(DEV)

    def make():
        torch.manual_seed(3)
        vae = ConvVAE(L, 1296, p_input=0.0, p=0.0).to(DEV)
        k0, k1 = la.generate_kernel_batched(L, **CFG, id_covariate=2)
        k0, k1 = k0.to(DEV), k1.to(DEV)
        lik = la.GaussianLikelihood(L, noise=1.0, constrain=False).to(DEV)
        with torch.no_grad():
            H = k0(z, z).evaluate() + 1e-6 * torch.eye(M, dtype=torch.float64, device=DEV)
        m = torch.zeros(L, M, 1, dtype=torch.float64, device=DEV)
        opt = torch.optim.Adam(list(k0.parameters()) + list(k1.parameters()) + list(vae.parameters()), lr=1e-3,
                               capturable=True)
        return HensmanStep(vae, k0, k1, lik, opt, m, H, z, P, T), vae, k0

    la.set_sync_checks(False)
    try:
        eager, vae_e, k0_e = make()
        eager(img[batches[0]], mask[batches[0]], X[batches[0]], eps)  # = the graph's warm-up step
        outs_e = [[float(v) for v in eager(img[b], mask[b], X[b], eps)] for b in batches]
        graph_step, vae_g, k0_g = make()
        s = (img[batches[0]].clone(), mask[batches[0]].clone(), X[batches[0]].clone(), eps)
        g = GraphedStep(graph_step, s, warmup=1)
        outs_g = []
        for b in batches:
            torch.index_select(img, 0, b, out=s[0])
            torch.index_select(mask, 0, b, out=s[1])
            torch.index_select(X, 0, b, out=s[2])
            outs_g.append([float(v) for v in g()])
        g.check()
    finally:
        la.set_sync_checks(True)
    for a, b in zip(outs_e, outs_g):
        assert np.allclose(a, b, rtol=1e-6), (a, b)
    assert rel(graph_step.m, eager.m) < 1e-6 and rel(graph_step.H, eager.H) < 1e-6
    for (n, p), (_, q) in zip(k0_g.named_parameters(), k0_e.named_parameters()):
        assert rel(p, q) < 1e-9, n


VAR_CFG = dict(cat_kernel=[2, 3], bin_kernel=[5], sqexp_kernel=[0],
               cat_int_kernel=[{'cont_covariate': 0, 'cat_covariate': 2},
                               {'cont_covariate': 1, 'cat_covariate': 4}],
               bin_int_kernel=[{'cont_covariate': 0, 'bin_covariate': 4}],
               covariate_missing_val=[{'covariate': 0, 'mask': 6}, {'covariate': 3, 'mask': 7}])


def test_hensman_kernel_variants_golden(hip):
    """The Hensman bound with bin / bin x RBF / masked kernels (kernel_variants_hensman.npz): the
    three Grams of the call convention (elbo_functions.py:171-174) and the bound + gradients."""
    import lvae_amd as la
    from lvae_amd.elbo import minibatch_KLD_upper_bound
    g = golden("kernel_variants_hensman.npz")
    L, P_b, T = int(g["L"]), int(g["P_b"]), int(g["T"])
    k0, k1 = la.generate_kernel_batched(L, **VAR_CFG, id_covariate=2)
    set_raw(k0, g["raw0"].T)
    set_raw(k1, g["raw1"].T)
    k0, k1 = k0.to(DEV), k1.to(DEV)
    lik = la.GaussianLikelihood(L, noise=1.0).to(DEV)
    lik.noise = torch.tensor(g["noise"][:, 0], device=DEV)
    X = torch.tensor(g["X_all"][g["idx"]], device=DEV)
    Z = torch.tensor(g["Z"], device=DEV)
    with torch.no_grad():
        xs = X.reshape(P_b, 1, T, -1).expand(P_b, L, T, X.shape[1])
        assert rel(k0(X, Z).evaluate(), g["K0xz"]) < 1e-13
        assert rel(k0(Z, Z).evaluate(), g["K0zz"]) < 1e-13
        assert rel(k1(xs, xs).evaluate(), g["K1_st"]) < 1e-13
    mu = torch.tensor(g["mu"], device=DEV, requires_grad=True)
    lv = torch.tensor(g["logv"], device=DEV, requires_grad=True)
    kld, gm, gH = minibatch_KLD_upper_bound(k0, k1, lik, L, torch.tensor(g["m"], device=DEV),
                                            torch.tensor(g["H"], device=DEV), X, mu, lv, Z, int(g["P_tot"]), P_b, T,
                                            True, float(g["eps"]))
    kld.backward()
    errs = {"kld": rel(kld, g["kld"]), "dmu": rel(mu.grad, g["dmu"]), "dlogv": rel(lv.grad, g["dlogv"]),
            "draw0": rel(torch.stack([p.grad for _, p in k0.named_parameters()]), g["draw0"]),
            "draw1": rel(torch.stack([p.grad for _, p in k1.named_parameters()]), g["draw1"]),
            "grad_m": rel(gm, g["grad_m"]), "grad_H": rel(gH, g["grad_H"])}
    print("hensman kernel variants rel errors:", {k: f"{v:.2e}" for k, v in errs.items()})
    assert errs["kld"] < 1e-8
    for k in ("dmu", "dlogv", "draw0", "grad_m", "grad_H"):
        assert errs[k] < 1e-6, (k, errs[k])
    assert errs["draw1"] < 1e-4


class _FixtureImages:
    """A device-resident dataset over the fixture's arrays with the HealthMNISTDatasetConv batch()
    interface (digit = uint8 / 255, label, mask), in fp64 as the reference's training casts them."""

    def __init__(self, g):
        self.pix = torch.tensor(g["pix"], device=DEV)
        self.msk = torch.tensor(g["msk"], device=DEV)
        self.lab = torch.tensor(g["X"], device=DEV)

    def __len__(self):
        return self.lab.shape[0]

    def batch(self, idx):
        idx = torch.as_tensor(idx, dtype=torch.int64, device=DEV)
        return {"idx": idx, "digit": self.pix.index_select(0, idx).to(torch.float64) / 255.0,
                "label": self.lab.index_select(0, idx), "mask": self.msk.index_select(0, idx).to(torch.float64)}


def test_hensman_training_two_epochs_vs_reference(hip):
    """Two epochs of the reference's training.hensman_training (hensman_training_2ep.npz) replayed
    through the product stack: the drop-in SubjectSampler under the same np.random.seed, torch's
    BatchSampler, the drop-in HensmanDataLoader (device batches), lvae_amd.HensmanStep (HIP bound,
    natural-gradient update) and Adam over the same parameter set.  The ConvVAE runs in fp64 here
    (the reference's dtype) so the comparison is at fp64 tolerances: per-step KL bound and recon
    sums, and the final (m, H), kernel and network parameters."""
    import lvae_amd as la
    from torch.utils.data.sampler import BatchSampler
    from dropin.utils import HensmanDataLoader, SubjectSampler
    from lvae_amd.steps import HensmanStep
    from lvae_amd.vae import ConvVAE
    g = golden("hensman_training_2ep.npz")
    P, T, L, P_b = int(g["P"]), int(g["T"]), int(g["L"]), int(g["P_b"])
    ds = _FixtureImages(g)
    ref_vae = O.ConvVAE(L).double()
    ref_vae.load_state_dict(O.vae_weights(ref_vae, int(g["seed"])))
    vae = ConvVAE(L, 1296, p_input=0.0, p=0.0).double()
    vae.load_state_dict(ref_vae.state_dict())
    vae = vae.to(DEV)
    k0, k1 = la.generate_kernel_batched(L, **CFG, id_covariate=2)
    set_raw(k0, g["raw0"].T)
    set_raw(k1, g["raw1"].T)
    k0, k1 = k0.to(DEV), k1.to(DEV)
    lik = la.GaussianLikelihood(L, noise=1.0, constrain=False).to(DEV)
    opt = torch.optim.Adam([{"params": k0.parameters()}, {"params": k1.parameters()},
                            {"params": vae.parameters()}], lr=1e-3)
    step = HensmanStep(vae, k0, k1, lik, opt, torch.tensor(g["m0"], device=DEV), torch.tensor(g["H0"], device=DEV),
                       torch.tensor(g["Z"], device=DEV), P, T, weight=0.15)
    np.random.seed(int(g["seed"]))
    loader = HensmanDataLoader(ds, BatchSampler(SubjectSampler(ds, P, T), P_b * T, drop_last=False))
    s = 0
    for e in range(int(g["epochs"])):
        for j, b in enumerate(loader):
            rows = b["idx"]
            pb = len(rows) // T
            # the reference's subject order, bit-exact (np.random.shuffle under the same seed)
            assert np.array_equal(rows[::T].cpu().numpy() // T, g["perms"][e][j * P_b:j * P_b + pb])
            eps = torch.tensor(g["eps"][s][:len(rows)], device=DEV)
            net, recon, nll, kld = step(b["digit"], b["mask"], b["label"], eps)
            assert rel(kld * L, g["step_kld"][s]) < 1e-7, s
            assert rel(recon * pb / P, g["step_recon"][s]) < 1e-9, s
            assert rel(nll * pb / P, g["step_nll"][s]) < 1e-9, s
            s += 1
    assert s == len(g["step_kld"])
    assert rel(step.m, g["m_final"]) < 1e-6
    assert rel(step.H, g["H_final"]) < 1e-6
    assert rel(torch.stack([p for _, p in k0.named_parameters()]), g["raw0_final"]) < 1e-8
    assert rel(torch.stack([p for _, p in k1.named_parameters()]), g["raw1_final"]) < 1e-8
    sd = dict(vae.named_parameters())
    for k in ("conv1.weight", "fc211.bias", "deconv2.weight", "_log_vy"):
        assert rel(sd[k], g["vae_" + k]) < 1e-8, k
    assert rel(sd["fc1.weight"].sum(1), g["vae_fc1_rowsum"]) < 1e-8
