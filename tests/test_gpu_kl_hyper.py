"""The exact KL backward's two hyper-parameter routes (kl_hyper.hip): the binned route (no S = K^-1 V K^-1 GEMM:
bin sums of K^-1 for the components without an id gate, the id runs' blocks for the others) against the fp64
oracle's autograd of KL_closed (elbo_functions.py:8-34) and against the S-GEMM route (LVAE_KL_HYPER=0) on the
same inputs.  Tolerance: the north star's 1e-4 relative (of the max-norm) on every raw-parameter gradient; the two
routes agree to 2e-5 (both fp32-equivalent inverses, different summation)."""
import os

import numpy as np
import pytest
import torch

from oracle import lvae_oracle as O
from test_gpu_regime_b import CFG, DEV, _random_hypers, rel, set_raw

pytestmark = pytest.mark.gpu


# Bin gates on far and near components: a Bin kernel (far) and a missing-value mask (covariate 5) on the
# components of covariate 1 -- the id x covariate-1 one (near).  Far bins: 2 + 16 + 32 (<= 128, sum nb^2 <= 4096)
HB_GATES = dict(cat_kernel=[2], bin_kernel=[4], sqexp_kernel=[0],
                cat_int_kernel=[{'cont_covariate': 0, 'cat_covariate': 3}, {'cont_covariate': 1, 'cat_covariate': 2}],
                bin_int_kernel=[], covariate_missing_val=[{'covariate': 1, 'mask': 5}])


def _run(P, L, seed, perm=None, hyper=None, cfg=CFG, T=16, xfn=None):
    """perm: row indices (a permutation, or an increasing subset: ragged subjects); xfn: edits the covariates"""
    import lvae_amd as la
    from lvae_amd.data import health_mnist_covariates
    from lvae_amd.elbo import kl_closed_hyper_log
    X = torch.tensor(health_mnist_covariates(P, T, seed=seed))
    if xfn is not None:
        X = xfn(X)
    gen = torch.Generator().manual_seed(seed)
    mu = torch.randn(P * T, L, generator=gen, dtype=torch.float64)
    lv = 0.1 * torch.randn(P * T, L, generator=gen, dtype=torch.float64)
    if perm is not None:
        X, mu, lv = X[perm], mu[perm], lv[perm]
    k = la.generate_kernel(**cfg, latent_dim=L).double()
    raw = _random_hypers(k, L, np.random.default_rng(seed))
    set_raw(k, raw)
    kd = k.to(DEV)
    lik = la.GaussianLikelihood(L, noise=1.0).to(DEV)
    mu_d, lv_d = mu.to(DEV).requires_grad_(), lv.to(DEV).requires_grad_()
    old = os.environ.get("LVAE_KL_HYPER")
    if hyper is not None:
        os.environ["LVAE_KL_HYPER"] = str(hyper)
    try:
        with kl_closed_hyper_log() as hlog:
            kl = la.KL_closed_batched(kd, X.to(DEV), lik, mu_d, lv_d)
        (kl * torch.arange(1, L + 1, device=DEV)).sum().backward()
        torch.cuda.synchronize()
    finally:
        if old is None:
            os.environ.pop("LVAE_KL_HYPER", None)
        else:
            os.environ["LVAE_KL_HYPER"] = old
    draw = torch.stack([p.grad for _, p in kd.named_parameters()], 1).cpu()
    dnoise = lik._log_noise.grad.cpu()
    return dict(X=X, mu=mu, lv=lv, raw=raw, kl=kl.detach().cpu(), draw=draw, dmu=mu_d.grad.cpu(), dlv=lv_d.grad.cpu(),
                on=int(hlog[0].item()), dnoise=dnoise)


def _oracle_grads(r, l, cfg=CFG):
    spec = O.spec_full(**cfg)
    raw = torch.tensor(r["raw"][l], requires_grad=True)
    ref = O.kl_closed(spec, O.constrain(raw), r["X"], 1.0, r["mu"][:, l], r["lv"][:, l])
    ((l + 1) * ref).backward()
    return ref.detach(), raw.grad


@pytest.mark.parametrize("P,L", [(64, 3), (13, 2), (256, 2)])  # N = 1024, 208 (ragged: padded to 256), 4096
def test_binned_hyper_route_vs_oracle(hip, P, L):
    r = _run(P, L, seed=P)
    assert r["on"] == 1, "the binned route should run on subject-contiguous integer covariates"
    for l in range(L):
        ref, g = _oracle_grads(r, l)
        assert rel(r["kl"][l], ref) < 1e-4
        e = rel(r["draw"][l], g)
        print(f"P={P} dim {l}: binned-route raw-parameter gradients rel err {e:.2e}")
        assert e < 1e-4


@pytest.mark.parametrize("P,L", [(64, 3), (256, 2)])
def test_binned_and_gemm_routes_agree(hip, P, L):
    a = _run(P, L, seed=P + 1)
    b = _run(P, L, seed=P + 1, hyper=0)
    assert a["on"] == 1 and b["on"] == 0
    assert torch.equal(a["kl"], b["kl"])  # (the forward is the same either way)
    assert torch.equal(a["dmu"], b["dmu"]) and torch.equal(a["dlv"], b["dlv"])
    e = rel(a["draw"], b["draw"])
    en = rel(a["dnoise"], b["dnoise"])
    print(f"P={P}: binned vs S-GEMM route raw gradients {e:.2e}, noise {en:.2e}")
    assert e < 2e-5 and en < 2e-5


def test_binned_route_bin_gates_vs_oracle(hip):
    """Bin gates in a far component (a Bin kernel) and in a near one (the missing-value mask on the id x
    covariate-1 component): the pair codes' Bin rule (both values 1) and the far bins' gate decode."""
    P, L = 64, 2
    r = _run(P, L, seed=11, cfg=HB_GATES)
    assert r["on"] == 1
    for l in range(L):
        ref, g = _oracle_grads(r, l, HB_GATES)
        assert rel(r["kl"][l], ref) < 1e-4
        e = rel(r["draw"][l], g)
        print(f"Bin gates dim {l}: binned-route raw-parameter gradients rel err {e:.2e}")
        assert e < 1e-4


def test_binned_route_off_for_unsorted_ids(hip):
    """Subjects interleaved (the id runs are not contiguous): the plan turns the binned route off and the S-GEMM
    route runs; gradients still match the oracle."""
    P, L, T = 16, 2, 16
    perm = torch.randperm(P * T, generator=torch.Generator().manual_seed(3))
    r = _run(P, L, seed=7, perm=perm)
    assert r["on"] == 0
    for l in range(L):
        _, g = _oracle_grads(r, l)
        assert rel(r["draw"][l], g) < 1e-4


def test_binned_route_deterministic(hip):
    a = _run(64, 2, seed=9)
    b = _run(64, 2, seed=9)
    assert torch.equal(a["draw"], b["draw"])


@pytest.mark.parametrize("group", [2, 4])
def test_binned_route_ragged_runs_across_slabs_vs_oracle(hip, group):
    """Id runs of 18..32 (group 2) or 36..64 points (group 4, up to the route's 64-point bound and its 24 near
    blocks) that start anywhere: 24 subjects of T = 16, each cut to a random prefix of 9..16 points, and every
    `group` consecutive subjects given one id (covariate 2).  Many runs then cross the slab pass's
    64-column boundaries, and its near blocks take the previous slab's columns too (kl_hyper.hip: a run ending in
    slab J that starts in slab J - 1).  ~300 points, padded to 512."""
    P, T, L = 24, 16, 2
    rng = np.random.default_rng(5)
    keep = np.concatenate([np.arange(s * T, s * T + int(rng.integers(9, T + 1))) for s in range(P)])

    def pair_ids(X):
        X = X.clone()
        X[:, 2] = torch.floor(X[:, 2] / group)
        return X

    r = _run(P, L, seed=17, perm=torch.tensor(keep), xfn=pair_ids)
    assert r["on"] == 1, "the binned route should run on these subject-contiguous runs (<= 64 points each)"
    starts = np.flatnonzero(np.diff(np.r_[-1, r["X"][:, 2].numpy()]))
    ends = np.r_[starts[1:], len(keep)] - 1
    assert any(s // 64 != e // 64 for s, e in zip(starts, ends)), "no run crosses a 64-point slab boundary"
    for l in range(L):
        ref, g = _oracle_grads(r, l)
        assert rel(r["kl"][l], ref) < 1e-4
        e = rel(r["draw"][l], g)
        print(f"ragged runs (group {group}) dim {l}: binned-route raw-parameter gradients rel err {e:.2e}")
        assert e < 1e-4
