"""Data-parallel plumbing on CPU with gloo, world_size 2 (the GPU path uses the same code over RCCL):
the per-step gradient all-reduce, the SUM reduce of the natural-gradient directions, and the
subject sharding of a Hensman epoch (each global step = world * P_b consecutive subjects)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from lvae_amd.distributed import GradAllReduce, allreduce_tensors
        from oracle import lvae_oracle as O
        from lvae_amd.data import health_mnist_covariates
        # --- Hensman estimator: mean over ranks of per-rank grads == union-batch grads ---
        cfg = dict(cat_kernel=[2], bin_kernel=[], sqexp_kernel=[0],
                   cat_int_kernel=[{'cont_covariate': 0, 'cat_covariate': 2},
                                   {'cont_covariate': 0, 'cat_covariate': 3},
                                   {'cont_covariate': 1, 'cat_covariate': 4}],
                   bin_int_kernel=[], covariate_missing_val=[])
        s0, s1 = O.spec_split(**cfg, id_covariate=2)
        P_tot, T, L, M, P_b = 12, 8, 2, 10, 2
        X = torch.tensor(health_mnist_covariates(P_tot, T, seed=5))
        gen = torch.Generator().manual_seed(0)
        mu_all = torch.randn(P_tot * T, L, generator=gen, dtype=torch.float64)
        lv_all = 0.1 * torch.randn(P_tot * T, L, generator=gen, dtype=torch.float64)
        z = torch.stack([torch.cat([X[:8], X[(P_tot - 1) * T:(P_tot - 1) * T + 2]])] * L)
        m = torch.randn(L, M, 1, generator=gen, dtype=torch.float64)
        Hr = torch.randn(L, M, M, generator=gen, dtype=torch.float64) / 5
        H = Hr @ Hr.transpose(1, 2) + 0.1 * torch.eye(M, dtype=torch.float64)
        subjects = [3, 7, 1, 10]  # global batch of world * P_b subjects
        mine = subjects[rank * P_b:(rank + 1) * P_b]
        rows = torch.cat([torch.arange(s * T, (s + 1) * T) for s in mine])
        raw0 = torch.zeros(L, O.n_params(s0), dtype=torch.float64, requires_grad=True)
        raw1 = torch.zeros(L, O.n_params(s1), dtype=torch.float64, requires_grad=True)
        mu = mu_all[rows].clone().requires_grad_()
        kld, _, _ = O.hensman_kld(s0, O.constrain(raw0), s1, O.constrain(raw1), torch.ones(L), m, H, X[rows], mu,
                                  lv_all[rows], z, P_tot, P_b, T, False, 1e-6)
        kld.backward()
        GradAllReduce([raw0, raw1], world)()
        kt = kld.detach().reshape(1).clone()
        allreduce_tensors([kt], average=True)
        q.put(("hensman", rank, raw0.grad.numpy().copy(), raw1.grad.numpy().copy(), float(kt)))
        # --- SUM reduce of several tensors ---
        a = torch.full((3,), float(rank + 1))
        b = torch.full((2, 2), float(10 * (rank + 1)))
        allreduce_tensors([a, b], average=False)
        q.put(("sum", rank, a.numpy().copy(), b.numpy().copy()))
        # --- hensman_batches refuses per-rank subject orders that differ ---
        from lvae_amd.samplers import SubjectSampler, hensman_batches
        same = SubjectSampler(P_tot, T, seed=4).permutation()
        hensman_batches(same, P_b, T, rank, world, check=True)  # agreeing orders pass
        hensman_batches(SubjectSampler(P_tot, T, seed=100 + rank).permutation(), P_b, T, rank, world)  # no collective
        own = SubjectSampler(P_tot, T, seed=100 + rank).permutation()
        try:
            hensman_batches(own, P_b, T, rank, world, check=True)
            q.put(("perm", rank, False))
        except ValueError:
            q.put(("perm", rank, True))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_dp_contract():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(3 * world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    hens = sorted([r for r in res if r[0] == "hensman"], key=lambda r: r[1])
    sums = [r for r in res if r[0] == "sum"]
    # every rank holds the same reduced gradient
    assert np.allclose(hens[0][2], hens[1][2]) and np.allclose(hens[0][3], hens[1][3])
    # union batch on one process
    from oracle import lvae_oracle as O
    from lvae_amd.data import health_mnist_covariates
    cfg = dict(cat_kernel=[2], bin_kernel=[], sqexp_kernel=[0],
               cat_int_kernel=[{'cont_covariate': 0, 'cat_covariate': 2},
                               {'cont_covariate': 0, 'cat_covariate': 3},
                               {'cont_covariate': 1, 'cat_covariate': 4}],
               bin_int_kernel=[], covariate_missing_val=[])
    s0, s1 = O.spec_split(**cfg, id_covariate=2)
    P_tot, T, L, M = 12, 8, 2, 10
    X = torch.tensor(health_mnist_covariates(P_tot, T, seed=5))
    gen = torch.Generator().manual_seed(0)
    mu_all = torch.randn(P_tot * T, L, generator=gen, dtype=torch.float64)
    lv_all = 0.1 * torch.randn(P_tot * T, L, generator=gen, dtype=torch.float64)
    z = torch.stack([torch.cat([X[:8], X[(P_tot - 1) * T:(P_tot - 1) * T + 2]])] * L)
    m = torch.randn(L, M, 1, generator=gen, dtype=torch.float64)
    Hr = torch.randn(L, M, M, generator=gen, dtype=torch.float64) / 5
    H = Hr @ Hr.transpose(1, 2) + 0.1 * torch.eye(M, dtype=torch.float64)
    rows = torch.cat([torch.arange(s * T, (s + 1) * T) for s in [3, 7, 1, 10]])
    raw0 = torch.zeros(L, O.n_params(s0), dtype=torch.float64, requires_grad=True)
    raw1 = torch.zeros(L, O.n_params(s1), dtype=torch.float64, requires_grad=True)
    kld, _, _ = O.hensman_kld(s0, O.constrain(raw0), s1, O.constrain(raw1), torch.ones(L), m, H, X[rows],
                              mu_all[rows], lv_all[rows], z, P_tot, 4, T, False, 1e-6)
    kld.backward()
    assert np.allclose(hens[0][2], raw0.grad.numpy(), rtol=1e-10, atol=1e-10)
    assert np.allclose(hens[0][3], raw1.grad.numpy(), rtol=1e-10, atol=1e-10)
    assert abs(hens[0][4] - kld.item()) <= 1e-10 * abs(kld.item())
    for _, _, a, b in sums:
        assert np.allclose(a, 3.0) and np.allclose(b, 30.0)
    assert all(r[2] for r in res if r[0] == "perm")  # every rank detected the mismatch


def test_hensman_batch_sharding():
    from lvae_amd.samplers import SubjectSampler, hensman_batches, subject_rows
    P, T, P_b = 23, 4, 3
    perm = SubjectSampler(P, T, seed=1).permutation()
    assert sorted(perm.tolist()) == list(range(P))
    world = 2
    shards = [hensman_batches(perm, P_b, T, r, world) for r in range(world)]
    assert len(shards[0]) == len(shards[1]) == -(-P // (world * P_b))
    seen = []
    for step in range(len(shards[0])):
        for r in range(world):
            b = shards[r][step]
            if b is not None:
                seen += b.tolist()
    # the union over ranks, step by step, is exactly the single-process epoch (utils.py:51-56 order)
    assert seen == subject_rows(perm, T).tolist()
    # subject-contiguous rows
    b = shards[0][0]
    assert (b.reshape(-1, T)[:, 1:] - b.reshape(-1, T)[:, :-1] == 1).all()
    single = hensman_batches(perm, P_b, T)
    assert torch.equal(torch.cat(single), subject_rows(perm, T))


def test_varying_length_batches():
    from lvae_amd.samplers import VaryingLengthSubjectSampler, varying_length_batches
    ids = [0, 0, 0, 1, 1, 2, 2, 2, 2, 3]
    s = VaryingLengthSubjectSampler(ids, seed=0)
    batches = list(varying_length_batches(s, 2))
    flat = sorted(i for b in batches for i in b)
    assert flat == list(range(len(ids)))
    for b in batches:
        assert len({ids[i] for i in b}) <= 2


CFG = dict(cat_kernel=[2], bin_kernel=[], sqexp_kernel=[0],
           cat_int_kernel=[{'cont_covariate': 0, 'cat_covariate': 2},
                           {'cont_covariate': 0, 'cat_covariate': 3},
                           {'cont_covariate': 1, 'cat_covariate': 4}],
           bin_int_kernel=[], covariate_missing_val=[])
SH_P, SH_T, SH_L = 8, 8, 4


def _sharded_problem():
    """Fixed weights / data of the latent-sharded closed-step test (identical on every process)."""
    import lvae_amd as la
    from lvae_amd.vae import ConvVAE
    from lvae_amd.data import health_mnist_batch
    from oracle import lvae_oracle as O
    img, mask, X = health_mnist_batch(SH_P, SH_T, seed=12, dtype=torch.float64)
    ref_vae = O.ConvVAE(SH_L).double()
    ref_vae.load_state_dict(O.vae_weights(ref_vae, 5))
    vae = ConvVAE(SH_L, 1296, p_input=0.0, p=0.0).double()
    vae.load_state_dict(ref_vae.state_dict())
    k = la.generate_kernel(**CFG, latent_dim=SH_L)
    rng = np.random.default_rng(3)
    with torch.no_grad():
        for _, p in k.named_parameters():
            p.copy_(torch.tensor(np.log(rng.uniform(0.5, 3.0, SH_L))))
    eps = torch.randn(SH_P * SH_T, SH_L, generator=torch.Generator().manual_seed(2), dtype=torch.float64)
    return img, mask, X, ref_vae, vae, k, eps


def _oracle_kl(spec, params, noise, mu, logv, X):
    from oracle import lvae_oracle as O
    s = O.spec_full(**CFG)
    return torch.stack([O.kl_closed(s, params[i], X, noise[i], mu[:, i], logv[:, i]) for i in range(params.shape[0])])


def _sharded_worker(rank, world, port, q):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import lvae_amd as la
        from lvae_amd.distributed import LatentShardedClosedStep, shard_bounds
        img, mask, X, _, vae, k, eps = _sharded_problem()
        lik = la.GaussianLikelihood(SH_L, noise=1.0)
        opt = torch.optim.SGD(list(vae.parameters()) + list(k.parameters()), lr=0.0)
        step = LatentShardedClosedStep(vae, k, lik, opt, weight=0.15, loss_function="mse", kl_fn=_oracle_kl)
        lo, hi = shard_bounds(SH_P * SH_T, world, rank)
        net, rl, _, gp = step(img[lo:hi], mask[lo:hi], X, eps[lo:hi])
        q.put((rank, float(net), float(rl), float(gp),
               torch.stack([p.grad for _, p in k.named_parameters()], 1).numpy().copy(),
               [p.grad.numpy().copy() for p in vae.parameters()]))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_latent_sharded_closed_step():
    """Regime B over 2 ranks (latent dims 0-1 / 2-3, images 0-31 / 32-63, gloo on CPU, the oracle KL
    as the engine) equals one process with the whole batch (oracle.closed_step): the loss terms, the
    raw kernel-parameter gradients and every network gradient, on both ranks."""
    from oracle import lvae_oracle as O
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    img, mask, X, ref_vae, _, k, eps = _sharded_problem()
    raw = torch.stack([p.detach().clone() for _, p in k.named_parameters()], 1).requires_grad_()
    loss, recon, gp = O.closed_step(ref_vae, O.spec_full(**CFG), raw, torch.ones(SH_L, dtype=torch.float64), img,
                                    mask, X, eps, 0.15)
    for rank, net, rl, g, draw, vgrads in res:
        assert abs(net - loss.item()) <= 1e-10 * abs(loss.item())
        assert abs(rl - recon.item()) <= 1e-10 * abs(recon.item())
        assert abs(g - gp.item()) <= 1e-10 * abs(gp.item())
        assert np.allclose(draw, raw.grad.numpy(), rtol=1e-9, atol=1e-12)
        for vg, (name, p) in zip(vgrads, ref_vae.named_parameters()):
            ref = np.zeros_like(vg) if p.grad is None else p.grad.numpy()
            assert np.allclose(vg, ref, rtol=1e-8, atol=1e-12), name
    # both ranks hold the same reduced gradients
    for a, b in zip(res[0][5], res[1][5]):
        assert np.array_equal(a, b)


def test_shard_bounds():
    from lvae_amd.distributed import shard_bounds
    for n, w in [(16, 8), (16, 3), (5, 8), (4096, 8)]:
        spans = [shard_bounds(n, w, r) for r in range(w)]
        assert spans[0][0] == 0 and spans[-1][1] == n
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
        assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1
