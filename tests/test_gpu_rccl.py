"""The RCCL ("nccl" backend) branches of the multi-GPU steps, run for real in a world-size-1 process
group on one GPU: LatentShardedClosedStep's all_gather_into_tensor + all-reduces (training.py:484-592)
and the two-graph GraphedStep of the data-parallel Hensman step with its gradient / natural-gradient
all-reduces between the graphs (training.py:90-140).  A world of one makes every collective an
identity, so each result must equal the single-process step (the gloo tests in
test_distributed_cpu.py cover the world-2 arithmetic).  Also: ClosedStep replayed as one HIP graph
against its eager form (the factor's side streams and events inside the capture)."""
import socket

import numpy as np
import pytest
import torch

from oracle import lvae_oracle as O
from test_gpu_regime_b import CFG, DEV, _random_hypers, rel, set_raw

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


class _NcclWorld1:
    def __enter__(self):
        import torch.distributed as dist
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                                device_id=torch.device("cuda", 0))
        assert dist.get_backend() == "nccl"
        return dist

    def __exit__(self, *exc):
        import torch.distributed as dist
        torch.cuda.synchronize()
        dist.destroy_process_group()
        return False


def test_rccl_world1_latent_sharded_closed_step(hip):
    """LatentShardedClosedStep over RCCL (all_gather_into_tensor of (mu, logvar), SUM all-reduces of
    d/d(mu, logvar), of the flat gradient bucket and of the loss terms) against the oracle's
    whole-batch standard_training step: loss terms and every gradient."""
    import lvae_amd as la
    from lvae_amd.distributed import LatentShardedClosedStep
    from lvae_amd.vae import ConvVAE
    from lvae_amd.data import health_mnist_batch
    L, P, T = 4, 32, 16
    img, mask, X = health_mnist_batch(P, T, seed=19, dtype=torch.float64)
    ref_vae = O.ConvVAE(L).double()
    ref_vae.load_state_dict(O.vae_weights(ref_vae, 23))
    vae = ConvVAE(L, 1296, p_input=0.0, p=0.0).double()
    vae.load_state_dict(ref_vae.state_dict())
    vae = vae.float().to(DEV)
    k = la.generate_kernel(**CFG, latent_dim=L)
    set_raw(k, _random_hypers(k, L, np.random.default_rng(19)))
    raw = torch.stack([p.detach().clone() for _, p in k.named_parameters()], 1).requires_grad_()
    kd = k.to(DEV)
    lik = la.GaussianLikelihood(L, noise=1.0).to(DEV)
    eps = torch.randn(P * T, L, generator=torch.Generator().manual_seed(5), dtype=torch.float64)
    loss, recon, gp = O.closed_step(ref_vae, O.spec_full(**CFG), raw, torch.ones(L, dtype=torch.float64), img, mask,
                                    X, eps, 0.15)
    with _NcclWorld1():
        opt = torch.optim.SGD(list(vae.parameters()) + list(kd.parameters()), lr=0.0)
        step = LatentShardedClosedStep(vae, kd, lik, opt, weight=0.15, loss_function="mse")
        net, rl, _, g = step(img.float().to(DEV), mask.float().to(DEV), X.to(DEV), eps.float().to(DEV))
        torch.cuda.synchronize()
    assert rel(net, loss) < 1e-4
    assert rel(rl, recon) < 1e-4
    assert rel(g, gp) < 1e-4
    assert rel(torch.stack([p.grad for _, p in kd.named_parameters()], 1), raw.grad) < 1e-4
    for (name, p), (_, q) in zip(vae.named_parameters(), ref_vae.named_parameters()):
        if q.grad is not None:
            assert rel(p.grad, q.grad) < 1e-3, name


def _hensman_setup(L=4, M=40, T=16, P=32):
    import lvae_amd as la
    from lvae_amd.data import health_mnist_batch
    img, mask, X = health_mnist_batch(P, T, seed=16, device=DEV)
    N = P * T
    z = torch.stack([torch.cat([X[0:M // 2], X[N // 2:N // 2 + M // 2]])] * L)
    batches = [torch.cat([torch.arange(s * T, (s + 1) * T) for s in ss]).to(DEV)
               for ss in ([3, 9, 20, 1, 27], [4, 11, 30, 0, 7], [2, 5, 8, 13, 21], [6, 10, 12, 14, 15])]
    eps = torch.randn(5 * T, L, generator=torch.Generator().manual_seed(4)).to(DEV)
    return la, img, mask, X, z, batches, eps


@pytest.mark.parametrize("capture_comm", [False, True])
def test_rccl_world1_graphed_hensman_two_graphs(hip, capture_comm):
    """The data-parallel Hensman step replayed as HIP graphs with the RCCL all-reduces (GradAllReduce of the Adam
    gradients, SUM all-reduce of the natural-gradient directions: GraphedStep's comm path) -- as TWO graphs around
    the eager collectives, and (capture_comm) as ONE graph with the collectives captured -- against the eager
    single-process step, step after step."""
    from lvae_amd.distributed import GradAllReduce, allreduce_tensors
    from lvae_amd.steps import GraphedStep, HensmanStep
    from lvae_amd.vae import ConvVAE
    la, img, mask, X, z, batches, eps = _hensman_setup()
    L, M, T, P = 4, 40, 16, 32

    def make(hooks):
        torch.manual_seed(3)
        vae = ConvVAE(L, 1296, p_input=0.0, p=0.0).to(DEV)
        k0, k1 = la.generate_kernel_batched(L, **CFG, id_covariate=2)
        k0, k1 = k0.to(DEV), k1.to(DEV)
        lik = la.GaussianLikelihood(L, noise=1.0, constrain=False).to(DEV)
        with torch.no_grad():
            H = k0(z, z).evaluate() + 1e-6 * torch.eye(M, dtype=torch.float64, device=DEV)
        m = torch.zeros(L, M, 1, dtype=torch.float64, device=DEV)
        params = list(k0.parameters()) + list(k1.parameters()) + list(vae.parameters())
        opt = torch.optim.Adam(params, lr=1e-3, capturable=True)
        kw = {}
        if hooks:
            kw = dict(world=1, grad_hook=GradAllReduce(params, 1),
                      ng_reduce=lambda ts: allreduce_tensors(ts, average=False))
        return HensmanStep(vae, k0, k1, lik, opt, m, H, z, P, T, **kw), k0

    la.set_sync_checks(False)
    try:
        eager, k0_e = make(False)
        eager(img[batches[0]], mask[batches[0]], X[batches[0]], eps)  # = the graph's warm-up step
        outs_e = [[float(v) for v in eager(img[b], mask[b], X[b], eps)] for b in batches]
        with _NcclWorld1():
            graph_step, k0_g = make(True)
            s = (img[batches[0]].clone(), mask[batches[0]].clone(), X[batches[0]].clone(), eps)
            g = GraphedStep(graph_step, s, warmup=1, capture_comm=capture_comm)
            assert (g.g2 is None) == capture_comm
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
    # (m, H) after five natural-gradient steps: the fp32 ConvVAE backward (MIOpen, run-to-run
    # reduction order) moves grad_m at ~1e-7, which the updates carry into m at ~1e-6 of its size
    assert rel(graph_step.m, eager.m) < 1e-5 and rel(graph_step.H, eager.H) < 1e-6
    for (n, p), (_, q) in zip(k0_g.named_parameters(), k0_e.named_parameters()):
        assert rel(p, q) < 1e-9, n


def test_rccl_world1_two_graphs_back_to_back(hip):
    """The bench's own pattern (bench.py run_hensman): 100 back-to-back replays of the data-parallel Hensman step
    as two HIP graphs around the collectives (world-1 RCCL group), a single deferred info check at the end, then
    the last loss terms, (m, H) and the kernel hyper-parameters against the same 100 steps run eagerly and as the
    one-graph step.  Round 5 left this path corrupt: a hipMemsetAsync captured into the second graph did not zero
    the natural-gradient update's info words on replays after the first (scripts/dp_replay_diag.py); the library
    now zeroes with kernel nodes only.
    Tolerances: 100 natural-gradient + Adam steps carry the fp32 ConvVAE backward's run-to-run rounding (MIOpen
    reductions, ~1e-7 per step) into the state, and the coupled updates amplify it: observed after 100 steps (r6)
    net 2.5e-6 (one graph vs eager) and 1.0e-4 (two graphs vs one graph), m 1.7e-3.  The bounds below are set
    an order above that spread; the corruption this test guards against moved the KL term by 26% (916 vs 725,
    profiles/r6_dp_replay_diag/) and left garbage in the info words, which g.check() raises on."""
    from lvae_amd.distributed import GradAllReduce, allreduce_tensors
    from lvae_amd.steps import GraphedStep, HensmanStep
    from lvae_amd.vae import ConvVAE
    la, img, mask, X, z, batches, eps = _hensman_setup()
    L, M, T, P = 4, 40, 16, 32
    n_steps = 100

    def make(hooks):
        torch.manual_seed(3)
        vae = ConvVAE(L, 1296, p_input=0.0, p=0.0).to(DEV)
        k0, k1 = la.generate_kernel_batched(L, **CFG, id_covariate=2)
        k0, k1 = k0.to(DEV), k1.to(DEV)
        lik = la.GaussianLikelihood(L, noise=1.0, constrain=False).to(DEV)
        with torch.no_grad():
            H = k0(z, z).evaluate() + 1e-6 * torch.eye(M, dtype=torch.float64, device=DEV)
        m = torch.zeros(L, M, 1, dtype=torch.float64, device=DEV)
        params = list(k0.parameters()) + list(k1.parameters()) + list(vae.parameters())
        opt = torch.optim.Adam(params, lr=1e-3, capturable=True, fused=True)
        kw = {}
        if hooks:
            kw = dict(world=1, grad_hook=GradAllReduce(params, 1),
                      ng_reduce=lambda ts: allreduce_tensors(ts, average=False))
        return HensmanStep(vae, k0, k1, lik, opt, m, H, z, P, T, **kw), k0

    def graphed(comm, capture=False):
        step, k0 = make(comm)
        s = (img[batches[0]].clone(), mask[batches[0]].clone(), X[batches[0]].clone(), eps)
        g = GraphedStep(step, s, warmup=1, capture_comm=capture)
        assert (g.g2 is not None) == (comm and not capture)
        for i in range(n_steps):
            b = batches[i % len(batches)]
            torch.index_select(img, 0, b, out=s[0])
            torch.index_select(mask, 0, b, out=s[1])
            torch.index_select(X, 0, b, out=s[2])
            out = g()
        torch.cuda.synchronize()
        g.check()
        return [float(v) for v in out], step, k0

    la.set_sync_checks(False)
    try:
        eager, k0_e = make(False)
        eager(img[batches[0]], mask[batches[0]], X[batches[0]], eps)  # = the graph's warm-up step
        for i in range(n_steps):
            b = batches[i % len(batches)]
            out_e = [float(v) for v in eager(img[b], mask[b], X[b], eps)]
        torch.cuda.synchronize()
        out_1, one, k0_1 = graphed(False)
        with _NcclWorld1():
            out_2, two, k0_2 = graphed(True)
    finally:
        la.set_sync_checks(True)
    dm_1, dm_2 = rel(one.m, eager.m), rel(two.m, one.m)
    print("last step: eager", out_e, "one graph", out_1, "two graphs", out_2)
    print(f"m: one graph vs eager {dm_1:.3e}, two graphs vs one graph {dm_2:.3e}; "
          f"H: {rel(one.H, eager.H):.3e}, {rel(two.H, one.H):.3e}")
    assert np.allclose(out_2, out_1, rtol=1e-3) and np.allclose(out_1, out_e, rtol=1e-3), (out_e, out_1, out_2)
    assert dm_2 < 3e-2 and dm_1 < 3e-2, (dm_1, dm_2)
    assert rel(two.H, one.H) < 1e-4 and rel(one.H, eager.H) < 1e-4
    for (n, p), (_, q), (_, r) in zip(k0_2.named_parameters(), k0_1.named_parameters(), k0_e.named_parameters()):
        assert rel(p, q) < 1e-5 and rel(q, r) < 1e-5, n


def test_graphed_closed_step_matches_eager(hip):
    """ClosedStep (the bench's exact-KL step: the factorisation on the caller's stream with the inverse's
    own side stream, the ConvVAE on a second stream joined by events) captured as ONE HIP graph and
    replayed, against the same step run eagerly: per-step loss terms and the parameters after three
    Adam steps."""
    import lvae_amd as la
    from lvae_amd.data import health_mnist_batch
    from lvae_amd.steps import ClosedStep, GraphedStep
    from lvae_amd.vae import ConvVAE
    L, P, T = 4, 32, 16
    img, mask, X = health_mnist_batch(P, T, seed=12, device=DEV)
    eps = torch.randn(P * T, L, generator=torch.Generator().manual_seed(6)).to(DEV)

    def make():
        torch.manual_seed(11)
        vae = ConvVAE(L, 1296, p_input=0.0, p=0.0).to(DEV)
        k = la.generate_kernel(**CFG, latent_dim=L).to(DEV)
        lik = la.GaussianLikelihood(L, noise=1.0, constrain=False).to(DEV)
        opt = torch.optim.Adam(list(k.parameters()) + list(vae.parameters()), lr=1e-3, capturable=True)
        return ClosedStep(vae, k, lik, opt, weight=0.15), k

    la.set_sync_checks(False)
    try:
        eager, k_e = make()
        eager(img, mask, X, eps)  # = the graph's warm-up step
        outs_e = [[float(v) for v in eager(img, mask, X, eps)] for _ in range(3)]
        graph_step, k_g = make()
        g = GraphedStep(graph_step, (img, mask, X, eps), warmup=1)
        outs_g = [[float(v) for v in g()] for _ in range(3)]
        g.check()
    finally:
        la.set_sync_checks(True)
    for a, b in zip(outs_e, outs_g):
        assert np.allclose(a, b, rtol=1e-6), (a, b)
    for (n, p), (_, q) in zip(k_g.named_parameters(), k_e.named_parameters()):
        assert rel(p, q) < 1e-6, n


def test_closed_step_backward_order_agrees(hip):
    """ClosedStep's overlapped order (the factor first, the ConvVAE on its own stream, the backward from
    the two loss terms as separate roots, the KL backward split into its (mu, logvar) and hyper-parameter
    nodes) against one plain backward from the summed loss on the same models and data: every parameter
    after two Adam steps within 1e-5 (the same fp32 terms summed on different streams; Adam's normalised
    steps carry that rounding into the parameters at ~1e-6: observed 1.53e-6 on one r4 box, hence 1e-5
    rather than 1e-6; a self-consistency check, the oracle tests pin the values)."""
    import lvae_amd as la
    from lvae_amd.data import health_mnist_batch
    from lvae_amd.steps import ClosedStep
    from lvae_amd.vae import ConvVAE
    L, P, T = 4, 32, 16
    img, mask, X = health_mnist_batch(P, T, seed=13, device=DEV)
    eps = torch.randn(P * T, L, generator=torch.Generator().manual_seed(7)).to(DEV)

    def make():
        torch.manual_seed(11)
        vae = ConvVAE(L, 1296, p_input=0.0, p=0.0).to(DEV)
        k = la.generate_kernel(**CFG, latent_dim=L).to(DEV)
        lik = la.GaussianLikelihood(L, noise=1.0, constrain=False).to(DEV)
        opt = torch.optim.Adam(list(k.parameters()) + list(vae.parameters()), lr=1e-3)
        return vae, k, lik, opt

    # reference: the same step as one plain backward from the loss (no streams, no early decoder pass)
    vae_r, k_r, lik_r, opt_r = make()
    for _ in range(2):
        opt_r.zero_grad(set_to_none=True)
        mu, lv = vae_r.encode(img)
        z = vae_r.sample_latent(mu, lv, eps)
        mse, _ = vae_r.loss_function(vae_r.decode(z), img, mask)
        kl = la.KL_closed_batched(k_r, X, lik_r, mu, lv)
        (mse.sum() + 0.15 * kl.sum() / L).backward()
        opt_r.step()
        lik_r.noise = 1.0
    vae_s, k_s, lik_s, opt_s = make()
    step = ClosedStep(vae_s, k_s, lik_s, opt_s, weight=0.15)
    for _ in range(2):
        step(img, mask, X, eps)
    torch.cuda.synchronize()
    for (n, p), (_, q) in zip(list(vae_s.named_parameters()) + list(k_s.named_parameters()),
                              list(vae_r.named_parameters()) + list(k_r.named_parameters())):
        assert rel(p, q) < 1e-5, n


def _overlap_worker(rank, world, port, L, q):
    """One rank of a gloo process group over CUDA tensors on the one GPU: LatentShardedClosedStep's
    overlapped path (_step_overlapped: factor first, ConvVAE stream, split backward) against its plain
    path (_step_plain) on identical fresh models and this rank's rows."""
    import os
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import lvae_amd as la
        from lvae_amd.data import health_mnist_batch
        from lvae_amd.distributed import LatentShardedClosedStep, shard_bounds
        from lvae_amd.vae import ConvVAE
        P, T = 32, 16
        N = P * T
        img, mask, X = health_mnist_batch(P, T, seed=29, device=DEV)
        eps = torch.randn(N, L, generator=torch.Generator().manual_seed(3)).to(DEV)
        lo, hi = shard_bounds(N, world, rank)
        out = {}
        for mode in ("overlapped", "plain"):
            torch.manual_seed(17)
            vae = ConvVAE(L, 1296, p_input=0.0, p=0.0).to(DEV)
            k = la.generate_kernel(**CFG, latent_dim=L)
            set_raw(k, _random_hypers(k, L, np.random.default_rng(29)))
            k = k.to(DEV)
            lik = la.GaussianLikelihood(L, noise=1.0).to(DEV)
            opt = torch.optim.SGD(list(vae.parameters()) + list(k.parameters()), lr=0.0)
            step = LatentShardedClosedStep(vae, k, lik, opt, weight=0.15, loss_function="mse")
            fn = step._step_overlapped if mode == "overlapped" else step._step_plain
            net, rl, _, gp = fn(img[lo:hi], mask[lo:hi], X, eps[lo:hi])
            torch.cuda.synchronize()
            out[mode] = ([float(net), float(rl), float(gp)],
                         [p.grad.detach().cpu().double().numpy().copy()  # (numpy: pickled by value, not an fd)
                          for p in list(k.parameters()) + list(vae.parameters())])
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("L", [4, 1])  # L = 1: world 2 > L, rank 1 owns no latent dim
def test_gloo_world2_cuda_overlapped_matches_plain(hip, L):
    """The sharded exact-KL step's overlapped GPU path at world 2 (gloo over CUDA tensors, both ranks on the
    one GPU) equals its plain path on every rank: loss terms and every gradient within 1e-5 of their max
    (fp32 ConvVAE sums in other stream orders), including a rank that owns no latent dim."""
    import multiprocessing as mp
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    procs = [ctx.Process(target=_overlap_worker, args=(r, world, port, L, qq)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(qq.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in range(world):
        (to, go), (tp, gp) = res[rank]["overlapped"], res[rank]["plain"]
        assert np.allclose(to, tp, rtol=1e-5), (rank, to, tp)
        for a, b in zip(go, gp):
            assert rel(torch.from_numpy(a), torch.from_numpy(b)) < 1e-5, rank
    # the replicas agree across ranks (the flat SUM all-reduce)
    for a, b in zip(res[0]["overlapped"][1], res[1]["overlapped"][1]):
        assert np.array_equal(a, b)
