"""Benchmark: ELBO-steps/s of the L-VAE exact-KL training step (BASELINE.json configs[2]:
Health-MNIST-shaped N=4096 observations (P=256 subjects x T=16), L=16 latent dims, one MI355X).

One step = full-batch ConvVAE forward/backward over the N images (fp32, PyTorch-ROCm) + the
exact GP-prior KL of all L latent dims (HIP: Gram, blocked MFMA Cholesky, inverse, reductions)
forward and backward + Adam (training.py:484-592, type_KL='closed', loss='mse').

Multi-GPU (torchrun, one process per GPU): data parallel over subject mini-batches -- every rank
runs the step on its own N-observation batch of subjects, gradients all-reduced over RCCL; weak
scaling, value = total ELBO-steps/s over all ranks.

Prints ONE JSON line on rank 0 (the driver's contract); diagnostics go to stderr.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "longitudinal-vae_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

CFG = dict(cat_kernel=[2], bin_kernel=[], sqexp_kernel=[0],
           cat_int_kernel=[{'cont_covariate': 0, 'cat_covariate': 2},
                           {'cont_covariate': 0, 'cat_covariate': 3},
                           {'cont_covariate': 1, 'cat_covariate': 4}],
           bin_int_kernel=[], covariate_missing_val=[])
FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: dense f32-input MFMA peak
F16_MFMA_PEAK_TFLOPS = 2500.0   # MI355X_MICROARCH.md: dense f16/bf16 MFMA peak (~2.5 PF, no sparsity)
X3_PRODUCTS = 3                 # f16 MFMA products per fp32-equivalent product (mfma_x3.hpp)
# Memory-side bytes per syrk launch from the committed rocprofv3 PMC passes (scripts/pmc.sh ->
# profiles/r1_v6_pmc_summary.json: FETCH_SIZE / WRITE_SIZE in KiB per dispatch; FETCH_SIZE x 2 for
# 16-B/lane coalesced reads on gfx950, MI355X_MICROARCH.md "HBM").  Counts L2 misses incl.
# Infinity-Cache hits, so it bounds HBM traffic from above.
PMC_SUMMARY = os.path.join(ROOT, "profiles", "r1_v7_pmc_summary.json")


def pmc_traffic(kernels):
    """Sum over the named kernels (one dispatch each per step) of FETCH_SIZE x 2 + WRITE_SIZE, bytes."""
    try:
        d = json.load(open(PMC_SUMMARY))
        tot = 0.0
        for name in kernels:
            f = [v["mean"] for k, v in d["FETCH_SIZE"].items() if name in k]
            w = [v["mean"] for k, v in d["WRITE_SIZE"].items() if name in k]
            if not (f and w):
                return None
            tot += (2 * f[0] + w[0]) * 1024
        return tot
    except (OSError, KeyError, ValueError):
        return None
HBM_PEAK_GBS = 8000.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def setup_dist(ngpu):
    """One process per GPU (torchrun env).  Returns (world, rank, device index).  RCCL ("nccl") by
    default; LVAE_DIST_BACKEND=gloo rehearses the multi-rank path with several ranks on fewer GPUs
    (device = LOCAL_RANK mod the visible GPU count)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = max(torch.cuda.device_count(), 1)
    dev = local % ndev
    if world > 1:
        torch.cuda.set_device(dev)
        backend = os.environ.get("LVAE_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    return world, rank, dev


def cpu_baseline(P, T, L, dims_timed=1):
    """Time the CPU oracle (fp64 torch, the reference's op sequence) on a bounded sample of the same
    step: ConvVAE fwd/bwd on all N images + KL_closed fwd/bwd of `dims_timed` latent dims, then
    extrapolate the KL part to L dims."""
    from oracle import lvae_oracle as O
    from lvae_amd.data import health_mnist_batch
    img, mask, X = health_mnist_batch(P, T, seed=0, dtype=torch.float64)
    torch.manual_seed(0)
    vae = O.ConvVAE(L).double()
    spec = O.spec_full(**CFG)
    raw = torch.zeros(L, O.n_params(spec), dtype=torch.float64)
    raw[:, :] = torch.log(torch.tensor(math.log(2.0)))
    N = P * T
    eps = torch.randn(N, L, dtype=torch.float64)
    t0 = time.perf_counter()
    mu, logv = vae.encode(img)
    recon = vae.decode(mu + eps * torch.exp(0.5 * logv))
    mse, _ = vae.loss_function(recon, img, mask)
    mse.sum().backward(retain_graph=True)
    t_vae = time.perf_counter() - t0
    t0 = time.perf_counter()
    for l in range(dims_timed):
        r = raw[l].clone().requires_grad_()
        m_ = mu[:, l].detach().clone().requires_grad_()
        v_ = logv[:, l].detach().clone().requires_grad_()
        O.kl_closed(spec, O.constrain(r), X, 1.0, m_, v_).backward()
    t_dim = (time.perf_counter() - t0) / dims_timed
    t_step = t_vae + L * t_dim
    return dict(value=1.0 / t_step, unit="ELBO-steps/s", cores=torch.get_num_threads(), kind="port",
                sample=(f"oracle fp64 torch-CPU: ConvVAE fwd/bwd on all {N} images ({t_vae:.2f} s) + KL_closed "
                        f"fwd/bwd of {dims_timed} of {L} latent dims ({t_dim:.2f} s/dim), step = vae + L x dim "
                        f"= {t_step:.1f} s"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--P", type=int, default=256, help="subjects per rank (N = P*T)")
    ap.add_argument("--T", type=int, default=16)
    ap.add_argument("--L", type=int, default=16)
    ap.add_argument("--regime", choices=["closed", "hensman"], default="closed",
                    help="closed: exact-KL step (headline, configs[2]); hensman: SVI mini-batch step (configs[3])")
    ap.add_argument("--P_b", type=int, default=5, help="hensman: subjects per batch per rank")
    ap.add_argument("--M", type=int, default=120, help="hensman: inducing points")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-phase-timing", action="store_true")
    args = ap.parse_args()

    world, rank, local = setup_dist(args.gpus)
    if args.regime == "hensman":
        return main_hensman(args, world, rank, local)
    dev = torch.device("cuda", local)
    import lvae_amd as la
    from lvae_amd import _lib
    from lvae_amd.data import health_mnist_batch
    from lvae_amd.steps import ClosedStep
    from lvae_amd.vae import ConvVAE

    la.set_sync_checks(False)
    P, T, L = args.P, args.T, args.L
    N = P * T
    torch.manual_seed(1234)  # identical initial weights on every rank
    vae = ConvVAE(L, 1296, p_input=0.0, p=0.0).to(dev)
    kernel = la.generate_kernel(**CFG, latent_dim=L).to(dev)
    lik = la.GaussianLikelihood(L, noise=1.0, constrain=False).to(dev)
    opt = torch.optim.Adam([{"params": kernel.parameters()}, {"params": vae.parameters()}], lr=1e-3)
    img, mask, X = health_mnist_batch(P, T, seed=100 + rank, device=dev)
    gen = torch.Generator(device=dev).manual_seed(7 + rank)
    eps = torch.randn(N, L, device=dev, generator=gen)

    hook = None
    if world > 1:
        from lvae_amd.distributed import GradAllReduce
        hook = GradAllReduce(list(vae.parameters()) + list(kernel.parameters()), world)
    step = ClosedStep(vae, kernel, lik, opt, weight=0.15, loss_function="mse", constrain_scales=True,
                      grad_hook=hook)

    for _ in range(args.warmup):
        out = step(img, mask, X, eps)
    torch.cuda.synchronize()
    la.check_pending()

    phase = {}
    if not args.no_phase_timing:
        _lib.prof_enable(True)
        _lib.prof_collect()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step(img, mask, X, eps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if not args.no_phase_timing:
        phase = _lib.prof_collect()
        _lib.prof_enable(False)
    la.check_pending()
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    net, recon, nll, gp = [float(v) for v in out]
    log(f"rank {rank}: last step net={net:.4f} recon={recon:.4f} gp={gp:.4f}; phases(ms total over {args.steps} "
        f"steps)={ {k: round(v[0], 3) for k, v in phase.items() if v[1]} }")

    if rank == 0:
        ms_per_step = 1000.0 * elapsed / args.steps
        value = world * args.steps / elapsed
        np_ = _lib.load().lvae_kl_closed_padded_n(N)
        res = {"metric": "ELBO-steps/sec (exact-KL L-VAE step, Health-MNIST N=4096 L=16)", "value": value,
               "unit": "ELBO-steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
               "dtype": "fp32", "data": "synthetic (Health-MNIST-shaped covariates/images, random-init ConvVAE)",
               "config": {"workload": f"closed-form KL step, N={N} (P={P} subjects x T={T}) per rank, L={L}, "
                                      f"R=5 additive components (config/LVAE_config_sample.txt)",
                          "N": N, "L": L, "parallelism": f"dp{world} over subject batches"}}
        if phase:
            potrf_ms = phase["potrf"][0] / args.steps
            syrk_ms = phase["syrk"][0] / args.steps
            res["gp_cholesky_gflops"] = L * N ** 3 / 3 / (potrf_ms * 1e-3) / 1e9 if potrf_ms > 0 else None
            res["phase_ms_per_step"] = {k: v[0] / args.steps for k, v in phase.items() if v[1]}
            # dominant kernel: the sweep's rank-256 update U2 (sw_update_kernel<false, false>, nt - 1
            # launches per step, 31% of the step's GPU time).  Algorithmic bytes per launch: every
            # updated lower 256-tile is read and written once in fp32 -> 2 x 4 B x 256^2 per tile,
            # (nt-1) nt / 2 - 1 tiles per dim (the grid without row / column k and tile (k+1, k+1)),
            # x L.  The W / C operand planes are L2-resident re-reads, not algorithmic traffic.
            nt = np_ // 256
            upd_ms, upd_n = phase.get("sweep_update", (0.0, 0))
            tiles = ((nt - 1) * nt // 2 - 1) * L
            upd_bytes = 2 * 4 * 256 * 256 * tiles
            if upd_n and np_ % 256 == 0:
                avg_s = upd_ms / upd_n * 1e-3
                ach = upd_bytes / avg_s / 1e9
                res["roofline"] = {"kernel": "sw_update_kernel<false, false> (sweep rank-256 update U2, spd_sweep.hip)",
                                   "bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                   "frac": ach / HBM_PEAK_GBS,
                                   "traffic": pmc_traffic(("sw_update_kernel<false, false",)),
                                   "algorithmic_bytes_per_launch": upd_bytes, "avg_launch_us": avg_s * 1e6,
                                   "launches_per_step": upd_n / args.steps, "padded_n": int(np_)}
            # secondary: S = K^-1 V K^-1, the largest single launch (one per step).  Algorithmic flops
            # = L * N^2 (N+1) (lower triangle incl. diagonal, 2 flop/FMA).  Engine: 3-product f16
            # split -> the f16 dense peak / 3 (each fp32 FMA costs three f16 MFMA FMAs).
            flops = L * np_ * np_ * (np_ + 1)
            achieved = flops / (syrk_ms * 1e-3) / 1e12 if syrk_ms > 0 else None
            fast_syrk = np_ % 256 == 0 and not int(os.environ.get("LVAE_SYRK_GENERIC", "0"))
            x3 = fast_syrk or bool((_lib.load().lvae_gemm_engine_mask() >> 5) & 1)
            peak = F16_MFMA_PEAK_TFLOPS / X3_PRODUCTS if x3 else FP32_MFMA_PEAK_TFLOPS
            syrk_line = {"kernel": "syrk_split_kernel + syrk_x3_kernel (S = K^-1 V K^-1)" if fast_syrk
                         else "syrk_scaled_kernel (S = K^-1 V K^-1)", "bound": "mfma",
                         "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                         "frac": (achieved / peak) if achieved else None,
                         "traffic": pmc_traffic(("syrk_x3_kernel", "syrk_split_kernel") if fast_syrk else
                                                ("syrk_scaled_kernel<true>" if x3 else "syrk_scaled_kernel<false>",)),
                         "padded_n": int(np_),
                         "engine": ("f16 MFMA, 3-product split (fp32-equivalent peak = 2.5 PF / 3)" if x3
                                    else "fp32-input MFMA")}
            if "roofline" in res:
                res["roofline_secondary"] = syrk_line
            else:
                res["roofline"] = syrk_line
        if not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(P, T, L)
            res["vs_cpu_baseline"] = value / world / res["cpu_baseline"]["value"]
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline_hensman(P, T, L, M, P_b, steps=12):
    """The oracle's Hensman step (training.py:91-135 restated, fp64 torch-CPU) on the same shapes."""
    from oracle import lvae_oracle as O
    from lvae_amd.data import health_mnist_batch
    img, mask, X = health_mnist_batch(P, T, seed=0, dtype=torch.float64)
    torch.manual_seed(0)
    vae = O.ConvVAE(L).double()
    s0, s1 = O.spec_split(**CFG, id_covariate=2)
    raw0 = torch.full((L, O.n_params(s0)), math.log(2.0), dtype=torch.float64, requires_grad=True)
    raw1 = torch.full((L, O.n_params(s1)), math.log(2.0), dtype=torch.float64, requires_grad=True)
    N = P * T
    z = torch.stack([torch.cat([X[0:M // 2], X[N // 2:N // 2 + M // 2]])] * L)
    m = torch.zeros(L, M, 1, dtype=torch.float64)
    H = O.gram(s0, O.constrain(raw0.detach()), z, z) + 1e-6 * torch.eye(M, dtype=torch.float64)
    opt = torch.optim.Adam([raw0, raw1] + list(vae.parameters()), lr=1e-3)
    noise = torch.ones(L, dtype=torch.float64)
    B = P_b * T
    times = []
    for it in range(steps):
        rows = torch.arange(B) + (it * B) % (N - B)
        t0 = time.perf_counter()
        eps = torch.randn(B, L, dtype=torch.float64)
        _, _, _, m, H = O.hensman_step(vae, s0, raw0, s1, raw1, noise, m, H, img[rows], mask[rows], X[rows], z, eps,
                                       P, T, 0.15, 0.01, opt=opt)
        times.append(time.perf_counter() - t0)
    t = sorted(times[2:])[len(times[2:]) // 2]
    return dict(value=1.0 / t, unit="ELBO-steps/s", cores=torch.get_num_threads(), kind="port",
                sample=f"oracle fp64 torch-CPU Hensman step (L={L}, M={M}, P_b={P_b}, T={T}), median of "
                       f"{steps - 2} steps after 2 warm-up: {1000 * t:.1f} ms/step")


def main_hensman(args, world, rank, local):
    """Hensman SVI training steps (training.py:91-135), data parallel over subject mini-batches."""
    dev = torch.device("cuda", local)
    import lvae_amd as la
    from lvae_amd import _lib
    from lvae_amd.data import health_mnist_batch
    from lvae_amd.samplers import hensman_batches, SubjectSampler
    from lvae_amd.steps import HensmanStep
    from lvae_amd.vae import ConvVAE

    la.set_sync_checks(False)
    P, T, L, M, P_b = args.P, args.T, args.L, args.M, args.P_b
    N = P * T
    torch.manual_seed(1234)
    vae = ConvVAE(L, 1296, p_input=0.0, p=0.0).to(dev)
    k0, k1 = la.generate_kernel_batched(L, **CFG, id_covariate=2)
    k0, k1 = k0.to(dev), k1.to(dev)
    lik = la.GaussianLikelihood(L, noise=1.0, constrain=False).to(dev)
    img, mask, X = health_mnist_batch(P, T, seed=100, device=dev)  # one data set, sharded by subject
    z = torch.stack([torch.cat([X[0:M // 2], X[N // 2:N // 2 + M // 2]])] * L)  # LVAE.py:199-203 pattern
    with torch.no_grad():
        H = k0(z, z).evaluate() + 1e-6 * torch.eye(M, dtype=torch.float64, device=dev)
    m = torch.zeros(L, M, 1, dtype=torch.float64, device=dev)
    opt = torch.optim.Adam([{"params": k0.parameters()}, {"params": k1.parameters()},
                            {"params": vae.parameters()}], lr=1e-3)
    hook = ngr = None
    if world > 1:
        from lvae_amd.distributed import GradAllReduce, allreduce_tensors
        hook = GradAllReduce(list(vae.parameters()) + list(k0.parameters()) + list(k1.parameters()), world)
        ngr = lambda ts: allreduce_tensors(ts, average=False)
    step = HensmanStep(vae, k0, k1, lik, opt, m, H, z, P, T, weight=0.15, natural_gradient=True,
                       natural_gradient_lr=0.01, world=world, grad_hook=hook, ng_reduce=ngr)
    perm = SubjectSampler(P, T, seed=0).permutation()
    batches = [b.to(dev) for b in hensman_batches(perm, P_b, T, rank, world) if b is not None and len(b) == P_b * T]
    gen = torch.Generator(device=dev).manual_seed(7 + rank)
    eps = torch.randn(P_b * T, L, device=dev, generator=gen)

    def run(n):
        out = None
        for i in range(n):
            rows = batches[i % len(batches)]
            out = step(img.index_select(0, rows), mask.index_select(0, rows), X.index_select(0, rows), eps)
        return out

    run(args.warmup)
    torch.cuda.synchronize()
    la.check_pending()
    if not args.no_phase_timing:
        _lib.prof_enable(True)
        _lib.prof_collect()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = run(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    phase = {}
    if not args.no_phase_timing:
        phase = _lib.prof_collect()
        _lib.prof_enable(False)
    la.check_pending()
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    log(f"rank {rank}: last step (net, recon, nll, kld) = {[round(float(v), 4) for v in out]}")
    if rank == 0:
        value = world * args.steps / elapsed
        res = {"metric": "ELBO-steps/sec (Hensman SVI L-VAE step, Health-MNIST N=4096 L=16)", "value": value,
               "unit": "ELBO-steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": 1000.0 * elapsed / args.steps, "higher_is_better": True, "scaling": "weak",
               "vs_baseline": None, "dtype": "fp64 GP / fp32 conv",
               "data": "synthetic (Health-MNIST-shaped covariates/images, random-init ConvVAE)",
               "config": {"workload": f"Hensman step: P_tot={P} subjects x T={T} (N={N}), L={L}, M={M}, "
                                      f"P_b={P_b} subjects per rank per step",
                          "samples_per_sec": value * P_b * T, "parallelism": f"dp{world} over subject batches"}}
        if phase:
            res["phase_ms_per_step"] = {k: v[0] / args.steps for k, v in phase.items() if v[1]}
        if not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline_hensman(P, T, L, M, P_b)
            res["vs_cpu_baseline"] = value / world / res["cpu_baseline"]["value"]
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
