"""Benchmark: ELBO-steps/s of the L-VAE training step (BASELINE.json: Health-MNIST N=4096, L=16).

Headline (`value`): the exact-KL step of standard_training (type_KL='closed', loss='mse';
training.py:484-592) at BASELINE configs[2] = N = 4096 observations (P = 256 subjects x T = 16),
L = 16 latent dims: full-batch ConvVAE forward / backward (fp32, PyTorch-ROCm) + the exact GP-prior
KL of all L dims forward and backward (HIP: Gram, blocked Cholesky potrf + trtri + lauum, fp64
refinement of K^-1 mu, S GEMM, Gram adjoint) + Adam.
  N = 1: one process.  N > 1: the SAME step (same objective, same N and L) with the latent dims
  sharded over the ranks and the images split over them (lvae_amd.distributed.
  LatentShardedClosedStep): strong scaling, value = whole-job ELBO-steps/s.

Sub-record `regime_a` (BASELINE configs[3], the path config/LVAE_config_sample.txt selects), at every N:
the Hensman SVI step (training.py:90-140) at L = 16, M = 120, P_b = 5 subjects x T = 16 per rank, data
parallel over subject mini-batches for N > 1 (weak scaling: value = whole-job ELBO-steps/s, samples_per_sec
= all ranks' images/s), replayed as HIP graphs -- one per step at N = 1, two around the RCCL all-reduces of
the Adam gradients and the natural-gradient statistics at N > 1.  At N = 1 its `dp_world1_rccl` sub-record
times that two-graph form through a world-1 RCCL group.

Sub-record `c2` (BASELINE configs[1], N = 1 only): HIP Gram + blocked Cholesky inverse + log-det (the
product route, lvae_spd_inv_chol_f32) vs PyTorch-ROCm Gram + torch.linalg.cholesky (+ cholesky_inverse)
at N = 1024, L = 8; GP-Cholesky GFLOP/s from the potrf phase alone on both sides.

Prints ONE JSON line on rank 0 (the driver's contract); diagnostics go to stderr.
"""
import argparse
import json
import math
import os
import platform
import subprocess
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
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E peak (spec)
F16_MFMA_PEAK_TFLOPS = 2500.0   # MI355X_MICROARCH.md: dense f16/bf16 MFMA peak (~2.5 PF, no sparsity)
X3_PRODUCTS = 3                 # f16 MFMA products per fp32-equivalent product (mfma_x3.hpp)
DTYPE = "f16x3-split (fp32-equivalent)"
# Memory-side bytes per launch from the committed rocprofv3 PMC passes (scripts/pmc.sh):
# FETCH_SIZE x 2 (16-B/lane coalesced reads on gfx950, MI355X_MICROARCH.md "HBM") + WRITE_SIZE.
# (LVAE_PROFILE_TAG: the round whose committed profile files price the line; scripts/gpu_evidence.sh writes them)
TAG = os.environ.get("LVAE_PROFILE_TAG", "r6")
PMC_SUMMARY = os.path.join(ROOT, "profiles", f"{TAG}_pmc_summary.json")
# The committed rocprofv3 --kernel-trace --stats summary of the default closed bench on the final tree
# (scripts/gpu_evidence.sh): the roofline's `frac` is priced on its average launch duration of the dominant
# kernel, so that it recomputes from profiles/; the live HIP-event figure is reported beside it.
KSTATS = os.path.join(ROOT, "profiles", f"{TAG}_headline_kernel_stats.csv")
# the Cholesky's trailing rank-256 update (chol_inv.hip): U2 alone (MODE kCiU2) when the lookahead chain
# runs on the side stream (schedule (b), > CI_FUSE_MAX_L dims per call), else fused with U1 (kCiU12)
CI_FUSE_MAX_L = 16
U2_NAMES = {False: "ci_update_kernel<0>", True: "ci_update_kernel<2>"}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def pmc_traffic(kernels, per_step=False):
    """FETCH_SIZE x 2 + WRITE_SIZE (bytes) of the named kernels from the committed PMC summary: per
    dispatch (mean), or per step (the summary's per-step total, for kernels launched several times
    a step with different sizes)."""
    try:
        d = json.load(open(PMC_SUMMARY))
        key = "per_step" if per_step else "mean"
        tot = 0.0
        for name in kernels:
            f = [v[key] for k, v in d["FETCH_SIZE"].items() if name in k.replace(" ", "")]
            w = [v[key] for k, v in d["WRITE_SIZE"].items() if name in k.replace(" ", "")]
            if not (f and w):
                return None
            tot += (2 * f[0] + w[0]) * 1024
        return tot
    except (OSError, KeyError, ValueError):
        return None


# MFMA utilisation per kernel from the committed rocprofv3 --pmc pass over this bench's closed step
# (scripts/gpu_mfma_pmc.sh, scripts/mfma_pmc.py): SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
MFMA_PMC = os.path.join(ROOT, "profiles", f"{TAG}_mfma_pmc.json")
MFMA_KERNELS = {"lauum + KL epilogue": "ci_gemm_kernel<3>", "trtri X step": "ci_gemm_kernel<0>",
                "trtri Y step": "ci_gemm_kernel<1>", "potrf trailing update": "ci_update_kernel<2>",
                "potrf panel": "ci_panel_kernel", "potrf pivot (split)": "ci_pivot_kernel<4>",
                "binned hyper slab pass": "hb_slab_kernel",
                "conv2 weight gradient (f32 MFMA)": "conv3x3_pool_wgrad_mfma_kernel",
                "conv2 input gradient (f32 MFMA)": "conv3x3_pool_dgrad_mfma_kernel",
                "deconv1 backward (f32 MFMA)": "deconv4s2_relu_bwd_mfma_kernel"}


def mfma_busy(name_part, path=MFMA_PMC):
    """(mfma_busy_frac, dispatches) of the kernel whose name contains name_part in the committed MFMA PMC summary."""
    try:
        for k, v in json.load(open(path)).items():
            if name_part in k.replace(" ", "") and "mfma_busy_frac" in v:
                return v["mfma_busy_frac"], v["dispatches"]
    except (OSError, ValueError):
        pass
    return None


def kstats_avg_us(name_part, path=KSTATS):
    """(average launch duration in us, calls) of the kernel whose name contains name_part in the
    committed rocprofv3 stats CSV, or None."""
    import csv
    try:
        for r in csv.DictReader(open(path)):
            if name_part in r["Name"]:
                return float(r["AverageNs"]) / 1e3, int(r["Calls"])
    except (OSError, KeyError, ValueError):
        pass
    return None


def setup_dist(force_group=False):
    """One process per GPU (torchrun env).  Returns (world, rank, device index).  RCCL ("nccl") by
    default; LVAE_DIST_BACKEND=gloo rehearses the multi-rank path with several ranks on fewer GPUs.
    force_group: a process group even at world 1 (--sharded-world1: the sharded step through RCCL)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = max(torch.cuda.device_count(), 1)
    dev = local % ndev
    if force_group and not dist.is_initialized() and "MASTER_ADDR" not in os.environ:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        import socket
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            os.environ["MASTER_PORT"] = str(so.getsockname()[1])
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if world > 1 or force_group:
        torch.cuda.set_device(dev)
        backend = os.environ.get("LVAE_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    return world, rank, dev


def cpu_share():
    """The host CPUs this process may use: the affinity mask, the cgroup v2 quota (cpu.max) and the
    OMP_NUM_THREADS the box sets (the harness assigns each GPU a 16-CPU share; os.cpu_count() is the
    whole machine's)."""
    share = {"sched_getaffinity": len(os.sched_getaffinity(0)), "os_cpu_count": os.cpu_count(),
             "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS")}
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        share["cgroup_cpu_max"] = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        share["cgroup_cpu_max"] = "unreadable"
    return share


def host_info():
    """lscpu model / sockets / physical cores, the NUMA node of GPU0 if sysfs shows it, and the CPU
    share (cpu_share) the timed threads come from."""
    info = {"threads_used": torch.get_num_threads(), "os_cpu_count": os.cpu_count(), "machine": platform.machine(),
            "cpu_share": cpu_share()}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        kv = {k.strip(): v.strip() for k, v in (ln.split(":", 1) for ln in out.splitlines() if ":" in ln)}
        info["model"] = kv.get("Model name")
        info["sockets"] = kv.get("Socket(s)")
        info["cores_per_socket"] = kv.get("Core(s) per socket")
        info["threads_per_core"] = kv.get("Thread(s) per core")
    except (OSError, subprocess.SubprocessError, ValueError):
        pass
    try:
        import glob
        for p in sorted(glob.glob("/sys/class/drm/card*/device/numa_node")):
            info["gpu0_numa_node"] = int(open(p).read().strip())
            break
    except (OSError, ValueError):
        pass
    return info


class ClockSampler:
    """The GFX clock of this process's GPU (amdsmi, matched by PCI bus) sampled by a thread every
    `period` s while the timed steps run: the evidence for kernel averages that differ between runs (a
    rocprofv3-traced run against an untraced one).  Reports nothing if amdsmi or the match is missing;
    LVAE_BENCH_CLOCKS=0 switches it off."""

    def __init__(self, dev, period=0.02):
        import threading
        self.samples, self.h, self.period = [], None, period
        self._stop = threading.Event()
        self._thread = None
        if os.environ.get("LVAE_BENCH_CLOCKS", "1") == "0":
            return
        try:
            import amdsmi
            amdsmi.amdsmi_init()
            props = torch.cuda.get_device_properties(dev)
            bus = getattr(props, "pci_bus_id", None)
            for h in amdsmi.amdsmi_get_processor_handles():
                if bus is not None and int(amdsmi.amdsmi_get_gpu_device_bdf(h).split(":")[1], 16) == bus:
                    self.h, self._smi = h, amdsmi
        except Exception as e:  # noqa: BLE001 -- diagnostics only
            log(f"clock sampler off: {e}")

    def _run(self):
        smi = self._smi
        while not self._stop.is_set():
            try:
                self.samples.append(smi.amdsmi_get_clock_info(self.h, smi.AmdSmiClkType.GFX)["clk"])
            except Exception:  # noqa: BLE001
                return
            self._stop.wait(self.period)

    def __enter__(self):
        if self.h is not None:
            import threading
            self._thread = threading.Thread(target=self._run, daemon=True)
            self._thread.start()
        return self

    def __exit__(self, *exc):
        if self._thread is not None:
            self._stop.set()
            self._thread.join()

    def record(self):
        v = sorted(x for x in self.samples if isinstance(x, (int, float)))
        if not v:
            return None
        return {"gfx_mhz_median": v[len(v) // 2], "gfx_mhz_min": v[0], "gfx_mhz_max": v[-1], "samples": len(v),
                "source": f"amdsmi GFX clock of this GPU every {1000 * self.period:.0f} ms over the timed steps"}


def sync_barrier(world):
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(x, world, dev):
    if world == 1:
        return x
    t = torch.tensor([x], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


# ------------------------------------------------------------------------------------------
# CPU baselines (the oracle, fp64 torch-CPU, the reference's op sequence) -- rank 0, N = 1 only
# ------------------------------------------------------------------------------------------
def cpu_baseline_closed(P, T, L, threads8_dims=1, warmups=3):
    """The C3 step on the CPU port (fp64), by BASELINE.md's / SURVEY.md 8(d)'s method within one lease:
    `warmups` warm-up steps (ConvVAE fwd/bwd on all N images + one latent dim's KL_closed fwd/bwd each),
    then ONE whole timed step: the ConvVAE fwd/bwd and all L latent dims' KL_closed fwd/bwd (~60 s at C3);
    plus an 8-thread figure (ConvVAE + one dim, x L dims) for comparison with the survey container's
    numbers."""
    from oracle import lvae_oracle as O
    from lvae_amd.data import health_mnist_batch
    img, mask, X = health_mnist_batch(P, T, seed=0, dtype=torch.float64)
    torch.manual_seed(0)
    vae = O.ConvVAE(L).double()
    spec = O.spec_full(**CFG)
    raw = torch.full((L, O.n_params(spec)), math.log(math.log(2.0)), dtype=torch.float64)
    N = P * T
    eps = torch.randn(N, L, dtype=torch.float64)

    def step(dims, l0=0):
        t0 = time.perf_counter()
        mu, logv = vae.encode(img)
        recon = vae.decode(mu + eps * torch.exp(0.5 * logv))
        mse, _ = vae.loss_function(recon, img, mask)
        mse.sum().backward(retain_graph=True)
        t_vae = time.perf_counter() - t0
        t0 = time.perf_counter()
        for l in range(l0, l0 + dims):
            r = raw[l % L].clone().requires_grad_()
            m_ = mu[:, l % L].detach().clone().requires_grad_()
            v_ = logv[:, l % L].detach().clone().requires_grad_()
            O.kl_closed(spec, O.constrain(r), X, 1.0, m_, v_).backward()
        return t_vae, time.perf_counter() - t0

    nthreads = torch.get_num_threads()
    for k in range(warmups):  # warm-ups (allocator, thread pool, first touch)
        step(1, l0=k)
    t_vae, t_kl = step(L)
    t_step = t_vae + t_kl
    res = dict(value=1.0 / t_step, unit="ELBO-steps/s", cores=nthreads, kind="port",
               sample=(f"oracle fp64 torch-CPU, {nthreads} threads, one whole step after {warmups} warm-ups: "
                       f"ConvVAE fwd/bwd on all {N} images ({t_vae:.2f} s) + KL_closed fwd/bwd of all {L} latent "
                       f"dims ({t_kl:.2f} s) = {t_step:.1f} s per step"))
    try:
        torch.set_num_threads(8)
        v8, k8 = step(threads8_dims)
        res["threads8"] = {"value": 1.0 / (v8 + L * k8 / threads8_dims), "unit": "ELBO-steps/s",
                           "sample": f"8 threads: ConvVAE {v8:.2f} s + {threads8_dims} dim(s) {k8:.2f} s, x{L} dims"}
    finally:
        torch.set_num_threads(nthreads)
    res["host"] = host_info()
    return res


def cpu_baseline_hensman(P, T, L, M, P_b, steps=12):
    """The oracle's Hensman step (training.py:91-135 restated, fp64 torch-CPU) on the same shapes."""
    from oracle import lvae_oracle as O
    from lvae_amd.data import health_mnist_batch
    img, mask, X = health_mnist_batch(P, T, seed=0, dtype=torch.float64)
    torch.manual_seed(0)
    vae = O.ConvVAE(L).double()
    s0, s1 = O.spec_split(**CFG, id_covariate=2)
    raw0 = torch.full((L, O.n_params(s0)), math.log(math.log(2.0)), dtype=torch.float64, requires_grad=True)
    raw1 = torch.full((L, O.n_params(s1)), math.log(math.log(2.0)), dtype=torch.float64, requires_grad=True)
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


# ------------------------------------------------------------------------------------------
# Regime B: the headline exact-KL step
# ------------------------------------------------------------------------------------------
def run_closed(args, world, rank, dev):
    import lvae_amd as la
    from lvae_amd import _lib
    from lvae_amd.data import health_mnist_batch
    from lvae_amd.steps import ClosedStep
    from lvae_amd.distributed import LatentShardedClosedStep, shard_bounds
    from lvae_amd.vae import ConvVAE

    la.set_sync_checks(False)
    P, T, L = args.P, args.T, args.L
    N = P * T
    torch.manual_seed(1234)  # identical initial weights on every rank
    vae = ConvVAE(L, 1296, p_input=0.0, p=0.0).to(dev)
    kernel = la.generate_kernel(**CFG, latent_dim=L).to(dev)
    lik = la.GaussianLikelihood(L, noise=1.0, constrain=False).to(dev)
    # --graph (one GPU): the whole step (forward, backward, Adam) captured once and replayed as ONE HIP
    # graph (steps.GraphedStep).  Measured slower than eager (15.4-15.7 vs 12.8 ms at L = 16, 8.9-9.0 vs
    # 5.2 ms at L = 2, scripts/graph_ab.sh): the replay does not keep the side stream's pivot chain and the
    # ConvVAE stream running beside the caller's stream, so the default stays eager.
    use_graph = world == 1 and args.graph
    opt = torch.optim.Adam([{"params": kernel.parameters()}, {"params": vae.parameters()}], lr=1e-3, fused=True,
                           capturable=use_graph)
    img, mask, X = health_mnist_batch(P, T, seed=100, device=dev)   # the same data set on every rank
    gen = torch.Generator(device=dev).manual_seed(7)
    eps = torch.randn(N, L, device=dev, generator=gen)
    share = args.rank_share if world == 1 else 0
    if world > 1 or share > 1 or args.sharded_world1:
        W, r = (world, rank) if world > 1 else (max(share, 1), 0)
        lo, hi = shard_bounds(N, W, r)
        step = LatentShardedClosedStep(vae, kernel, lik, opt, weight=0.15, loss_function="mse", constrain_scales=True,
                                       sim_world=share if share > 1 else None,
                                       vae_stream_priority=args.vae_stream_priority)
        inputs = (img[lo:hi].contiguous(), mask[lo:hi].contiguous(), X, eps[lo:hi].contiguous())
        d0, d1 = shard_bounds(L, W, r)
    else:
        step = ClosedStep(vae, kernel, lik, opt, weight=0.15, loss_function="mse", constrain_scales=True,
                          vae_stream_priority=args.vae_stream_priority)
        inputs = (img, mask, X, eps)
        d0, d1 = 0, L

    if use_graph:
        from lvae_amd.steps import GraphedStep
        graph = GraphedStep(step, inputs, warmup=max(args.warmup, 1))  # warm-up steps, then the capture
        run = graph
    else:
        def run():
            return step(*inputs)
        for _ in range(args.warmup):
            run()
    torch.cuda.synchronize()
    la.check_pending()
    if not args.no_phase_timing and not use_graph:
        _lib.prof_enable(True)
        _lib.prof_collect()
    clocks = ClockSampler(dev) if rank == 0 else None
    sync_barrier(world)
    if clocks:
        clocks.__enter__()
    # LVAE_BENCH_CPROFILE=path: the host side (Python) of the timed steps under cProfile (scripts/gpu_host_prof.sh)
    cprof_path = os.environ.get("LVAE_BENCH_CPROFILE")
    if cprof_path and rank == 0:
        import cProfile
        cprof = cProfile.Profile()
        cprof.enable()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = run()
    t_enq = time.perf_counter() - t0  # (host enqueue of all steps; the GPU drains the rest below)
    sync_barrier(world)
    elapsed = time.perf_counter() - t0
    if cprof_path and rank == 0:
        cprof.disable()
        cprof.dump_stats(cprof_path)
    if clocks:
        clocks.__exit__(None, None, None)
    if use_graph:
        graph.check()
    phase = {}
    if not args.no_phase_timing:
        if use_graph:
            # the phase (and roofline kernel) times come from the same number of eager steps right after
            # the graph-timed region: the library's HIP events bracket its own launches on their streams
            _lib.prof_enable(True)
            _lib.prof_collect()
            for _ in range(args.steps):
                step(*inputs)
            torch.cuda.synchronize()
        phase = _lib.prof_collect()
        _lib.prof_enable(False)
    la.check_pending()
    elapsed = max_over_ranks(elapsed, world, dev)
    net, recon, nll, gp = [float(v) for v in out]
    log(f"rank {rank}: dims [{d0},{d1}) last step net={net:.4f} recon={recon:.4f} gp={gp:.4f}; "
        f"phases(ms over {args.steps} steps)={ {k: round(v[0], 3) for k, v in phase.items() if v[1]} }")
    Lr = d1 - d0
    res = {"metric": "ELBO-steps/sec (exact-KL L-VAE step, Health-MNIST N=4096 L=16)",
           "value": args.steps / elapsed, "unit": "ELBO-steps/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": 1000.0 * elapsed / args.steps, "higher_is_better": True,
           "scaling": "strong" if world > 1 else "weak", "vs_baseline": None, "dtype": DTYPE,
           "data": "synthetic (Health-MNIST-shaped covariates/images, random-init ConvVAE)",
           "config": {"workload": f"closed-form KL step (standard_training, type_KL='closed'): N={N} (P={P} subjects "
                                  f"x T={T}), L={L}, R=5 additive components (config/LVAE_config_sample.txt)",
                      "N": N, "L": L,
                      "parallelism": (f"rank-share rehearsal on one GPU: rank 0 of {share} ({Lr} dims, {N // share} "
                                      f"images), collectives replaced by local stand-ins -- NOT the union step"
                                      if share > 1 else
                                      "single GPU, LatentShardedClosedStep through a world-1 RCCL group"
                                      if args.sharded_world1 and world == 1 else
                                      ("single GPU, the step replayed as one HIP graph" if use_graph else "single GPU")
                                      if world == 1 else
                                      f"latent dims sharded over {world} ranks ({Lr} dims/rank on rank 0), images "
                                      f"split {N // world}/rank, 1 all-gather + 2 all-reduces per step")}}
    if clocks and clocks.record():
        res["clock"] = clocks.record()
    # host-side pacing: the loop's host time per step, and the queued GPU work left when the host finished (a
    # drain of about one step or less: the host, not the GPU, paced the loop)
    res["host"] = {"enqueue_ms_per_step": 1000.0 * t_enq / args.steps, "drain_ms": 1000.0 * (elapsed - t_enq)}
    if phase and Lr > 0:
        np_ = _lib.load().lvae_kl_closed_padded_n(N)
        potrf_ms = phase["potrf"][0] / args.steps
        potri_ms = phase.get("potri", (0.0, 0))[0] / args.steps
        syrk_ms = phase["syrk"][0] / args.steps
        res["gp_cholesky_gflops"] = Lr * N ** 3 / 3 / (potrf_ms * 1e-3) / 1e9 if potrf_ms > 0 else None
        res["gp_cholesky_gflops_basis"] = (f"L*N^3/3 (the LAPACK potrf count, SURVEY.md §8(d)) / time of the blocked "
                                           f"Cholesky factorisation phase (potrf: {potrf_ms:.2f} ms/step on rank 0; the "
                                           f"triangular inverse + product, trtri + lauum, take {potri_ms:.2f} ms more)")
        res["phase_ms_per_step"] = {k: v[0] / args.steps for k, v in phase.items() if v[1]}
        if use_graph:
            res["phase_timing"] = (f"HIP events around the library's launches over {args.steps} eager steps run "
                                   f"right after the graph-timed region (the same kernels, host-enqueued)")
        # the rooflines of the step's throughput-bound kernels, each on its average launch (the committed
        # rocprofv3 summary of this command where there is one for the shape, else live HIP events); the
        # primary "roofline" is the one with the most GPU time per step
        roofs = []
        hb_ms, hb_n = phase.get("hb_slab", (0.0, 0))
        hyper_binned = hb_n > 0 and hb_ms > syrk_ms * args.steps  # (the route that did the work: the other exits)
        res["hyper_route"] = ("binned (kl_hyper.hip: no S GEMM)" if hyper_binned else
                              "S GEMM + table adjoint (LVAE_KL_HYPER=0 or the binned route's conditions unmet)")
        headline_prof = world == 1 and Lr == 16 and np_ == 4096
        if not hyper_binned and syrk_ms > 0:
            # the S GEMM S = K^-1 V K^-1 (one launch per step), L np^2 (np + 1) fp32-equivalent flop (lower
            # 256-tiles incl. the diagonal ones, whole), each a 3-product f16 split: 3 x that in f16 MFMA flop
            flops = Lr * np_ * np_ * (np_ + 1)
            ach_ev = X3_PRODUCTS * flops / (syrk_ms * 1e-3) / 1e12
            prof = kstats_avg_us("syrk_c16_kernel") if headline_prof else None
            avg_us = prof[0] if prof else syrk_ms * 1e3
            ach = X3_PRODUCTS * flops / (avg_us * 1e-6) / 1e12
            roofs.append((syrk_ms, {
                "kernel": "syrk_c16_kernel<5> (S = K^-1 V K^-1, syrk_x3.hip on the chunk-major core x3_c16.hpp)",
                "bound": "mfma", "achieved": ach, "peak": F16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": ach / F16_MFMA_PEAK_TFLOPS,
                "traffic": pmc_traffic(("syrk_c16_kernel",)) if world == 1 else None,
                "traffic_source": os.path.basename(PMC_SUMMARY), "algorithmic_flop_per_launch": X3_PRODUCTS * flops,
                "fp32_equivalent_tflops": flops / (avg_us * 1e-6) / 1e12, "avg_launch_us": avg_us,
                "avg_launch_source": (f"profiles/{os.path.basename(KSTATS)} (rocprofv3 --kernel-trace --stats of this "
                                      f"bench command, {prof[1]} launches)") if prof else "live HIP events",
                "achieved_event": ach_ev, "frac_event": ach_ev / F16_MFMA_PEAK_TFLOPS, "avg_launch_us_event": syrk_ms * 1e3,
                "engine": "f16 MFMA (v_mfma_f32_32x32x16_f16), 3-product split: achieved counts the 3 f16 products "
                          "per fp32-equivalent product"}))
        if hyper_binned:
            # the binned route's slab pass: one streaming read of the symmetric K^-1 (fp32, L np^2 x 4 B) per
            # launch; its other inputs (bins, keys, tables: O(np)) and its record writes (O(L np/64 x 8 KB)) apart
            hb_step_ms = hb_ms / args.steps
            hbytes = Lr * np_ * np_ * 4
            prof = kstats_avg_us("hb_slab_kernel") if headline_prof else None
            avg_us = prof[0] if prof else hb_ms / hb_n * 1e3
            ach = hbytes / (avg_us * 1e-6) / 1e9
            ach_ev = hbytes / (hb_ms / hb_n * 1e-3) / 1e9
            roofs.append((hb_step_ms, {
                "kernel": "hb_slab_kernel (binned hyper-gradient slab pass over K^-1, kl_hyper.hip)",
                "bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                "traffic": pmc_traffic(("hb_slab_kernel",)) if world == 1 else None,
                "traffic_source": os.path.basename(PMC_SUMMARY), "algorithmic_bytes_per_launch": hbytes,
                "avg_launch_us": avg_us,
                "avg_launch_source": (f"profiles/{os.path.basename(KSTATS)} (rocprofv3 --kernel-trace --stats of this "
                                      f"bench command, {prof[1]} launches)") if prof else "live HIP events",
                "achieved_event": ach_ev, "frac_event": ach_ev / HBM_PEAK_GBS, "avg_launch_us_event": hb_ms / hb_n * 1e3}))
        # the trailing rank-256 update of the Cholesky (U2, HBM-streaming); per step the passes k = 0 .. nt-3
        # update (nt-k-2)(nt-k-1)/2 tiles per dim, each read and written once in fp32 (at <= CI_FUSE_MAX_L dims
        # the same launch also turns column k+1's nt-k-2 tiles into the next pass's planes: read fp32, write 2
        # fp16 planes, the same 8 bytes per element)
        nt = np_ // 256
        fused = Lr <= CI_FUSE_MAX_L
        upd_ms, upd_n = phase.get("sweep_update", (0.0, 0))
        tiles = sum((nt - k - 2) * (nt - k - 1) // 2 + (nt - k - 2 if fused else 0) for k in range(nt - 2)) * Lr
        upd_bytes = 2 * 4 * 256 * 256 * tiles
        u2_name = U2_NAMES[fused]
        if upd_n:
            launches = upd_n / args.steps
            prof = kstats_avg_us(u2_name) if headline_prof else None
            avg_us = prof[0] if prof else upd_ms / upd_n * 1e3
            ach = upd_bytes / launches / (avg_us * 1e-6) / 1e9
            ach_ev = upd_bytes / (upd_ms / args.steps * 1e-3) / 1e9
            roofs.append((upd_ms / args.steps, {
                "kernel": f"{u2_name} (potrf trailing rank-256 update U2{' + U1' if fused else ''}, chol_inv.hip)",
                "bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                "traffic": pmc_traffic((u2_name,), per_step=True) / launches if (world == 1 and pmc_traffic(
                    (u2_name,), per_step=True)) else None,
                "traffic_source": os.path.basename(PMC_SUMMARY),
                "algorithmic_bytes_per_step": upd_bytes, "algorithmic_bytes_per_launch": upd_bytes / launches,
                "avg_launch_us": avg_us,
                "avg_launch_source": (f"profiles/{os.path.basename(KSTATS)} ({prof[1]} launches)") if prof
                                     else "live HIP events", "launches_per_step": launches,
                "achieved_event": ach_ev, "frac_event": ach_ev / HBM_PEAK_GBS,
                "avg_launch_us_event": upd_ms / upd_n * 1e3, "padded_n": int(np_)}))
        if headline_prof:
            # north_star's "MFMA utilisation against the gfx950 peak": the matrix pipes' busy fraction per kernel
            mu = {}
            for what, kname in MFMA_KERNELS.items():
                b = mfma_busy(kname)
                if b:
                    mu[what] = {"kernel": kname, "mfma_busy_frac": b[0], "dispatches_profiled": b[1]}
            if mu:
                res["mfma_utilisation"] = dict(mu, source=f"profiles/{os.path.basename(MFMA_PMC)} (rocprofv3 --pmc "
                                               "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE over this bench's closed step; "
                                               "busy / (1024 SIMDs x GRBM_GUI_ACTIVE / 8))")
            for _, r in roofs:
                b = mfma_busy(r["kernel"].split(" ")[0])
                if b:
                    r["mfma_busy_frac"] = b[0]
        roofs.sort(key=lambda r: -r[0])
        for i, (ms, r) in enumerate(roofs):
            r["gpu_ms_per_step"] = ms
            res["roofline" if i == 0 else ("roofline_secondary" if i == 1 else f"roofline_{i + 1}")] = r
    return res


# ------------------------------------------------------------------------------------------
# Regime A: Hensman SVI step, HIP-graph replayed
# ------------------------------------------------------------------------------------------
def run_hensman(args, world, rank, dev, dp_hooks=False):
    import lvae_amd as la
    from lvae_amd.data import health_mnist_batch
    from lvae_amd.samplers import check_same_permutation, hensman_batches, SubjectSampler
    from lvae_amd.steps import GraphedStep, HensmanStep
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
                            {"params": vae.parameters()}], lr=1e-3, capturable=True, fused=True)
    hook = ngr = None
    if world > 1 or dp_hooks:  # (dp_hooks at world 1: the data-parallel step through a world-1 RCCL group)
        from lvae_amd.distributed import GradAllReduce, allreduce_tensors
        hook = GradAllReduce(list(vae.parameters()) + list(k0.parameters()) + list(k1.parameters()), world)
        ngr = lambda ts: allreduce_tensors(ts, average=False)
    step = HensmanStep(vae, k0, k1, lik, opt, m, H, z, P, T, weight=0.15, natural_gradient=True,
                       natural_gradient_lr=0.01, world=world, grad_hook=hook, ng_reduce=ngr)
    perm = SubjectSampler(P, T, seed=0).permutation()
    if world > 1:
        check_same_permutation(perm)  # once per run (a collective)
    batches = [b.to(dev) for b in hensman_batches(perm, P_b, T, rank, world) if b is not None and len(b) == P_b * T]
    gen = torch.Generator(device=dev).manual_seed(7 + rank)
    eps = torch.randn(P_b * T, L, device=dev, generator=gen)
    rows = batches[0].clone()
    s_img, s_mask, s_X = img.index_select(0, rows), mask.index_select(0, rows), X.index_select(0, rows)

    def load(i):  # next batch into the static inputs (device gathers, no host sync)
        r = batches[i % len(batches)]
        torch.index_select(img, 0, r, out=s_img)
        torch.index_select(mask, 0, r, out=s_mask)
        torch.index_select(X, 0, r, out=s_X)

    graphed = GraphedStep(step, (s_img, s_mask, s_X, eps), warmup=max(args.warmup, 2))
    for i in range(args.warmup):
        load(i)
        graphed()
    torch.cuda.synchronize()
    graphed.check()
    sync_barrier(world)
    t0 = time.perf_counter()
    for i in range(args.h_steps):
        load(i)
        out = graphed()
    sync_barrier(world)
    elapsed = max_over_ranks(time.perf_counter() - t0, world, dev)
    graphed.check()
    log(f"rank {rank}: Hensman last step (net, recon, nll, kld) = {[round(float(v), 4) for v in out]}")
    value = args.h_steps / elapsed
    return {"metric": "ELBO-steps/sec (Hensman SVI step, training.py:90-140)", "value": value,
            "unit": "ELBO-steps/s", "ms_per_step": 1000.0 * elapsed / args.h_steps, "steps": args.h_steps,
            "samples_per_sec": value * world * P_b * T, "scaling": "weak",
            "dtype": "fp64 GP (f64 MFMA / VALU) + fp32 ConvVAE",
            "config": {"workload": f"Hensman step: P_tot={P} subjects x T={T} (N={N}), L={L}, M={M}, P_b={P_b} "
                                   f"subjects per rank per step, natural gradient, one HIP graph per step"
                                   + (" (two around the all-reduces)" if world > 1 or dp_hooks else ""),
                       "parallelism": f"dp{world} over subject mini-batches"}}


# ------------------------------------------------------------------------------------------
# C2: HIP Gram + inverse vs PyTorch-ROCm Gram + torch.linalg.cholesky (N = 1024, L = 8)
# ------------------------------------------------------------------------------------------
def run_hensman_dp_world1(args, dev):
    """Regime A's data-parallel step at world 1: the SUM all-reduces of the Adam gradients and of the natural-
    gradient statistics through a world-1 RCCL ("nccl") group, i.e. the step as two HIP graphs around the eager
    collectives (GraphedStep with grad_hook / ng_reduce) -- the per-rank shape of the N-GPU Regime A line without
    the other ranks.  Reported beside the one-graph step (the same batches)."""
    created = False
    if not dist.is_initialized():
        import socket
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            os.environ["MASTER_PORT"] = str(so.getsockname()[1])
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        dist.init_process_group("nccl", device_id=dev)
        created = True
    try:
        r = run_hensman(args, 1, 0, dev, dp_hooks=True)
    finally:
        if created:
            dist.destroy_process_group()
    return {"ms_per_step": r["ms_per_step"], "value": r["value"], "unit": r["unit"],
            "config": r["config"]["workload"],
            "note": "world-1 RCCL group: GradAllReduce + natural-gradient statistics all-reduce between the two graphs"}


def torch_gram_f32(params, X):
    """The sample-config additive Gram (+ noise = 1 on the diagonal) in plain PyTorch fp32 ops."""
    x = X.to(torch.float32)
    t, dt, subj, gen, dis = x[:, 0], x[:, 1], x[:, 2], x[:, 3], x[:, 4]
    p = params.to(torch.float32)[:, :, None, None]
    rbf = lambda a, ell: torch.exp(-(a[:, None] - a[None, :]) ** 2 / (2 * ell ** 2))
    cat = lambda a: (a[:, None] == a[None, :]).to(torch.float32)
    K = (p[:, 0] * cat(subj) + p[:, 1] * rbf(t, p[:, 2]) + p[:, 3] * cat(subj) * rbf(t, p[:, 4])
         + p[:, 5] * cat(gen) * rbf(t, p[:, 6]) + p[:, 7] * cat(dis) * rbf(dt, p[:, 8]))
    return K + torch.eye(x.shape[0], device=x.device)


def run_c2(dev, reps=20):
    """BASELINE configs[1]: the product's Gram + blocked Cholesky route (lvae_gram_f32 +
    lvae_spd_inv_chol_f32: potrf, trtri, lauum -- the inverse KL_closed uses, elbo_functions.py:26-29)
    against PyTorch-ROCm fp32 Gram + torch.linalg.cholesky (rocSOLVER potrf) and + cholesky_inverse.
    gp_cholesky_gflops_hip is the potrf phase ALONE (the library's HIP events around its potrf
    sequence, LVAE_PH_POTRF), against torch.linalg.cholesky alone; the whole inverse is compared with
    cholesky + cholesky_inverse."""
    import lvae_amd as la
    from lvae_amd import _lib
    from lvae_amd.data import health_mnist_covariates
    P, T, L = 64, 16, 8
    N = P * T
    X = torch.tensor(health_mnist_covariates(P, T, seed=2), device=dev)
    k = la.generate_kernel(**CFG, latent_dim=L).to(dev)
    spec, params = la.kernel_spec_and_params(k)
    params = params.detach().contiguous()
    lib = _lib.load()
    np_ = lib.lvae_kl_closed_padded_n(N)
    A = torch.empty(L, np_, np_, dtype=torch.float32, device=dev)
    Kinv = torch.empty_like(A)
    scr = torch.empty(int(lib.lvae_spd_inv_chol_scratch_size(np_, L)), dtype=torch.uint8, device=dev)
    logdet = torch.empty(L, dtype=torch.float64, device=dev)
    info = torch.empty(L, dtype=torch.int32, device=dev)
    noise = torch.ones(L, dtype=torch.float64, device=dev)
    xv = _lib.xview(X, 0, 0)

    def gram():
        _lib.check(lib.lvae_gram_f32(spec, xv, xv, 1, L, N, N, _lib.ptr(params), _lib.ptr(noise), _lib.ptr(A), 0,
                                     np_ * np_, np_, _lib.stream_ptr()), "gram")

    def hip():
        gram()
        _lib.check(lib.lvae_spd_inv_chol_f32(np_, L, _lib.ptr(A), _lib.ptr(scr), _lib.ptr(Kinv), _lib.ptr(logdet),
                                             _lib.ptr(info), _lib.stream_ptr()), "chol")

    def torch_chol():
        return torch.linalg.cholesky(torch_gram_f32(params, X))

    def torch_potrf_only(Kt):
        return torch.linalg.cholesky(Kt)

    def torch_chol_inv():
        Lc = torch_chol()
        return torch.cholesky_inverse(Lc), 2 * torch.log(torch.diagonal(Lc, dim1=-2, dim2=-1)).sum(-1)

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    # the potrf phase of the product route alone (HIP events around the library's potrf sequence)
    for _ in range(3):
        hip()
    torch.cuda.synchronize()
    _lib.prof_enable(True)
    _lib.prof_collect()
    for _ in range(reps):
        hip()
    ph = _lib.prof_collect()
    _lib.prof_enable(False)
    t_potrf = ph["potrf"][0] / max(ph["potrf"][1], 1)
    t_hip = timed(hip)
    info_ok = int(info.abs().sum()) == 0
    inv_chol = Kinv[:, :N, :N].clone()
    ld_chol = logdet.clone()
    Kt = torch_gram_f32(params, X)
    t_gram_torch = timed(lambda: torch_gram_f32(params, X))
    t_potrf_torch = timed(lambda: torch_potrf_only(Kt))
    t_chol, t_inv = timed(torch_chol), timed(torch_chol_inv)
    # the exported N x N factor (lvae_potrf_f32 / _f64 through lvae_amd.linalg) on the same prebuilt Gram,
    # against torch.linalg.cholesky on it: the same input, the same output (L)
    import lvae_amd.linalg as LA
    t_potrf_export = timed(lambda: LA.cholesky_ex(Kt))
    Kt64 = Kt.double()
    t_potrf64_export = timed(lambda: LA.cholesky_ex(Kt64))
    t_potrf64_torch = timed(lambda: torch_potrf_only(Kt64))
    L32 = LA.cholesky_ex(Kt)[0]
    Lref64 = torch.linalg.cholesky(Kt64)
    err_l32 = float((L32.double() - Lref64).abs().max() / Lref64.abs().max())
    err_l64 = float((LA.cholesky_ex(Kt64)[0] - Lref64).abs().max() / Lref64.abs().max())
    ref_inv, ref_ld = torch_chol_inv()
    err = float((inv_chol - ref_inv).abs().max() / ref_inv.abs().max())
    flop = L * N ** 3 / 3
    return {"config": f"N={N} (P={P} x T={T}), L={L}, sample-config kernel, fp32",
            "hip_route": "lvae_gram_f32 + lvae_spd_inv_chol_f32 (blocked potrf + trtri + lauum, chol_inv.hip)",
            "hip_gram_chol_inverse_ms": t_hip, "hip_potrf_ms": t_potrf,
            "torch_gram_ms": t_gram_torch, "torch_potrf_ms": t_potrf_torch,
            "torch_gram_cholesky_ms": t_chol, "torch_gram_cholesky_inverse_ms": t_inv,
            "speedup_potrf_vs_torch_cholesky": t_potrf_torch / t_potrf if t_potrf > 0 else None,
            "speedup_vs_torch_cholesky_inverse": t_inv / t_hip,
            "gp_cholesky_gflops_hip": flop / (t_potrf * 1e-3) / 1e9 if t_potrf > 0 else None,
            "gp_cholesky_gflops_torch": flop / (t_potrf_torch * 1e-3) / 1e9,
            "gp_cholesky_gflops_basis": "L*N^3/3 / potrf time alone (HIP: the library's potrf phase events; "
                                        "torch: torch.linalg.cholesky on the prebuilt fp32 Gram)",
            "hip_vs_torch_inverse_max_rel_diff": err, "hip_info_ok": info_ok,
            "logdet_max_rel_diff": float(((ld_chol.float() - ref_ld).abs() / ref_ld.abs()).max()),
            "potrf_export": {"lvae_potrf_f32_ms": t_potrf_export, "torch_cholesky_f32_ms": t_potrf_torch,
                             "speedup_f32": t_potrf_torch / t_potrf_export,
                             "gflops_f32": flop / (t_potrf_export * 1e-3) / 1e9,
                             "lvae_potrf_f64_ms": t_potrf64_export, "torch_cholesky_f64_ms": t_potrf64_torch,
                             "speedup_f64": t_potrf64_torch / t_potrf64_export,
                             "gflops_f64": flop / (t_potrf64_export * 1e-3) / 1e9,
                             "L_max_rel_diff_vs_torch_f64": {"f32": err_l32, "f64": err_l64},
                             "note": "the C-ABI N x N factor (potrf.hip) on the prebuilt Gram, returning L, vs "
                                     "torch.linalg.cholesky (rocSOLVER) on the same matrix; f32 includes the copy "
                                     "into the padded workspace and out of it"},
            "note": "HIP: Gram + Cholesky route (K^-1 and log|K|); torch: PyTorch fp32 Gram + torch.linalg.cholesky "
                    "(rocSOLVER) [+ cholesky_inverse + log-det for the same outputs]"}


def main():
    # ONE JSON line on stdout: libraries that print there (RCCL's version banner at communicator init,
    # MIOpen notes) write to stderr instead -- fd 1 is pointed at fd 2 and the line goes to the saved fd
    out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--P", type=int, default=256, help="subjects (N = P*T)")
    ap.add_argument("--T", type=int, default=16)
    ap.add_argument("--L", type=int, default=16)
    ap.add_argument("--P_b", type=int, default=5, help="Regime A: subjects per batch per rank")
    ap.add_argument("--M", type=int, default=120, help="Regime A: inducing points")
    ap.add_argument("--h-steps", dest="h_steps", type=int, default=100, help="Regime A timed steps")
    # default: both regimes at every N -- the exact-KL line (latent dims sharded over the ranks at N > 1) and its
    # `regime_a` sub-record (BASELINE configs[3]: the Hensman step data parallel over subject mini-batches, two HIP
    # graphs around the RCCL all-reduces at N > 1)
    ap.add_argument("--regime", choices=["auto", "both", "closed", "hensman"], default="auto")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-phase-timing", action="store_true")
    ap.add_argument("--no-c2", action="store_true")
    ap.add_argument("--graph", action="store_true",
                    help="closed regime on one GPU: time the step as one replayed HIP graph (slower, see run_closed)")
    ap.add_argument("--sharded-world1", dest="sharded_world1", action="store_true",
                    help="one GPU: the latent-sharded step (distributed.LatentShardedClosedStep) through a world-1 "
                         "RCCL group instead of ClosedStep (its overlap against the single-GPU step's)")
    ap.add_argument("--rank-share", dest="rank_share", type=int, default=0,
                    help="one GPU: time rank 0's share of a W-rank latent-sharded step (L/W dims, N/W images; "
                         "collectives replaced by local stand-ins) -- the per-rank compute of the W-GPU line")
    ap.add_argument("--no-dp-world1", dest="dp_world1", action="store_false",
                    help="one GPU: skip timing Regime A's data-parallel step (two graphs around the all-reduces) "
                         "through a world-1 RCCL group (the regime_a.dp_world1_rccl sub-record)")
    ap.add_argument("--vae-stream-priority", dest="vae_stream_priority", type=int, default=-1,
                    help="priority of the ConvVAE's stream in the closed step (lower = higher; 0 = default)")
    args = ap.parse_args()

    world, rank, local = setup_dist(force_group=args.sharded_world1)
    dev = torch.device("cuda", local)
    if args.regime == "auto":
        args.regime = "both"
    res = None
    if args.regime in ("both", "closed"):
        res = run_closed(args, world, rank, dev)
    if args.regime in ("both", "hensman"):
        if res is not None:
            # (the sub-record of the closed line: a failure here is recorded in it, the line itself stands)
            try:
                ra = run_hensman(args, world, rank, dev)
            except Exception as e:
                if os.environ.get("LVAE_BENCH_RAISE") == "1":
                    raise
                ra = {"error": f"{type(e).__name__}: {e}"[:300]}
        else:
            ra = run_hensman(args, world, rank, dev)
        if world == 1 and args.dp_world1:
            try:
                ra["dp_world1_rccl"] = run_hensman_dp_world1(args, dev)
            except Exception as e:  # (a record of the failure; the line itself stands)
                if os.environ.get("LVAE_BENCH_RAISE") == "1":
                    raise
                ra["dp_world1_rccl"] = {"error": f"{type(e).__name__}: {e}"[:300]}
        if res is None:
            res = dict(ra, n_gpus=world, warmup=args.warmup, higher_is_better=True, vs_baseline=None,
                       data="synthetic (Health-MNIST-shaped covariates/images, random-init ConvVAE)")
        else:
            res["regime_a"] = ra
    if rank == 0:
        if world == 1 and not args.no_c2 and args.regime != "hensman":
            res["c2"] = run_c2(dev)
        if world == 1 and not args.no_cpu_baseline:
            if args.regime in ("both", "closed"):
                res["cpu_baseline"] = cpu_baseline_closed(args.P, args.T, args.L)
                res["vs_cpu_baseline"] = res["value"] / res["cpu_baseline"]["value"]
            ra = res["regime_a"] if "regime_a" in res else res
            if args.regime in ("both", "hensman") and "value" in ra:
                cb = cpu_baseline_hensman(args.P, args.T, args.L, args.M, args.P_b)
                ra["cpu_baseline"] = cb
                ra["vs_cpu_baseline"] = ra["value"] / cb["value"]
                if "regime_a" not in res:
                    res["vs_cpu_baseline"] = ra["vs_cpu_baseline"]
        print(json.dumps(res), file=out, flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
