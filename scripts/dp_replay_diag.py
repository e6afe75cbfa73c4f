"""Diagnose the data-parallel two-graph Hensman replay (GraphedStep with grad_hook / ng_reduce).

One process, one GPU.  Builds bench.py's Regime A step and replays it as two graphs around the
collectives, 100 times back to back, then reads every deferred info array and checks (m, H).
Variants (env):
  DIAG_COMM  = rccl | fake | none   the collectives through a world-1 RCCL group, the same flatten / copy
                                    without any process group, or no-op hooks (still two graphs)
  DIAG_POOL  = own | shared         g2 captured in its own private pool or in g1's
  DIAG_SYNC  = k                    torch.cuda.synchronize() after every k-th replay (0 = never)
  DIAG_STEPS = n                    replays (default 100)
  DIAG_L, DIAG_M                    shapes (default 4, 40)
"""
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "longitudinal-vae_amd"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

CFG = dict(cat_kernel=[2], bin_kernel=[], sqexp_kernel=[0],
           cat_int_kernel=[{'cont_covariate': 0, 'cat_covariate': 2},
                           {'cont_covariate': 0, 'cat_covariate': 3},
                           {'cont_covariate': 1, 'cat_covariate': 4}],
           bin_int_kernel=[], covariate_missing_val=[])


def main():
    import lvae_amd as la
    from lvae_amd.data import health_mnist_batch
    from lvae_amd.distributed import GradAllReduce, allreduce_tensors
    from lvae_amd.samplers import SubjectSampler, hensman_batches
    from lvae_amd.steps import GraphedStep, HensmanStep
    from lvae_amd.vae import ConvVAE
    from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors

    comm = os.environ.get("DIAG_COMM", "rccl")
    steps = int(os.environ.get("DIAG_STEPS", "100"))
    sync_every = int(os.environ.get("DIAG_SYNC", "0"))
    L, M = int(os.environ.get("DIAG_L", "4")), int(os.environ.get("DIAG_M", "40"))
    P, T, P_b = 256, 16, 5
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if comm == "rccl":
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    la.set_sync_checks(False)
    N = P * T
    torch.manual_seed(1234)
    vae = ConvVAE(L, 1296, p_input=0.0, p=0.0).to(dev)
    k0, k1 = la.generate_kernel_batched(L, **CFG, id_covariate=2)
    k0, k1 = k0.to(dev), k1.to(dev)
    lik = la.GaussianLikelihood(L, noise=1.0, constrain=False).to(dev)
    img, mask, X = health_mnist_batch(P, T, seed=100, device=dev)
    z = torch.stack([torch.cat([X[0:M // 2], X[N // 2:N // 2 + M // 2]])] * L)
    with torch.no_grad():
        H = k0(z, z).evaluate() + 1e-6 * torch.eye(M, dtype=torch.float64, device=dev)
    m = torch.zeros(L, M, 1, dtype=torch.float64, device=dev)
    params = list(vae.parameters()) + list(k0.parameters()) + list(k1.parameters())
    opt = torch.optim.Adam([{"params": k0.parameters()}, {"params": k1.parameters()},
                            {"params": vae.parameters()}], lr=1e-3, capturable=True, fused=True)

    def fake_reduce(ts):
        flat = _flatten_dense_tensors(ts)
        for t, r in zip(ts, _unflatten_dense_tensors(flat, ts)):
            t.copy_(r)

    if comm == "rccl":
        hook = GradAllReduce(params, 1)
        ngr = lambda ts: allreduce_tensors(ts, average=False)
    elif comm == "fake":
        hook = lambda: fake_reduce([p.grad for p in params if p.grad is not None])
        ngr = fake_reduce
    else:
        hook = lambda: None
        ngr = lambda ts: None
    step = HensmanStep(vae, k0, k1, lik, opt, m, H, z, P, T, weight=0.15, natural_gradient=True,
                       natural_gradient_lr=0.01, world=1, grad_hook=hook, ng_reduce=ngr)
    perm = SubjectSampler(P, T, seed=0).permutation()
    batches = [b.to(dev) for b in hensman_batches(perm, P_b, T, 0, 1) if b is not None and len(b) == P_b * T]
    eps = torch.randn(P_b * T, L, device=dev, generator=torch.Generator(device=dev).manual_seed(7))
    rows = batches[0].clone()
    s_img, s_mask, s_X = img.index_select(0, rows), mask.index_select(0, rows), X.index_select(0, rows)

    def load(i):
        r = batches[i % len(batches)]
        torch.index_select(img, 0, r, out=s_img)
        torch.index_select(mask, 0, r, out=s_mask)
        torch.index_select(X, 0, r, out=s_X)

    if os.environ.get("DIAG_NOMIOPEN") == "1":
        torch.backends.cudnn.enabled = False  # (MIOpen off: PyTorch's own convolution kernels)
    real_empty = torch.cuda.empty_cache
    if os.environ.get("DIAG_NOEMPTY") == "1":
        torch.cuda.empty_cache = lambda: None  # (torch.cuda.graph's empty_cache at each capture start)
    hist = os.environ.get("DIAG_HIST") == "1"
    if hist:
        torch.cuda.memory._record_memory_history(max_entries=200000)
    g = GraphedStep(step, (s_img, s_mask, s_X, eps), warmup=3, shared_pool=os.environ.get("DIAG_POOL") == "shared")
    torch.cuda.empty_cache = real_empty
    print(f"comm={comm} pool={os.environ.get('DIAG_POOL', 'own')} L={L} M={M} two graphs: {g.g2 is not None}",
          flush=True)
    for info, what in g.pending:
        print(f"  pending {what[:40]!r}: ptr {info.data_ptr():#x} numel {info.numel()}", flush=True)
    for i in range(steps):
        load(i)
        g()
        if sync_every and (i + 1) % sync_every == 0:
            torch.cuda.synchronize()
            for info, what in g.pending:
                if int(info.abs().sum()):
                    print(f"  replay {i}: {what[:40]!r} info = {info.tolist()}", flush=True)
    torch.cuda.synchronize()
    bad = 0
    for info, what in g.pending:
        v = info.tolist()
        print(f"  final {what[:40]!r}: {v}", flush=True)
        bad += any(v)
    if hist:
        snap = torch.cuda.memory._snapshot()
        targets = [(info.data_ptr(), what[:30]) for info, what in g.pending]
        for tp, what in targets:
            print(f"== events touching {what!r} @ {tp:#x}", flush=True)
            for dev_tr in snap["device_traces"]:
                for ev in dev_tr:
                    a, sz = ev.get("addr", 0), ev.get("size", 0)
                    if a <= tp < a + max(sz, 1):
                        fr = [f"{f['filename'].split('/')[-1]}:{f['line']}:{f['name']}" for f in ev.get("frames", [])
                              if "site-packages" not in f["filename"] and "dist-packages" not in f["filename"]]
                        print(f"  {ev['action']:>16} addr {a:#x} size {sz} stream {ev.get('stream')} "
                              f"{' <- '.join(fr[:6])}", flush=True)
            for seg in snap["segments"]:
                if seg["address"] <= tp < seg["address"] + seg["total_size"]:
                    print(f"  segment {seg['address']:#x} size {seg['total_size']} pool {seg.get('segment_pool_id')} "
                          f"type {seg.get('segment_type')}", flush=True)
                    off = seg["address"]
                    for b in seg["blocks"]:
                        if off <= tp < off + b["size"]:
                            print(f"   block {off:#x} size {b['size']} state {b['state']}", flush=True)
                        off += b["size"]
    fin = bool(torch.isfinite(step.m).all() and torch.isfinite(step.H).all())
    print(f"RESULT comm={comm} bad_info={bad} mH_finite={fin} out={[round(float(x), 3) for x in g.out]}", flush=True)
    if comm == "rccl":
        dist.destroy_process_group()
    return 1 if (bad or not fin) else 0


if __name__ == "__main__":
    sys.exit(main())
