"""Timing harness for the batched SPD sweep alone (L dims of n x n), for rocprofv3 kernel traces.
Usage: python scripts/sweep_micro.py [n] [L] [reps].  LVAE_MICRO_VARIANTS=base[,...] names VARIANTS entries."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "longitudinal-vae_amd"))
import lvae_amd as la  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
L = int(sys.argv[2]) if len(sys.argv) > 2 else 16
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
dev = "cuda"
P = la._lib
hip = P.load()
torch.manual_seed(0)
X = torch.randn(L, n, n, device=dev) / n ** 0.5
A0 = X @ X.transpose(1, 2) + torch.eye(n, device=dev)
del X
scr = torch.zeros(hip.lvae_spd_sweep_scratch_size(n, L) // 4, device=dev)
Ai = torch.zeros_like(A0)
logdet = torch.zeros(L, dtype=torch.float64, device=dev)
info = torch.zeros(L, dtype=torch.int32, device=dev)
A = A0.clone()
VARIANTS = {"base": {}}  # add env overrides here to time variants side by side
for var in os.environ.get("LVAE_MICRO_VARIANTS", "base").split(","):
    os.environ.update(VARIANTS[var])
    ts = []
    for r in range(reps):
        A.copy_(A0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        P.check(hip.lvae_spd_sweep_f32(n, L, P.ptr(A), P.ptr(scr), P.ptr(Ai), P.ptr(logdet), P.ptr(info),
                                       P.stream_ptr()), "spd_sweep")
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    if True:  # residual check (dim 0)
        I = torch.eye(n, device=dev)
        err = float((A0[0] @ Ai[0] - I).abs().max())
        print(f"max|A A^-1 - I| (dim 0) = {err:.3e}, info = {info.tolist()[:4]}")
    print(f"{var} sweep n={n} L={L}: {[round(1e3 * t, 3) for t in ts]} ms  (min {1e3 * min(ts):.3f})", flush=True)
