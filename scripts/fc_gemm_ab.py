"""Dev A/B: the ConvVAE fc layers' weight-gradient GEMMs (dW = g^T x over the 4096-image batch, K = 4096) on
hipBLASLt as one torch.mm vs split-K as a torch.bmm over S batch chunks + a fixed-order sum."""
import time

import torch

dev = "cuda"
B = 4096
g0 = torch.Generator(device=dev).manual_seed(0)


def tm(f, n=30):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e6


for out_f, in_f in ((300, 2592), (2592, 300), (30, 300), (300, 30)):
    g = torch.randn(B, out_f, device=dev, generator=g0)
    x = torch.randn(B, in_f, device=dev, generator=g0)
    ref = (g.double().t() @ x.double())
    res = [f"dW [{out_f} x {in_f}]: mm {tm(lambda: torch.mm(g.t(), x)):.1f} us"]
    for S in (2, 4, 8, 16):
        def f(S=S):
            return torch.bmm(g.view(S, B // S, out_f).transpose(1, 2), x.view(S, B // S, in_f)).sum(0)
        err = float((f() - ref).abs().max() / ref.abs().max())
        res.append(f"S={S} {tm(f):.1f} us (err {err:.1e})")
    print("; ".join(res), flush=True)
