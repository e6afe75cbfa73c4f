"""Dev: the ConvVAE's linear-layer GEMMs at the headline batch (B = 4096; VAE.py fc1 .. fc4, latent L):
forward y = x W^T, backward dX = g W and dW = g^T x, fp32, timed per backend (hipBLASLt / rocBLAS via
torch.backends.cuda.preferred_blas_library), plus the same products as an explicit split-K sum for the
tall-skinny dW shapes."""
import sys

import torch

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
L = int(sys.argv[2]) if len(sys.argv) > 2 else 16
LAYERS = {"fc1": (2592, 300), "fc21": (300, 30), "fc211": (30, L), "fc221": (30, L), "fc3": (L, 30),
          "fc31": (30, 300), "fc4": (300, 2592)}


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    dev = torch.device("cuda")
    for lib in ("cublaslt", "cublas"):
        torch.backends.cuda.preferred_blas_library(lib)
        tot = 0.0
        for name, (fi, fo) in LAYERS.items():
            x = torch.randn(B, fi, device=dev)
            W = torch.randn(fo, fi, device=dev)
            g = torch.randn(B, fo, device=dev)
            t_f = timeit(lambda: x @ W.t())
            t_dx = timeit(lambda: g @ W)
            t_dw = timeit(lambda: g.t() @ x)
            t_dw8 = timeit(lambda: torch.bmm(g.t().reshape(fo, 8, B // 8).transpose(0, 1),
                                             x.reshape(8, B // 8, fi)).sum(0))
            tot += t_f + t_dx + t_dw
            print(f"{lib:9s} {name:6s} [{B}x{fi}]->{fo}: fwd {t_f:7.1f} us  dX {t_dx:7.1f} us  dW {t_dw:7.1f} us  "
                  f"dW split-8 {t_dw8:7.1f} us", flush=True)
        print(f"{lib}: total fwd + dX + dW {tot:.0f} us", flush=True)


if __name__ == "__main__":
    main()
