"""Time the ConvVAE forward + backward at the headline batch (4096 x 1 x 36 x 36, L = 16) under
memory-format / backend variants (diagnostic; not part of the product path)."""
import sys, os, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "longitudinal-vae_amd"))
import torch
from lvae_amd.vae import ConvVAE

dev = torch.device("cuda")
B, L = int(os.environ.get("B", 4096)), 16


def run(name, cl=False, bench=False):
    torch.backends.cudnn.benchmark = bench
    torch.manual_seed(0)
    vae = ConvVAE(L, 1296, p_input=0.0, p=0.0).to(dev)
    x = torch.rand(B, 1, 36, 36, device=dev)
    mask = (torch.rand(B, 1, 36, 36, device=dev) < 0.75).float()
    eps = torch.randn(B, L, device=dev)
    if cl:
        vae = vae.to(memory_format=torch.channels_last)
        x = x.contiguous(memory_format=torch.channels_last)
    def step():
        vae.zero_grad(set_to_none=False)
        recon, mu, lv = vae(x, eps)
        mse, nll = vae.loss_function(recon, x, mask)
        (mse.sum() + (mu.sum() + lv.sum()) * 1e-3).backward()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    print(f"{name:30s} {1000 * (time.perf_counter() - t0) / 10:8.3f} ms", flush=True)


run("default")
run("cudnn.benchmark", bench=True)
run("channels_last", cl=True)
run("channels_last+benchmark", cl=True, bench=True)
