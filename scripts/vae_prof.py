"""torch.profiler table of one ConvVAE forward + backward at the headline batch (diagnostic)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "longitudinal-vae_amd"))
import torch
from torch.profiler import profile, ProfilerActivity
from lvae_amd.vae import ConvVAE

dev = torch.device("cuda")
B, L = 4096, 16
torch.manual_seed(0)
vae = ConvVAE(L, 1296, p_input=0.0, p=0.0).to(dev)
x = torch.rand(B, 1, 36, 36, device=dev)
mask = (torch.rand(B, 1, 36, 36, device=dev) < 0.75).float()
eps = torch.randn(B, L, device=dev)


def step():
    vae.zero_grad(set_to_none=True)
    recon, mu, lv = vae(x, eps)
    mse, nll = vae.loss_function(recon, x, mask)
    (mse.sum() + (mu.sum() + lv.sum()) * 1e-3).backward()


for _ in range(3):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    for _ in range(3):
        step()
    torch.cuda.synchronize()
print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=45, max_name_column_width=50,
                                                         max_shapes_column_width=70))
