"""MIOpen's accuracy on the ConvVAE's library convolutions at the bench's 4096 images, against fp64 on the
CPU: the encoder's conv2 (3x3, 16 -> 32, 18 x 18; forward, input and weight gradients) and the decoder's
deconv1 weight gradient (ConvTranspose2d(32, 16, 4, 2, 1)).  Run with LVAE_MIOPEN_WINOGRAD=1 for MIOpen's
default solvers (lvae_amd turns the Winograd ones off otherwise)."""
import sys
import torch
sys.path.insert(0, "longitudinal-vae_amd")
import lvae_amd  # noqa: F401  (MIOpen solver policy)


def rel(a, b):
    a = a.detach().cpu().double(); b = b.detach().cpu().double()
    return float((a - b).abs().max() / b.abs().max())


N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
torch.manual_seed(5)
x = torch.randn(N, 16, 18, 18, device="cuda", requires_grad=True)
w = torch.randn(32, 16, 3, 3, device="cuda", requires_grad=True)
y = torch.nn.functional.conv2d(x, w, None, 1, 1)
g = torch.randn_like(y)
(y * g).sum().backward()
x64, w64 = x.detach().cpu().double().requires_grad_(), w.detach().cpu().double().requires_grad_()
y64 = torch.nn.functional.conv2d(x64, w64, None, 1, 1)
(y64 * g.cpu().double()).sum().backward()
print(f"conv2 N={N}: y {rel(y, y64):.2e} dx {rel(x.grad, x64.grad):.2e} dw {rel(w.grad, w64.grad):.2e}")
z = torch.randn(N, 32, 9, 9, device="cuda")
wd = torch.randn(32, 16, 4, 4, device="cuda")
gd = torch.randn(N, 16, 18, 18, device="cuda")
dw = torch.ops.aten.convolution_backward(gd, z, wd, None, [2, 2], [1, 1], [1, 1], True, [0, 0], 1, [False, True, False])[1]
z64, wd64 = z.cpu().double(), wd.cpu().double().requires_grad_()
(torch.nn.functional.conv_transpose2d(z64, wd64, None, 2, 1) * gd.cpu().double()).sum().backward()
print(f"deconv1 wgrad N={N}: dw {rel(dw, wd64.grad):.2e}")
