import sys, torch
sys.path.insert(0, "longitudinal-vae_amd")
from lvae_amd.vae import deconv_relu
def rel(a, b):
    a = a.detach().cpu().double(); b = b.detach().cpu().double()
    return float((a - b).abs().max() / b.abs().max())
for N in (37, 512, 4096):
    torch.manual_seed(N)
    dc = torch.nn.ConvTranspose2d(32, 16, kernel_size=4, stride=2, padding=1).cuda()
    x = torch.randn(N, 32, 9, 9, device="cuda", requires_grad=True)
    g = torch.randn(N, 16, 18, 18, device="cuda")
    y = deconv_relu(dc, x); (y * g).sum().backward()
    fx, fw, fb = x.grad.clone(), dc.weight.grad.clone(), dc.bias.grad.clone()
    x.grad = None; dc.weight.grad = None; dc.bias.grad = None
    yt = torch.relu(dc(x)); (yt * g).sum().backward()
    tx, tw, tb = x.grad.clone(), dc.weight.grad.clone(), dc.bias.grad.clone()
    x64 = x.detach().cpu().double().requires_grad_()
    dc64 = torch.nn.ConvTranspose2d(32, 16, kernel_size=4, stride=2, padding=1).double()
    with torch.no_grad():
        dc64.weight.copy_(dc.weight.double().cpu()); dc64.bias.copy_(dc.bias.double().cpu())
    y64 = torch.relu(dc64(x64)); (y64 * g.cpu().double()).sum().backward()
    print(N, "fused vs torch-gpu", rel(fx, tx), rel(fw, tw), rel(fb, tb), "| torch-gpu vs fp64", rel(tx, x64.grad),
          rel(tw, dc64.weight.grad), rel(tb, dc64.bias.grad), "| fused vs fp64", rel(fx, x64.grad), rel(fw, dc64.weight.grad), rel(fb, dc64.bias.grad))
