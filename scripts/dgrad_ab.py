"""Dev A/B: the second encoder conv's input gradient at the headline shape (N = 4096 images, 32 <- 16
channels, 18 x 18): lvae_conv3x3_pool_dgrad_f32 vs the routed gradient + MIOpen backward-data conv."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "longitudinal-vae_amd"))
from lvae_amd import _lib  # noqa: E402

lib = _lib.lib()
dev = "cuda"
N, C, Cin, H = int(os.environ.get("N", 4096)), 32, 16, 18
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(N, Cin, H, H, device=dev, generator=g)
w = torch.randn(C, Cin, 3, 3, device=dev, generator=g)
gy = torch.randn(N, C, H // 2, H // 2, device=dev, generator=g)
y = torch.randn(N, C, H // 2, H // 2, device=dev, generator=g).clamp_min(0)
idx = torch.randint(0, 4, y.shape, device=dev, generator=g, dtype=torch.int32).to(torch.uint8)
gx = torch.empty(N, Cin, H, H, device=dev)
g0 = torch.empty(N, C, H, H, device=dev)


def hip():
    _lib.check(lib.lvae_conv3x3_pool_dgrad_f32(_lib.ptr(gy), _lib.ptr(y), _lib.ptr(idx), _lib.ptr(w), N, C, Cin, H, H,
                                                _lib.ptr(gx), _lib.stream_ptr()), "dgrad")
    return gx


def miopen():
    _lib.check(lib.lvae_relu_maxpool2_bwd_f32(_lib.ptr(gy), _lib.ptr(y), _lib.ptr(idx), N * C, H, H, _lib.ptr(g0),
                                               _lib.stream_ptr()), "route")
    return torch.ops.aten.convolution_backward(g0, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                               [True, False, False])[0]


a, b = hip(), miopen()
torch.cuda.synchronize()
print("max rel diff", float((a - b).abs().max() / b.abs().max()))
for name, f in (("hip", hip), ("miopen", miopen), ("hip", hip), ("miopen", miopen)):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(50):
        f()
    torch.cuda.synchronize()
    print(f"{name}: {(time.perf_counter() - t) / 50 * 1e6:.1f} us")
