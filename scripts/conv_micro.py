"""Time the fused ConvVAE conv kernels alone (vae_ops.hip) at the headline batch: the second encoder conv's forward,
the first decoder transposed conv forward and backward (diagnostic; not part of the product path)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "longitudinal-vae_amd"))
import torch  # noqa: E402
from lvae_amd import _lib  # noqa: E402

N = int(os.environ.get("N", 4096))
REPS = int(os.environ.get("REPS", 50))
lib = _lib.lib()
dev = torch.device("cuda")
st = _lib.stream_ptr


def timed(fn):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(REPS):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / REPS * 1e3


x2 = torch.rand(N, 16, 18, 18, device=dev)
w2 = torch.randn(32, 16, 3, 3, device=dev) * 0.1
b2 = torch.randn(32, device=dev) * 0.1
y2 = torch.empty(N, 32, 9, 9, device=dev)
i2 = torch.empty(N, 32, 9, 9, dtype=torch.uint8, device=dev)
P = _lib.ptr
t = timed(lambda: lib.lvae_conv3x3_relu_maxpool2_fwd_f32(P(x2), P(w2), P(b2), N, 16, 32, 18, 18, P(y2), P(i2), st()))
mac = N * 32 * 324 * 144
print(f"conv2 fwd  {t:7.1f} us  {2 * mac / t / 1e6:6.1f} TFLOP/s")
xd = torch.randn(N, 32, 9, 9, device=dev)
wd = torch.randn(32, 16, 4, 4, device=dev) * 0.1
bd = torch.randn(16, device=dev) * 0.1
yd = torch.empty(N, 16, 18, 18, device=dev)
t = timed(lambda: lib.lvae_deconv4s2_relu_fwd_f32(P(xd), P(wd), P(bd), N, 32, 16, 9, 9, P(yd), st()))
mac = N * 16 * 324 * 128
print(f"deconv fwd {t:7.1f} us  {2 * mac / t / 1e6:6.1f} TFLOP/s")
gy = torch.randn(N, 16, 18, 18, device=dev)
dx = torch.empty_like(xd)
dw = torch.empty_like(wd)
db = torch.empty_like(bd)
ws = torch.empty(lib.lvae_deconv4s2_relu_bwd_workspace_size(N, 32, 16) // 4 + 1, device=dev)
t = timed(lambda: lib.lvae_deconv4s2_relu_bwd_f32(P(gy), P(yd), P(xd), P(wd), N, 32, 16, 9, 9, P(dx), P(dw), P(db),
                                                  P(ws), st()))
mac = 2 * N * 16 * 324 * 128
print(f"deconv bwd {t:7.1f} us  {2 * mac / t / 1e6:6.1f} TFLOP/s (dx + dW)")
# the second encoder conv's backward: weight / bias gradients and input gradient from the pooled gradient
gp = torch.randn(N, 32, 9, 9, device=dev)
ip = torch.randint(0, 4, (N, 32, 9, 9), device=dev, dtype=torch.int32).to(torch.uint8)
yp = torch.randn(N, 32, 9, 9, device=dev).clamp_min(0.0)
dw2 = torch.empty_like(w2)
db2 = torch.empty_like(b2)
ws2 = torch.empty(lib.lvae_conv3x3_pool_wgrad_workspace_size(N, 32, 16) // 4 + 1, device=dev)
t = timed(lambda: lib.lvae_conv3x3_pool_wgrad_f32(P(gp), P(yp), P(ip), P(x2), N, 32, 16, 18, 18, P(dw2), P(db2), P(ws2),
                                                  st()))
print(f"conv2 wgrad {t:7.1f} us  {2 * N * 32 * 324 * 144 / t / 1e6:6.1f} TFLOP/s (dense-equivalent)")
gx2 = torch.empty_like(x2)
t = timed(lambda: lib.lvae_conv3x3_pool_dgrad_f32(P(gp), P(yp), P(ip), P(w2), N, 32, 16, 18, 18, P(gx2), st()))
print(f"conv2 dgrad {t:7.1f} us  {2 * N * 32 * 324 * 144 / t / 1e6:6.1f} TFLOP/s (dense-equivalent)")
# the first encoder conv's weight / bias gradients (1 input channel, 16 channels, 36 x 36)
x1 = torch.rand(N, 1, 36, 36, device=dev)
g1 = torch.randn(N, 16, 18, 18, device=dev)
i1 = torch.randint(0, 4, (N, 16, 18, 18), device=dev, dtype=torch.int32).to(torch.uint8)
y1 = torch.randn(N, 16, 18, 18, device=dev).clamp_min(0.0)
dw1 = torch.empty(16, 1, 3, 3, device=dev)
db1 = torch.empty(16, device=dev)
ws1 = torch.empty(lib.lvae_conv3x3_pool_wgrad_workspace_size(N, 16, 1) // 4 + 1, device=dev)
t = timed(lambda: lib.lvae_conv3x3_pool_wgrad_f32(P(g1), P(y1), P(i1), P(x1), N, 16, 1, 36, 36, P(dw1), P(db1), P(ws1),
                                                  st()))
print(f"conv1 wgrad {t:7.1f} us  {2 * N * 16 * 1296 * 9 / t / 1e6:6.1f} TFLOP/s (dense-equivalent)")
