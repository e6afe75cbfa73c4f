"""Conv encoder / decoder of the L-VAE (VAE.py:16-162), on PyTorch-ROCm (MIOpen / hipBLASLt).

Same layer names and shapes as the reference's ConvVAE so its state dicts load unchanged.  The
reference runs it in fp64 (LVAE.py:139-140, 152); here it runs in the dtype of its parameters
(fp32 by default: mu / logvar drift ~1e-7 relative vs fp64).
"""
import math
import os

import torch
import torch.nn.functional as F
from torch import nn


# LVAE_CONV_DGRAD=0: the second encoder conv's input gradient on MIOpen (routed gradient + backward-data conv)
# instead of lvae_conv3x3_pool_dgrad_f32 (A/B runs)
_CONV_DGRAD = os.environ.get("LVAE_CONV_DGRAD", "1") != "0"
# LVAE_CONV_BWD_FORK=0: that layer's weight-gradient and input-gradient kernels one after the other on the
# backward's stream instead of side by side (the weight gradient on a side stream, joined before returning)
_CONV_BWD_FORK = os.environ.get("LVAE_CONV_BWD_FORK", "1") != "0"
_FORK_UNDER_CAPTURE = os.environ.get("LVAE_FORK_UNDER_CAPTURE", "0") == "1"
# LVAE_CONV_FUSED=0: the second encoder conv's forward and the first decoder transposed conv (forward and backward)
# on MIOpen (+ the fused bias / relu / pool passes) instead of the direct HIP kernels (vae_ops.hip)
_CONV2_FUSED = os.environ.get("LVAE_CONV_FUSED", "1") != "0"
_SIDE_STREAMS = {}


def _side_stream(dev):
    s = _SIDE_STREAMS.get(dev)
    if s is None:
        s = _SIDE_STREAMS[dev] = torch.cuda.Stream(device=dev)
    return s


class _ReluMaxPool2(torch.autograd.Function):
    """max_pool2d(relu(x), 2, 2) in one HIP pass (lvae_relu_maxpool2_fwd/bwd_f32, vae_ops.hip):
    one byte of argmax per output instead of torch's int64 indices, one write per input in the
    backward.  Same values and gradient routing as relu + max_pool2d (first strict maximum)."""

    @staticmethod
    def forward(ctx, x):
        from . import _lib
        lib = _lib.lib()
        x = x.contiguous()
        N, C, H, W = x.shape
        y = torch.empty(N, C, H // 2, W // 2, dtype=x.dtype, device=x.device)
        idx = torch.empty(N, C, H // 2, W // 2, dtype=torch.uint8, device=x.device)
        _lib.check(lib.lvae_relu_maxpool2_fwd_f32(_lib.ptr(x), N * C, H, W, _lib.ptr(y), _lib.ptr(idx),
                                                   _lib.stream_ptr()), "relu_maxpool2_fwd")
        ctx.save_for_backward(y, idx)
        ctx.shape = (N, C, H, W)
        return y

    @staticmethod
    def backward(ctx, gy):
        from . import _lib
        lib = _lib.lib()
        y, idx = ctx.saved_tensors
        N, C, H, W = ctx.shape
        gy = gy.contiguous()
        gx = torch.empty(N, C, H, W, dtype=gy.dtype, device=gy.device)
        _lib.check(lib.lvae_relu_maxpool2_bwd_f32(_lib.ptr(gy), _lib.ptr(y), _lib.ptr(idx), N * C, H, W, _lib.ptr(gx),
                                                   _lib.stream_ptr()), "relu_maxpool2_bwd")
        return gx


class _ConvReluMaxPool2(torch.autograd.Function):
    """max_pool2d(relu(conv2d(x, w, b, padding=1)), 2, 2) (VAE.py:44-50).
    Forward: a 1-channel input (the first conv) is one direct HIP pass (lvae_conv1_relu_maxpool2_fwd_f32);
    otherwise the conv runs without its bias on MIOpen and bias add, relu and pool are one HIP pass
    (lvae_relu_maxpool2_bias_fwd_f32).  Backward: weight and bias gradients straight from the pooled
    gradient (lvae_conv3x3_pool_wgrad_f32), and for 16 input channels the input gradient too
    (lvae_conv3x3_pool_dgrad_f32; the first conv needs none); otherwise the routed full-resolution
    gradient is formed for MIOpen's backward-data conv."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        from . import _lib
        lib = _lib.lib()
        b = bias.contiguous()
        if x.shape[1] == 1:  # first conv: one direct HIP pass, no full-resolution output
            xc, wc = x.contiguous(), weight.contiguous()
            N, C, H, W = x.shape[0], weight.shape[0], x.shape[2], x.shape[3]
            y = torch.empty(N, C, H // 2, W // 2, dtype=x.dtype, device=x.device)
            idx = torch.empty(N, C, H // 2, W // 2, dtype=torch.uint8, device=x.device)
            _lib.check(lib.lvae_conv1_relu_maxpool2_fwd_f32(_lib.ptr(xc), _lib.ptr(wc), _lib.ptr(b), N, C, H, W,
                                                             _lib.ptr(y), _lib.ptr(idx), _lib.stream_ptr()),
                       "conv1_relu_maxpool2_fwd")
        elif _CONV2_FUSED and x.shape[1] == 16 and x.shape[2] == x.shape[3] == 18 and weight.shape[0] % 16 == 0:
            # the second conv end to end: one direct HIP pass (no MIOpen conv, no layout transposes, no
            # full-resolution output)
            xc, wc = x.contiguous(), weight.contiguous()
            N, C, H, W = x.shape[0], weight.shape[0], x.shape[2], x.shape[3]
            y = torch.empty(N, C, H // 2, W // 2, dtype=x.dtype, device=x.device)
            idx = torch.empty(N, C, H // 2, W // 2, dtype=torch.uint8, device=x.device)
            _lib.check(lib.lvae_conv3x3_relu_maxpool2_fwd_f32(_lib.ptr(xc), _lib.ptr(wc), _lib.ptr(b), N, x.shape[1], C,
                                                               H, W, _lib.ptr(y), _lib.ptr(idx), _lib.stream_ptr()),
                       "conv3x3_relu_maxpool2_fwd")
        else:
            y0 = F.conv2d(x, weight, None, 1, 1).contiguous()
            N, C, H, W = y0.shape
            y = torch.empty(N, C, H // 2, W // 2, dtype=y0.dtype, device=y0.device)
            idx = torch.empty(N, C, H // 2, W // 2, dtype=torch.uint8, device=y0.device)
            _lib.check(lib.lvae_relu_maxpool2_bias_fwd_f32(_lib.ptr(y0), _lib.ptr(b), N, C, H, W, _lib.ptr(y),
                                                            _lib.ptr(idx), _lib.stream_ptr()), "relu_maxpool2_bias_fwd")
        ctx.save_for_backward(x, weight, y, idx)
        ctx.shape = (N, C, H, W)
        return y

    @staticmethod
    def backward(ctx, gy):
        from . import _lib
        lib = _lib.lib()
        x, weight, y, idx = ctx.saved_tensors
        N, C, H, W = ctx.shape
        gy = gy.contiguous()
        Cin = x.shape[1]
        if N >= 512 and C * Cin <= 1024 and 4 * (Cin * (((H + 2) * (W + 2)) | 1) + 2 * C * (H // 2) * (W // 2)) <= 65536:
            # (below a few hundred images the per-image kernel cannot fill the GPU: MIOpen path)
            # weight and bias gradients from the pooled gradient (lvae_conv3x3_pool_wgrad_f32); the first
            # conv (image input) needs no input gradient
            xc = x.contiguous()
            dgrad = (ctx.needs_input_grad[0] and _CONV_DGRAD and Cin == 16 and H * W <= 1024
                     and lib.lvae_conv3x3_pool_dgrad_lds(C, H, W) <= 65536)
            cur = torch.cuda.current_stream(gy.device)
            # (eager only: with this fork inside a HIP graph capture the process segfaults in torch.cuda.graph's
            # capture_end, i.e. in the runtime's hipStreamEndCapture / graph instantiation -- still after r6's
            # memset fix, so not the memset nodes (profiles/r6_fork_under_capture_segv.log,
            # LVAE_FORK_UNDER_CAPTURE=1); captured steps keep the one-stream order)
            side = (_side_stream(gy.device) if dgrad and _CONV_BWD_FORK and (
                _FORK_UNDER_CAPTURE or not torch.cuda.is_current_stream_capturing()) else None)
            if side is not None:  # (the weight gradient beside the input gradient; joined below)
                side.wait_stream(cur)
            with torch.cuda.stream(side if side is not None else cur):
                dw = torch.empty_like(weight)
                db = torch.empty(C, dtype=gy.dtype, device=gy.device)
                ws = torch.empty(lib.lvae_conv3x3_pool_wgrad_workspace_size(N, C, Cin) // 4 + 1, dtype=torch.float32,
                                 device=gy.device)
                _lib.check(lib.lvae_conv3x3_pool_wgrad_f32(_lib.ptr(gy), _lib.ptr(y), _lib.ptr(idx), _lib.ptr(xc), N, C,
                                                            Cin, H, W, _lib.ptr(dw), _lib.ptr(db), _lib.ptr(ws),
                                                            _lib.stream_ptr()), "conv3x3_pool_wgrad")
            gx = None
            if dgrad:
                # the input gradient straight from the pooled gradient too (lvae_conv3x3_pool_dgrad_f32: the
                # routed gradient formed per image in LDS; no MIOpen backward-data conv, no transposes)
                gx = torch.empty(N, Cin, H, W, dtype=gy.dtype, device=gy.device)
                _lib.check(lib.lvae_conv3x3_pool_dgrad_f32(_lib.ptr(gy), _lib.ptr(y), _lib.ptr(idx),
                                                            _lib.ptr(weight.contiguous()), N, C, Cin, H, W,
                                                            _lib.ptr(gx), _lib.stream_ptr()), "conv3x3_pool_dgrad")
                if side is not None:
                    cur.wait_stream(side)
                    dw.record_stream(cur)
                    db.record_stream(cur)
            elif ctx.needs_input_grad[0]:
                g0 = torch.empty(N, C, H, W, dtype=gy.dtype, device=gy.device)
                _lib.check(lib.lvae_relu_maxpool2_bwd_f32(_lib.ptr(gy), _lib.ptr(y), _lib.ptr(idx), N * C, H, W,
                                                           _lib.ptr(g0), _lib.stream_ptr()), "relu_maxpool2_bwd")
                gx = torch.ops.aten.convolution_backward(g0, x, weight, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                                         [True, False, False])[0]
            return gx, dw if ctx.needs_input_grad[1] else None, db if ctx.needs_input_grad[2] else None
        g0 = torch.empty(N, C, H, W, dtype=gy.dtype, device=gy.device)
        db = torch.empty(C, dtype=gy.dtype, device=gy.device)
        ws = torch.empty(lib.lvae_relu_maxpool2_bias_workspace_size(N, C) // 4 + 1, dtype=torch.float32,
                         device=gy.device)
        _lib.check(lib.lvae_relu_maxpool2_bias_bwd_f32(_lib.ptr(gy), _lib.ptr(y), _lib.ptr(idx), N, C, H, W,
                                                        _lib.ptr(g0), _lib.ptr(db), _lib.ptr(ws), _lib.stream_ptr()),
                   "relu_maxpool2_bias_bwd")
        gx = gw = None
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            gx, gw, _ = torch.ops.aten.convolution_backward(
                g0, x, weight, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                [ctx.needs_input_grad[0], ctx.needs_input_grad[1], False])
        return gx, gw, db if ctx.needs_input_grad[2] else None


def conv_relu_maxpool2(conv, x):
    """pool(relu(conv(x))) for the encoder's 3x3 / padding-1 convs: fused bias path for CUDA fp32."""
    if (x.is_cuda and x.dtype == torch.float32 and conv.bias is not None and conv.weight.dtype == torch.float32
            and tuple(conv.kernel_size) == (3, 3) and tuple(conv.padding) == (1, 1) and tuple(conv.stride) == (1, 1)
            and tuple(conv.dilation) == (1, 1) and conv.groups == 1 and x.shape[-1] % 2 == 0 and x.shape[-2] % 2 == 0):
        return _ConvReluMaxPool2.apply(x, conv.weight, conv.bias)
    return relu_maxpool2(conv(x))


class _Deconv2Sigmoid(torch.autograd.Function):
    """sigmoid(ConvTranspose2d(Cin, 1, 4, stride 2, padding 1)(z)) (VAE.py:75, 124) as one direct HIP pass
    each way (lvae_deconv2_sigmoid_fwd/bwd_f32): the backward forms the pre-sigmoid gradient on the fly
    and returns the input, weight and bias gradients together (no MIOpen transposed conv, no
    sigmoid / bias-sum kernels)."""

    @staticmethod
    def forward(ctx, z, weight, bias):
        from . import _lib
        lib = _lib.lib()
        zc, wc, bc = z.contiguous(), weight.contiguous(), bias.contiguous()
        N, Cin, Hi, Wi = zc.shape
        out = torch.empty(N, 1, 2 * Hi, 2 * Wi, dtype=z.dtype, device=z.device)
        _lib.check(lib.lvae_deconv2_sigmoid_fwd_f32(_lib.ptr(zc), _lib.ptr(wc), _lib.ptr(bc), N, Cin, Hi, Wi,
                                                     _lib.ptr(out), _lib.stream_ptr()), "deconv2_sigmoid_fwd")
        ctx.save_for_backward(zc, wc, out)
        return out

    @staticmethod
    def backward(ctx, g):
        from . import _lib
        lib = _lib.lib()
        z, w, out = ctx.saved_tensors
        N, Cin, Hi, Wi = z.shape
        g = g.contiguous()
        gz = torch.empty_like(z)
        dw = torch.empty_like(w)
        db = torch.empty(1, dtype=z.dtype, device=z.device)
        ws = torch.empty(lib.lvae_deconv2_sigmoid_workspace_size(N, Cin, Hi, Wi) // 4 + 1, dtype=torch.float32,
                         device=z.device)
        _lib.check(lib.lvae_deconv2_sigmoid_bwd_f32(_lib.ptr(g), _lib.ptr(out), _lib.ptr(z), _lib.ptr(w), N, Cin, Hi,
                                                     Wi, _lib.ptr(gz), _lib.ptr(dw), _lib.ptr(db), _lib.ptr(ws),
                                                     _lib.stream_ptr()), "deconv2_sigmoid_bwd")
        return gz, dw, db


def _deconv2_lds_ok(cin, hi, wi):
    """The LDS bounds lvae_deconv2_sigmoid_fwd / _bwd_f32 enforce (64 KB each; rc -3 beyond):
    forward Cin ((Hi+2)(Wi+2) | 1) floats, backward (2Hi+2)(2Wi+2) + Cin Hi Wi floats."""
    return (4 * cin * (((hi + 2) * (wi + 2)) | 1) <= 65536
            and 4 * ((2 * hi + 2) * (2 * wi + 2) + cin * hi * wi) <= 65536)


def deconv_sigmoid(deconv, z):
    """sigmoid(deconv(z)) for the decoder's last layer: fused HIP path for CUDA fp32 (torch's
    transposed conv + sigmoid when the geometry or the kernel's LDS bound rules it out)."""
    if (z.is_cuda and z.dtype == torch.float32 and deconv.weight.dtype == torch.float32 and deconv.bias is not None
            and z.dim() == 4 and _deconv2_lds_ok(z.shape[1], z.shape[2], z.shape[3])
            and deconv.out_channels == 1 and deconv.in_channels <= 16 and tuple(deconv.kernel_size) == (4, 4)
            and tuple(deconv.stride) == (2, 2) and tuple(deconv.padding) == (1, 1)
            and tuple(deconv.output_padding) == (0, 0) and tuple(deconv.dilation) == (1, 1) and deconv.groups == 1):
        return _Deconv2Sigmoid.apply(z, deconv.weight, deconv.bias)
    return torch.sigmoid(deconv(z))


def _act_bwd(gy, y, relu, N, C, HW):
    """(g, db): g = gy [y > 0] (gy itself without relu) and the bias gradient, one HIP pass
    (lvae_act_bwd_f32, glue.hip)."""
    from . import _lib
    lib = _lib.lib()
    g = torch.empty_like(gy) if relu else gy
    db = torch.empty(C, dtype=gy.dtype, device=gy.device)
    ws = torch.empty(lib.lvae_act_bwd_workspace_size(N, C) // 4 + 1, dtype=torch.float32, device=gy.device)
    _lib.check(lib.lvae_act_bwd_f32(_lib.ptr(gy), _lib.ptr(y) if relu else None, N, C, HW, 1 if relu else 0,
                                    _lib.ptr(g) if relu else None, _lib.ptr(db), _lib.ptr(ws), _lib.stream_ptr()),
               "act_bwd")
    return g, db


class _LinearAct(torch.autograd.Function):
    """relu(x W^T + b) or x W^T + b: the ConvVAE's fc layers (VAE.py:44-75).  The GEMMs stay on hipBLASLt
    (torch.mm / addmm); bias + ReLU is one HIP pass forward (lvae_bias_relu_fwd_f32) and the backward's
    pre-activation gradient and bias gradient one more (lvae_act_bwd_f32), in place of PyTorch's relu,
    threshold_backward and the strided bias reduction."""

    @staticmethod
    def forward(ctx, x, weight, bias, relu):
        from . import _lib
        x2 = x.contiguous()
        B, F_ = x2.shape[0], weight.shape[0]
        if relu:
            y = torch.mm(x2, weight.t())
            _lib.check(_lib.lib().lvae_bias_relu_fwd_f32(_lib.ptr(y), _lib.ptr(bias.contiguous()), B, F_, 1,
                                                          _lib.stream_ptr()), "bias_relu_fwd")
        else:
            y = torch.addmm(bias, x2, weight.t())
        ctx.relu = relu
        ctx.save_for_backward(x2, weight, y if relu else None)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, y = ctx.saved_tensors
        gy = gy.contiguous()
        g, db = _act_bwd(gy, y, ctx.relu, gy.shape[0], gy.shape[1], 1)
        dx = torch.mm(g, w) if ctx.needs_input_grad[0] else None
        dw = torch.mm(g.t(), x)
        return dx, dw, db, None


def _deconv4s2_fused(x, weight, stride, padding, output_padding, dilation, groups):
    """The shapes lvae_deconv4s2_relu_fwd / _bwd_f32 take: the ConvVAE's deconv1 (32 -> 16, 4 x 4, stride 2,
    padding 1) on 9 x 9 inputs."""
    return (_CONV2_FUSED and x.dim() == 4 and tuple(x.shape[1:]) == (32, 9, 9) and tuple(weight.shape) == (32, 16, 4, 4)
            and tuple(stride) == (2, 2) and tuple(padding) == (1, 1) and tuple(output_padding) == (0, 0)
            and tuple(dilation) == (1, 1) and groups == 1)


class _DeconvRelu(torch.autograd.Function):
    """relu(ConvTranspose2d(x)) (VAE.py:73, 122).  The ConvVAE's shape (32 -> 16, 4 x 4, stride 2, padding 1, 9 x 9
    inputs): one direct HIP pass each way (lvae_deconv4s2_relu_fwd / _bwd_f32: the backward returns the input,
    weight and bias gradients together from the masked output gradient).  Other shapes: the transposed conv
    without its bias on MIOpen, then bias + ReLU in place as one HIP pass; backward: the pre-activation and bias
    gradients in one HIP pass, the input / weight gradients from MIOpen's convolution backward."""

    @staticmethod
    def forward(ctx, x, weight, bias, stride, padding, output_padding, dilation, groups):
        from . import _lib
        ctx.fused = _deconv4s2_fused(x, weight, stride, padding, output_padding, dilation, groups)
        if ctx.fused:
            xc, wc = x.contiguous(), weight.contiguous()
            N = x.shape[0]
            y = torch.empty(N, 16, 18, 18, dtype=x.dtype, device=x.device)
            _lib.check(_lib.lib().lvae_deconv4s2_relu_fwd_f32(_lib.ptr(xc), _lib.ptr(wc), _lib.ptr(bias.contiguous()), N,
                                                               32, 16, 9, 9, _lib.ptr(y), _lib.stream_ptr()),
                       "deconv4s2_relu_fwd")
            ctx.save_for_backward(xc, wc, y)
            return y
        y = F.conv_transpose2d(x, weight, None, stride, padding, output_padding, groups, dilation).contiguous()
        N, C = y.shape[0], y.shape[1]
        _lib.check(_lib.lib().lvae_bias_relu_fwd_f32(_lib.ptr(y), _lib.ptr(bias.contiguous()), N, C,
                                                      y.shape[2] * y.shape[3], _lib.stream_ptr()), "bias_relu_fwd")
        ctx.conf = (stride, padding, output_padding, dilation, groups)
        ctx.save_for_backward(x, weight, y)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, y = ctx.saved_tensors
        gy = gy.contiguous()
        if ctx.fused:
            from . import _lib
            lib = _lib.lib()
            N = x.shape[0]
            dx = torch.empty_like(x)
            dw = torch.empty_like(w)
            db = torch.empty(16, dtype=x.dtype, device=x.device)
            ws = torch.empty(lib.lvae_deconv4s2_relu_bwd_workspace_size(N, 32, 16) // 4 + 1, dtype=torch.float32,
                             device=x.device)
            _lib.check(lib.lvae_deconv4s2_relu_bwd_f32(_lib.ptr(gy), _lib.ptr(y), _lib.ptr(x), _lib.ptr(w), N, 32, 16,
                                                        9, 9, _lib.ptr(dx), _lib.ptr(dw), _lib.ptr(db), _lib.ptr(ws),
                                                        _lib.stream_ptr()), "deconv4s2_relu_bwd")
            return dx if ctx.needs_input_grad[0] else None, dw, db, None, None, None, None, None
        stride, padding, output_padding, dilation, groups = ctx.conf
        g, db = _act_bwd(gy, y, True, y.shape[0], y.shape[1], y.shape[2] * y.shape[3])
        dx, dw, _ = torch.ops.aten.convolution_backward(g, x, w, None, list(stride), list(padding), list(dilation),
                                                        True, list(output_padding), groups,
                                                        [ctx.needs_input_grad[0], True, False])
        return dx, dw, db, None, None, None, None, None


def _f32_cuda(*ts):
    return all(t.is_cuda and t.dtype == torch.float32 for t in ts)


def linear_act(fc, x, relu):
    """relu(fc(x)) / fc(x) for the fc layers: the fused bias / ReLU HIP passes for CUDA fp32 2-D inputs."""
    if fc.bias is not None and x.dim() == 2 and _f32_cuda(x, fc.weight, fc.bias):
        return _LinearAct.apply(x, fc.weight, fc.bias, relu)
    y = fc(x)
    return F.relu(y) if relu else y


def deconv_relu(deconv, x):
    """relu(deconv(x)) for the decoder's first transposed conv: bias + ReLU fused for CUDA fp32."""
    if deconv.bias is not None and x.dim() == 4 and _f32_cuda(x, deconv.weight, deconv.bias):
        return _DeconvRelu.apply(x, deconv.weight, deconv.bias, tuple(deconv.stride), tuple(deconv.padding),
                                 tuple(deconv.output_padding), tuple(deconv.dilation), deconv.groups)
    return F.relu(deconv(x))


def relu_maxpool2(x):
    """pool(relu(x)) of the encoder (VAE.py:44-50): fused HIP kernel for CUDA fp32 activations."""
    if x.is_cuda and x.dtype == torch.float32 and x.shape[-1] % 2 == 0 and x.shape[-2] % 2 == 0:
        return _ReluMaxPool2.apply(x)
    return F.max_pool2d(F.relu(x), kernel_size=2, stride=2)


class ConvVAE(nn.Module):
    def __init__(self, latent_dim, num_dim=1296, vy_init=1.0, vy_fixed=False, p_input=0.2, p=0.5):
        super().__init__()
        self.latent_dim = latent_dim
        self.num_dim = num_dim
        self.p_input = p_input
        self.p = p
        log_vy_init = math.log(vy_init - math.exp(-8.0))
        self._log_vy = nn.Parameter(torch.full((num_dim,), log_vy_init))
        if vy_fixed:
            self._log_vy.requires_grad_(False)
        # encoder (VAE.py:44-60)
        self.conv1 = nn.Conv2d(1, 16, kernel_size=3, stride=1, padding=1)
        self.pool1 = nn.MaxPool2d(kernel_size=2, stride=2, padding=0)
        self.dropout2d_1 = nn.Dropout2d(p=p)
        self.conv2 = nn.Conv2d(16, 32, kernel_size=3, stride=1, padding=1)
        self.pool2 = nn.MaxPool2d(kernel_size=2, stride=2, padding=0)
        self.dropout2d_2 = nn.Dropout2d(p=p)
        self.fc1 = nn.Linear(32 * 9 * 9, 300)
        self.dropout1 = nn.Dropout(p=p)
        self.fc21 = nn.Linear(300, 30)
        self.dropout2 = nn.Dropout(p=p)
        self.fc211 = nn.Linear(30, latent_dim)
        self.fc221 = nn.Linear(30, latent_dim)
        # decoder (VAE.py:62-75)
        self.fc3 = nn.Linear(latent_dim, 30)
        self.dropout3 = nn.Dropout(p=p)
        self.fc31 = nn.Linear(30, 300)
        self.dropout4 = nn.Dropout(p=p)
        self.fc4 = nn.Linear(300, 32 * 9 * 9)
        self.dropout2d_3 = nn.Dropout2d(p=p)
        self.deconv1 = nn.ConvTranspose2d(32, 16, kernel_size=4, stride=2, padding=1)
        self.dropout2d_4 = nn.Dropout2d(p=p)
        self.deconv2 = nn.ConvTranspose2d(16, 1, kernel_size=4, stride=2, padding=1)
        self.register_buffer("min_log_vy", torch.full((1,), -8.0))

    @property
    def vy(self):
        return torch.exp(self.min_log_vy + F.softplus(self._log_vy - self.min_log_vy))

    def encode(self, x):
        z = self.dropout2d_1(conv_relu_maxpool2(self.conv1, x))   # pool1(relu(conv1))
        z = self.dropout2d_2(conv_relu_maxpool2(self.conv2, z))   # pool2(relu(conv2))
        h1 = self.dropout1(linear_act(self.fc1, z.reshape(-1, 32 * 9 * 9), True))
        h2 = self.dropout2(linear_act(self.fc21, h1, True))
        return linear_act(self.fc211, h2, False), linear_act(self.fc221, h2, False)

    def decode(self, z):
        x = self.dropout3(linear_act(self.fc3, z, True))
        x = self.dropout4(linear_act(self.fc31, x, True))
        x = linear_act(self.fc4, x, True)
        x = self.dropout2d_3(x.reshape(-1, 32, 9, 9))
        x = self.dropout2d_4(deconv_relu(self.deconv1, x))
        return deconv_sigmoid(self.deconv2, x)

    def sample_latent(self, mu, log_var, eps=None):
        if eps is None:
            eps = torch.randn_like(log_var)
        if _glue_ok(mu, log_var, eps) and mu.shape == log_var.shape == eps.shape:
            return _ReparamFn.apply(mu, log_var, eps)  # (glue.hip: one launch each way)
        return mu + eps * torch.exp(0.5 * log_var)

    def forward(self, x, eps=None):
        mu, log_var = self.encode(x)
        return self.decode(self.sample_latent(mu, log_var, eps)), mu, log_var

    def loss_function(self, recon_x, x, mask):
        """(per-image masked MSE, per-image NLL) -- VAE.py:144-162."""
        d = self.num_dim
        if _glue_ok(recon_x, x, mask, self._log_vy) and self._log_vy.numel() == d:
            return _VaeLossFn.apply(recon_x, x, mask, self._log_vy)  # (glue.hip: one launch each way)
        se = (recon_x.reshape(-1, d) - x.reshape(-1, d)) ** 2 * mask.reshape(-1, d)
        msum = mask.reshape(-1, d).sum(1)
        msum = torch.where(msum == 0, torch.ones_like(msum), msum)
        mse = se.sum(1) / msum
        nll = se / (2 * torch.exp(self._log_vy)) + 0.5 * (math.log(2 * math.pi) + self._log_vy)
        return mse, nll.sum(1)


class _VaeLossFn(torch.autograd.Function):
    """(mse [B], nll [B]) of ConvVAE.loss_function in one HIP launch (glue.hip); backward: d recon and
    d log_vy in one launch + the column sum of the d log_vy partials."""

    @staticmethod
    def forward(ctx, recon, x, mask, log_vy):
        from . import _lib
        lib = _lib.lib()
        d = log_vy.numel()
        r, xx, mm = (t.reshape(-1, d).contiguous() for t in (recon, x, mask))
        lv = log_vy.contiguous()
        B = r.shape[0]
        mse, nll, msum = (torch.empty(B, dtype=torch.float32, device=r.device) for _ in range(3))
        _lib.check(lib.lvae_vae_loss_fwd_f32(_lib.ptr(r), _lib.ptr(xx), _lib.ptr(mm), _lib.ptr(lv), B, d, _lib.ptr(mse),
                                             _lib.ptr(nll), _lib.ptr(msum), _lib.stream_ptr()), "vae_loss_fwd")
        ctx.save_for_backward(r, xx, mm, lv, msum)
        ctx.rshape = recon.shape
        ctx.need_lv = log_vy.requires_grad
        return mse, nll

    @staticmethod
    def backward(ctx, g_mse, g_nll):
        from . import _lib
        lib = _lib.lib()
        r, xx, mm, lv, msum = ctx.saved_tensors
        B, d = r.shape
        g_mse, g_nll = (g.to(torch.float32).reshape(B) for g in (g_mse, g_nll))  # (stride 0 kept: broadcasts)
        dr = torch.empty_like(r)
        part = torch.empty(int(lib.lvae_vae_loss_bwd_partials(B)), d, dtype=torch.float32, device=r.device)
        _lib.check(lib.lvae_vae_loss_bwd_f32(_lib.ptr(r), _lib.ptr(xx), _lib.ptr(mm), _lib.ptr(lv), _lib.ptr(msum),
                                             _lib.ptr(g_mse), g_mse.stride(0), _lib.ptr(g_nll), g_nll.stride(0), B, d,
                                             _lib.ptr(dr), _lib.ptr(part), _lib.stream_ptr()), "vae_loss_bwd")
        dlv = part.sum(0) if ctx.need_lv else None
        return dr.reshape(ctx.rshape), None, None, dlv


class _ReparamFn(torch.autograd.Function):
    """z = mu + eps exp(log_var / 2) in one HIP launch (glue.hip); backward: d log_var in one launch."""

    @staticmethod
    def forward(ctx, mu, log_var, eps):
        from . import _lib
        lib = _lib.lib()
        mu_, lv_, e_ = (t.contiguous() for t in (mu, log_var, eps))
        z = torch.empty_like(mu_)
        _lib.check(lib.lvae_reparam_fwd_f32(_lib.ptr(mu_), _lib.ptr(lv_), _lib.ptr(e_), mu_.numel(), _lib.ptr(z),
                                            _lib.stream_ptr()), "reparam_fwd")
        ctx.save_for_backward(lv_, e_)
        return z

    @staticmethod
    def backward(ctx, gz):
        from . import _lib
        lib = _lib.lib()
        lv_, e_ = ctx.saved_tensors
        gz = gz.contiguous()
        glv = torch.empty_like(lv_)
        _lib.check(lib.lvae_reparam_bwd_f32(_lib.ptr(gz), _lib.ptr(lv_), _lib.ptr(e_), lv_.numel(), _lib.ptr(glv),
                                            _lib.stream_ptr()), "reparam_bwd")
        return gz, glv, None


def _glue_ok(*ts):
    return all(t.is_cuda and t.dtype == torch.float32 for t in ts)


class _EncoderPart(nn.Module):
    """ConvVAE.encode as a module owning only the encoder's parameters (for make_graphed_callables)."""

    def __init__(self, vae):
        super().__init__()
        for n in ("conv1", "conv2", "fc1", "fc21", "fc211", "fc221"):
            setattr(self, n, getattr(vae, n))
        self._vae = [vae]

    def forward(self, x):
        return self._vae[0].encode(x)


class _DecoderLossPart(nn.Module):
    """decode + loss_function summed over images: (sum of per-image MSE, sum of per-image NLL)."""

    def __init__(self, vae):
        super().__init__()
        for n in ("fc3", "fc31", "fc4", "deconv1", "deconv2"):
            setattr(self, n, getattr(vae, n))
        self._log_vy = vae._log_vy
        self._vae = [vae]

    def forward(self, z, img, mask):
        v = self._vae[0]
        mse, nll = v.loss_function(v.decode(z), img, mask)
        return mse.sum(), nll.sum()


class GraphedConvVAE:
    """The ConvVAE's encoder and its decoder + recon loss, each replayed as a HIP graph forward and a HIP graph
    backward (torch.cuda.make_graphed_callables: torch.cuda.CUDAGraph is a hipGraph on ROCm), for the exact-KL
    step's ConvVAE stream.  Eager, the ConvVAE is ~100 small launches a step, which host overhead paces once
    the GPU work per launch is small (a rank's share of the images on several GPUs).  The graphs are built on
    first use for the batch's shapes (and rebuilt when they change); the arithmetic is the eager modules'."""

    def __init__(self, vae, warmup=3):
        self.vae = vae
        self.warmup = warmup
        self._key = None
        self.enc = self.dec = None

    def _build(self, img, mask):
        n = img.shape[0]
        L = self.vae.latent_dim
        x = img.detach().clone()
        z = torch.zeros(n, L, device=img.device, dtype=img.dtype, requires_grad=True)
        m = mask.detach().clone()
        self.enc, self.dec = torch.cuda.make_graphed_callables(
            (_EncoderPart(self.vae), _DecoderLossPart(self.vae)), ((x,), (z, x, m)), num_warmup_iters=self.warmup)
        self._key = (tuple(img.shape), tuple(mask.shape), img.dtype, img.device, self.vae.training)

    def _ensure(self, img, mask):
        if self._key != (tuple(img.shape), tuple(mask.shape), img.dtype, img.device, self.vae.training):
            self._build(img, mask)

    def encode(self, img, mask):
        self._ensure(img, mask)
        return self.enc(img)

    def decode_loss(self, z, img, mask):
        self._ensure(img, mask)
        return self.dec(z, img, mask)
