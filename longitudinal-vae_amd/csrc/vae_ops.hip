// vae_ops.hip -- fused pieces of the ConvVAE encoder (VAE.py:44-60): pool(relu(conv(x))) with a
// 2x2 / stride-2 max pool.  relu and a max commute, so the pair is one pass over the conv output:
// y = max(0, max of the window), with the argmax position kept as one byte (0..3, scan order,
// first strict maximum -- the element torch's max_pool2d routes the gradient to).  Backward writes
// every input element once: g_y to the argmax element when y > 0 (relu'(y) = 0 otherwise), 0 to
// the rest.  Replaces torch's relu + max_pool2d (+ int64 indices) + their two backward kernels.
//
// The _bias forms also take the conv's per-channel bias (the conv itself then runs without one):
// the window is max of fl(x + b) (first strict maximum, so ties and rounding match torch's
// conv-with-bias -> relu -> pool exactly), and the backward also returns db_c = sum of the routed
// gradient over channel c -- the conv's bias gradient, which torch otherwise takes as a separate
// sum over the full-resolution [N, C, H, W] gradient (strided, ~0.5 ms at the headline batch).
// The bias sum is deterministic: per-(image chunk, channel) partials, then one fixed-order tree.
#include "common.hpp"

namespace lvae {

typedef float vo_f32x2 __attribute__((ext_vector_type(2)));

// one thread per output element; planes = N * C, H, W even
__global__ __launch_bounds__(256) void relu_maxpool2_fwd_kernel(const float* __restrict__ x, int64_t total, int Ho,
                                                                int Wo, float* __restrict__ y,
                                                                uint8_t* __restrict__ idx) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= total) return;
  const int64_t plane = e / ((int64_t)Ho * Wo);
  const int r = (int)(e % ((int64_t)Ho * Wo)), i = r / Wo, j = r % Wo;
  const int W = 2 * Wo;
  const float* p = x + plane * 4 * Ho * Wo + (int64_t)(2 * i) * W + 2 * j;
  const vo_f32x2 a = *reinterpret_cast<const vo_f32x2*>(p);
  const vo_f32x2 b = *reinterpret_cast<const vo_f32x2*>(p + W);
  float m = a[0];
  uint8_t k = 0;
  if (a[1] > m) m = a[1], k = 1;
  if (b[0] > m) m = b[0], k = 2;
  if (b[1] > m) m = b[1], k = 3;
  y[e] = m > 0.f ? m : 0.f;
  idx[e] = k;
}

// one thread per output element, writes its 2x2 input window
__global__ __launch_bounds__(256) void relu_maxpool2_bwd_kernel(const float* __restrict__ gy,
                                                                const float* __restrict__ y,
                                                                const uint8_t* __restrict__ idx, int64_t total, int Ho,
                                                                int Wo, float* __restrict__ gx) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= total) return;
  const int64_t plane = e / ((int64_t)Ho * Wo);
  const int r = (int)(e % ((int64_t)Ho * Wo)), i = r / Wo, j = r % Wo;
  const int W = 2 * Wo;
  const float g = y[e] > 0.f ? gy[e] : 0.f;
  const int k = idx[e];
  float* p = gx + plane * 4 * Ho * Wo + (int64_t)(2 * i) * W + 2 * j;
  vo_f32x2 a, b;
  a[0] = k == 0 ? g : 0.f;
  a[1] = k == 1 ? g : 0.f;
  b[0] = k == 2 ? g : 0.f;
  b[1] = k == 3 ? g : 0.f;
  *reinterpret_cast<vo_f32x2*>(p) = a;
  *reinterpret_cast<vo_f32x2*>(p + W) = b;
}

// one thread per output element; plane = n * C + c
__global__ __launch_bounds__(256) void relu_maxpool2_bias_fwd_kernel(const float* __restrict__ x,
                                                                     const float* __restrict__ bias, int C,
                                                                     int64_t total, int Ho, int Wo,
                                                                     float* __restrict__ y,
                                                                     uint8_t* __restrict__ idx) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= total) return;
  const int64_t plane = e / ((int64_t)Ho * Wo);
  const int r = (int)(e % ((int64_t)Ho * Wo)), i = r / Wo, j = r % Wo;
  const int W = 2 * Wo;
  const float bc = bias[plane % C];
  const float* p = x + plane * 4 * Ho * Wo + (int64_t)(2 * i) * W + 2 * j;
  const vo_f32x2 a = *reinterpret_cast<const vo_f32x2*>(p);
  const vo_f32x2 b = *reinterpret_cast<const vo_f32x2*>(p + W);
  float m = a[0] + bc;
  uint8_t k = 0;
  if (a[1] + bc > m) m = a[1] + bc, k = 1;
  if (b[0] + bc > m) m = b[0] + bc, k = 2;
  if (b[1] + bc > m) m = b[1] + bc, k = 3;
  y[e] = m > 0.f ? m : 0.f;
  idx[e] = k;
}

// grid (nb, C): block (bx, c) routes the gradient of planes (n, c), n in [bx per, (bx+1) per), and
// writes its channel partial sum to part[c][bx]
__global__ __launch_bounds__(256) void relu_maxpool2_bias_bwd_kernel(const float* __restrict__ gy,
                                                                     const float* __restrict__ y,
                                                                     const uint8_t* __restrict__ idx, int N, int C,
                                                                     int Ho, int Wo, int per, float* __restrict__ gx,
                                                                     float* __restrict__ part) {
  __shared__ float red[256];
  const int c = blockIdx.y, n0 = blockIdx.x * per, n1 = min(N, n0 + per);
  const int P = Ho * Wo, W = 2 * Wo;
  const int total = (n1 - n0) * P;
  float s = 0.f;
  for (int t = threadIdx.x; t < total; t += 256) {
    const int n = n0 + t / P, r = t % P, i = r / Wo, j = r % Wo;
    const int64_t plane = (int64_t)n * C + c, e = plane * P + r;
    const float g = y[e] > 0.f ? gy[e] : 0.f;
    s += g;
    const int k = idx[e];
    float* q = gx + plane * 4 * P + (int64_t)(2 * i) * W + 2 * j;
    vo_f32x2 a, b;
    a[0] = k == 0 ? g : 0.f;
    a[1] = k == 1 ? g : 0.f;
    b[0] = k == 2 ? g : 0.f;
    b[1] = k == 3 ? g : 0.f;
    *reinterpret_cast<vo_f32x2*>(q) = a;
    *reinterpret_cast<vo_f32x2*>(q + W) = b;
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[(int64_t)c * gridDim.x + blockIdx.x] = red[0];
}

// db[c] = sum_b part[c][b], fixed order (one block per channel)
__global__ __launch_bounds__(256) void bias_partial_sum_kernel(const float* __restrict__ part, int nb,
                                                               float* __restrict__ db) {
  __shared__ float red[256];
  const int c = blockIdx.x;
  float s = 0.f;
  for (int b = threadIdx.x; b < nb; b += 256) s += part[(int64_t)c * nb + b];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) db[c] = red[0];
}

constexpr int kPoolBiasPer = 16;  // images per backward block (x C channels in the grid)

// The first encoder conv (1 input channel, 3 x 3, padding 1) needs no input gradient, so its whole
// backward reduces to dW[c][ky][kx] = sum g * x[r + ky - 1][s + kx - 1] and db[c] = sum g over the
// pooled outputs, (r, s) = the argmax position of each window (the only nonzero of the routed
// gradient): the full-resolution gradient is never written and no conv kernel runs.  Grid (nb, C);
// partials part[c][bx][10] (9 taps + bias), reduced in a fixed order by conv1_wgrad_sum_kernel.
__global__ __launch_bounds__(256) void relu_maxpool2_conv1_wgrad_kernel(const float* __restrict__ gy,
                                                                        const float* __restrict__ y,
                                                                        const uint8_t* __restrict__ idx,
                                                                        const float* __restrict__ x, int N, int C,
                                                                        int Ho, int Wo, int per,
                                                                        float* __restrict__ part) {
  __shared__ float red[10][256];
  const int c = blockIdx.y, n0 = blockIdx.x * per, n1 = min(N, n0 + per);
  const int P = Ho * Wo, H = 2 * Ho, W = 2 * Wo;
  const int total = (n1 - n0) * P;
  float acc[10];
#pragma unroll
  for (int q = 0; q < 10; ++q) acc[q] = 0.f;
  for (int t = threadIdx.x; t < total; t += 256) {
    const int n = n0 + t / P, r = t % P, i = r / Wo, j = r % Wo;
    const int64_t e = ((int64_t)n * C + c) * P + r;
    const float g = y[e] > 0.f ? gy[e] : 0.f;
    acc[9] += g;
    const int k = idx[e], rr = 2 * i + (k >> 1), ss = 2 * j + (k & 1);
    const float* xp = x + (int64_t)n * H * W;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int yy = rr + ky - 1, xx = ss + kx - 1;
        const float v = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? xp[yy * W + xx] : 0.f;
        acc[3 * ky + kx] += g * v;
      }
  }
#pragma unroll
  for (int q = 0; q < 10; ++q) red[q][threadIdx.x] = acc[q];
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o)
#pragma unroll
      for (int q = 0; q < 10; ++q) red[q][threadIdx.x] += red[q][threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x < 10) part[((int64_t)c * gridDim.x + blockIdx.x) * 10 + threadIdx.x] = red[threadIdx.x][0];
}

// dw[c][q] = sum_b part[c][b][q] (q < 9), db[c] = sum_b part[c][b][9]; one block per channel
__global__ __launch_bounds__(256) void conv1_wgrad_sum_kernel(const float* __restrict__ part, int nb,
                                                              float* __restrict__ dw, float* __restrict__ db) {
  __shared__ float red[10][256];
  const int c = blockIdx.x;
  float s[10];
#pragma unroll
  for (int q = 0; q < 10; ++q) s[q] = 0.f;
  for (int b = threadIdx.x; b < nb; b += 256)
#pragma unroll
    for (int q = 0; q < 10; ++q) s[q] += part[((int64_t)c * nb + b) * 10 + q];
#pragma unroll
  for (int q = 0; q < 10; ++q) red[q][threadIdx.x] = s[q];
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o)
#pragma unroll
      for (int q = 0; q < 10; ++q) red[q][threadIdx.x] += red[q][threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x < 9) dw[c * 9 + threadIdx.x] = red[threadIdx.x][0];
  if (threadIdx.x == 9) db[c] = red[9][0];
}

}  // namespace lvae

using namespace lvae;

extern "C" {

int lvae_relu_maxpool2_fwd_f32(const float* x, int64_t planes, int H, int W, float* y, uint8_t* idx, void* stream) {
  if (!x || !y || !idx) return -1;
  if (planes < 0 || H < 2 || W < 2 || (H & 1) || (W & 1)) return -2;
  const int Ho = H / 2, Wo = W / 2;
  const int64_t total = planes * Ho * Wo;
  if (total == 0) return 0;
  relu_maxpool2_fwd_kernel<<<cdiv(total, 256), 256, 0, (hipStream_t)stream>>>(x, total, Ho, Wo, y, idx);
  LVAE_CHECK_LAUNCH();
  return 0;
}

int lvae_relu_maxpool2_bwd_f32(const float* gy, const float* y, const uint8_t* idx, int64_t planes, int H, int W,
                               float* gx, void* stream) {
  if (!gy || !y || !idx || !gx) return -1;
  if (planes < 0 || H < 2 || W < 2 || (H & 1) || (W & 1)) return -2;
  const int Ho = H / 2, Wo = W / 2;
  const int64_t total = planes * Ho * Wo;
  if (total == 0) return 0;
  relu_maxpool2_bwd_kernel<<<cdiv(total, 256), 256, 0, (hipStream_t)stream>>>(gy, y, idx, total, Ho, Wo, gx);
  LVAE_CHECK_LAUNCH();
  return 0;
}

size_t lvae_relu_maxpool2_bias_workspace_size(int N, int C) {
  return N <= 0 || C <= 0 ? 0 : sizeof(float) * (size_t)C * (size_t)cdiv(N, kPoolBiasPer);
}

int lvae_relu_maxpool2_bias_fwd_f32(const float* x, const float* bias, int N, int C, int H, int W, float* y,
                                    uint8_t* idx, void* stream) {
  if (!x || !bias || !y || !idx) return -1;
  if (N < 0 || C <= 0 || H < 2 || W < 2 || (H & 1) || (W & 1)) return -2;
  const int Ho = H / 2, Wo = W / 2;
  const int64_t total = (int64_t)N * C * Ho * Wo;
  if (total == 0) return 0;
  relu_maxpool2_bias_fwd_kernel<<<cdiv(total, 256), 256, 0, (hipStream_t)stream>>>(x, bias, C, total, Ho, Wo, y,
                                                                                    idx);
  LVAE_CHECK_LAUNCH();
  return 0;
}

size_t lvae_conv1_relu_maxpool2_wgrad_workspace_size(int N, int C) {
  return N <= 0 || C <= 0 ? 0 : sizeof(float) * 10 * (size_t)C * (size_t)cdiv(N, kPoolBiasPer);
}

int lvae_conv1_relu_maxpool2_wgrad_f32(const float* gy, const float* y, const uint8_t* idx, const float* x, int N,
                                       int C, int H, int W, float* dw, float* db, void* workspace, void* stream) {
  if (!gy || !y || !idx || !x || !dw || !db || !workspace) return -1;
  if (N < 0 || C <= 0 || H < 2 || W < 2 || (H & 1) || (W & 1)) return -2;
  hipStream_t st = (hipStream_t)stream;
  if (N == 0) {
    (void)hipMemsetAsync(dw, 0, sizeof(float) * 9 * C, st);
    (void)hipMemsetAsync(db, 0, sizeof(float) * C, st);
    return 0;
  }
  const int nb = (int)cdiv(N, kPoolBiasPer);
  float* part = (float*)workspace;
  relu_maxpool2_conv1_wgrad_kernel<<<dim3(nb, C), 256, 0, st>>>(gy, y, idx, x, N, C, H / 2, W / 2, kPoolBiasPer,
                                                                 part);
  conv1_wgrad_sum_kernel<<<C, 256, 0, st>>>(part, nb, dw, db);
  LVAE_CHECK_LAUNCH();
  return 0;
}

int lvae_relu_maxpool2_bias_bwd_f32(const float* gy, const float* y, const uint8_t* idx, int N, int C, int H, int W,
                                    float* gx, float* db, void* workspace, void* stream) {
  if (!gy || !y || !idx || !gx || !db || !workspace) return -1;
  if (N < 0 || C <= 0 || H < 2 || W < 2 || (H & 1) || (W & 1)) return -2;
  const int Ho = H / 2, Wo = W / 2;
  hipStream_t st = (hipStream_t)stream;
  if (N == 0) {
    (void)hipMemsetAsync(db, 0, sizeof(float) * C, st);
    return 0;
  }
  const int nb = (int)cdiv(N, kPoolBiasPer);
  float* part = (float*)workspace;
  relu_maxpool2_bias_bwd_kernel<<<dim3(nb, C), 256, 0, st>>>(gy, y, idx, N, C, Ho, Wo, kPoolBiasPer, gx, part);
  bias_partial_sum_kernel<<<C, 256, 0, st>>>(part, nb, db);
  LVAE_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
