// vae_ops.hip -- fused pieces of the ConvVAE encoder (VAE.py:44-60): pool(relu(conv(x))) with a
// 2x2 / stride-2 max pool.  relu and a max commute, so the pair is one pass over the conv output:
// y = max(0, max of the window), with the argmax position kept as one byte (0..3, scan order,
// first strict maximum -- the element torch's max_pool2d routes the gradient to).  Backward writes
// every input element once: g_y to the argmax element when y > 0 (relu'(y) = 0 otherwise), 0 to
// the rest.  Replaces torch's relu + max_pool2d (+ int64 indices) + their two backward kernels.
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

}  // extern "C"
