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

#include <algorithm>
#include <cstdlib>

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

// ---- the decoder's last layer (VAE.py:75, 124): recon = sigmoid(ConvTranspose2d(Cin, 1, 4, stride 2,
// padding 1)(z) + b), z [N, Cin, Hi, Wi] -> [N, 1, 2 Hi, 2 Wi].  Output (oy, ox) takes input rows
// iy = (oy + 1 - ky) / 2 for the two ky of parity (oy + 1) & 1 (same for columns): 4 taps per input
// channel.  MIOpen's transposed conv for this shape took ~230 us forward and ~250 us backward.
__device__ inline float dc_sigmoid(float v) { return 1.0f / (1.0f + __expf(-v)); }

// One block per `per` images: the image's Cin planes staged in LDS; thread q owns input position
// q (and q + 256 ...) and writes its 2 x 2 output block (2 iy + a, 2 ix + b): rows iy - 1 .. iy + 1
// and columns ix - 1 .. ix + 1 of every plane feed those four outputs (4 taps each per channel).
__global__ __launch_bounds__(256) void deconv2_sigmoid_fwd_kernel(const float* __restrict__ z,
                                                                  const float* __restrict__ w,
                                                                  const float* __restrict__ bias, int N, int Cin,
                                                                  int Hi, int Wi, int per, float* __restrict__ out) {
  extern __shared__ float zl[];  // [Cin][Hi + 2][Wi + 2], zero border
  const int Hp = Hi + 2, Wp = Wi + 2, HWp = (Hp * Wp) | 1, Pi = Hi * Wi, Wo = 2 * Wi;
  const int t = threadIdx.x, n0 = blockIdx.x * per, n1 = min(N, n0 + per);
  for (int e = t; e < Cin * HWp; e += 256) zl[e] = 0.f;
  const float b0 = bias[0];
  for (int n = n0; n < n1; ++n) {
    __syncthreads();
    const float* zn = z + (int64_t)n * Cin * Pi;
    for (int e = t; e < Cin * Pi; e += 256) {
      const int ci = e / Pi, r = e % Pi;
      zl[ci * HWp + (r / Wi + 1) * Wp + r % Wi + 1] = zn[e];
    }
    __syncthreads();
    for (int q = t; q < Pi; q += 256) {
      const int iy = q / Wi, ix = q % Wi;
      float o[2][2] = {{0.f, 0.f}, {0.f, 0.f}};
      for (int ci = 0; ci < Cin; ++ci) {
        const float* zc = zl + ci * HWp + iy * Wp + ix;  // padded (iy - 1, ix - 1)
        const float* wc = w + 16 * ci;
        float v[3][3];
#pragma unroll
        for (int u = 0; u < 3; ++u)
#pragma unroll
          for (int c = 0; c < 3; ++c) v[u][c] = zc[u * Wp + c];
        // output row 2 iy + a: a = 0 -> (ky 1, row iy), (ky 3, row iy - 1); a = 1 -> (ky 0, row iy + 1),
        // (ky 2, row iy); columns likewise
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int bb = 0; bb < 2; ++bb) {
            float s = o[a][bb];
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
              for (int c = 0; c < 2; ++c) {
                const int ky = a == 0 ? 1 + 2 * u : 2 * u, kx = bb == 0 ? 1 + 2 * c : 2 * c;
                const int ry = a == 0 ? 1 - u : 2 - u, rx = bb == 0 ? 1 - c : 2 - c;  // padded row / col
                s = fmaf(v[ry][rx], wc[ky * 4 + kx], s);
              }
            o[a][bb] = s;
          }
      }
      float* on = out + (int64_t)n * 4 * Pi + (int64_t)(2 * iy) * Wo + 2 * ix;
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        vo_f32x2 r2;
        r2[0] = dc_sigmoid(o[a][0] + b0);
        r2[1] = dc_sigmoid(o[a][1] + b0);
        *reinterpret_cast<vo_f32x2*>(on + a * Wo) = r2;
      }
    }
  }
}

// backward: gp = g s (1 - s) (the pre-sigmoid gradient) staged per image in LDS with a zero border,
// and the image's z planes: gz[ci][iy][ix] = sum_{ky, kx} w[ci][ky][kx] gp(2 iy - 1 + ky, 2 ix - 1 + kx);
// thread (ci, tap) = (t >> 4, t & 15) accumulates dW[ci][tap] = sum z[ci][iy][ix] gp(...) over the
// block's images; db = sum gp.  Partials part[bx][Cin 16 + 1], summed by wgrad_sum_kernel.
__global__ __launch_bounds__(256) void deconv2_sigmoid_bwd_kernel(const float* __restrict__ g,
                                                                  const float* __restrict__ sout,
                                                                  const float* __restrict__ z,
                                                                  const float* __restrict__ w, int N, int Cin,
                                                                  int Hi, int Wi, int per, float* __restrict__ gz,
                                                                  float* __restrict__ part) {
  extern __shared__ float sm[];
  const int Ho = 2 * Hi, Wo = 2 * Wi, Gp = Wo + 2, Pi = Hi * Wi;
  float* gl = sm;                          // [Ho + 2][Wo + 2] (zero border)
  float* zl = gl + (Ho + 2) * Gp;          // [Cin][Pi]
  __shared__ float red[256];
  const int t = threadIdx.x, n0 = blockIdx.x * per, n1 = min(N, n0 + per);
  const int wci = t >> 4, tap = t & 15, ky = tap >> 2, kx = tap & 3;
  for (int e = t; e < (Ho + 2) * Gp; e += 256) gl[e] = 0.f;
  float dacc = 0.f, bacc = 0.f;
  for (int n = n0; n < n1; ++n) {
    __syncthreads();
    const float* gn = g + (int64_t)n * Ho * Wo;
    const float* sn = sout + (int64_t)n * Ho * Wo;
    for (int e = t; e < Ho * Wo; e += 256) {
      const float sv = sn[e], gp = gn[e] * (sv * (1.0f - sv));
      gl[(e / Wo + 1) * Gp + e % Wo + 1] = gp;
      bacc += gp;
    }
    const float* zn = z + (int64_t)n * Cin * Pi;
    for (int e = t; e < Cin * Pi; e += 256) zl[e] = zn[e];
    __syncthreads();
    float* gzn = gz + (int64_t)n * Cin * Pi;
    for (int q = t; q < Pi; q += 256) {  // the 4 x 4 gp patch once, then every channel
      const int iy = q / Wi, ix = q % Wi;
      const float* gp = gl + (2 * iy) * Gp + 2 * ix;  // padded (2 iy - 1, 2 ix - 1)
      float pt[16];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c) pt[4 * a + c] = gp[a * Gp + c];
      for (int ci = 0; ci < Cin; ++ci) {
        const float* wc = w + 16 * ci;
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < 16; ++k) s = fmaf(wc[k], pt[k], s);
        gzn[(int64_t)ci * Pi + q] = s;
      }
    }
    if (wci < Cin) {
      const float* zc = zl + wci * Pi;
      for (int iy = 0; iy < Hi; ++iy) {
        const float* zr = zc + iy * Wi;
        const float* gr = gl + (2 * iy + ky) * Gp + kx;
        for (int ix = 0; ix < Wi; ++ix) dacc = fmaf(zr[ix], gr[2 * ix], dacc);
      }
    }
  }
  float* pb = part + (int64_t)blockIdx.x * (Cin * 16 + 1);
  if (wci < Cin) pb[wci * 16 + tap] = dacc;
  red[t] = bacc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) red[t] += red[t + o];
    __syncthreads();
  }
  if (t == 0) pb[Cin * 16] = red[0];
}

// The first encoder conv end to end: 1 input channel, 3 x 3, padding 1, bias, relu, 2x2 pool, one
// thread per pooled position (n, i, j) for all C channels.  The 4 x 4 input patch under the window
// is loaded once; per channel the 2 x 2 conv outputs are sum_ky sum_kx p w (this order) + b, then
// relu + first-strict-max as in relu_maxpool2_bias_fwd_kernel.  The full-resolution conv output
// (16 x the image bytes) is never written; MIOpen's Winograd conv for this shape took ~270 us.
__global__ __launch_bounds__(256) void conv1_relu_maxpool2_fwd_kernel(const float* __restrict__ x,
                                                                      const float* __restrict__ w,
                                                                      const float* __restrict__ bias, int N, int C,
                                                                      int Ho, int Wo, float* __restrict__ y,
                                                                      uint8_t* __restrict__ idx) {
  const int P = Ho * Wo, H = 2 * Ho, W = 2 * Wo;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)N * P) return;
  const int n = (int)(e / P), r = (int)(e % P), i = r / Wo, j = r % Wo;
  const float* xn = x + (int64_t)n * H * W;
  float p[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int yy = 2 * i - 1 + a, xx = 2 * j - 1 + b;
      p[a][b] = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? xn[yy * W + xx] : 0.f;
    }
  for (int c = 0; c < C; ++c) {
    const float* wc = w + 9 * c;
    const float bc = bias[c];
    float v[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int dy = d >> 1, dx = d & 1;
      float s = 0.f;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) s = fmaf(p[dy + ky][dx + kx], wc[3 * ky + kx], s);
      v[d] = s + bc;
    }
    float m = v[0];
    uint8_t k = 0;
    if (v[1] > m) m = v[1], k = 1;
    if (v[2] > m) m = v[2], k = 2;
    if (v[3] > m) m = v[3], k = 3;
    const int64_t o = ((int64_t)n * C + c) * P + r;
    y[o] = m > 0.f ? m : 0.f;
    idx[o] = k;
  }
}
// images per block of the per-image LDS-staged kernels: 4 at large batches (fewer partials), 1 below
// 2048 images, where the grid would not fill the GPU
static inline int imgs_per_block(int N) { return N >= 2048 ? 4 : 1; }

// Weight and bias gradients of a 3 x 3 / stride-1 / padding-1 conv followed by the fused relu + 2x2
// pool, straight from the pooled gradient: the routed full-resolution gradient has one nonzero per
// window (at its argmax), so dW[co][ci][ky][kx] = sum g * x[ci][r + ky - 1][s + kx - 1] and
// db[co] = sum g over the pooled outputs (r, s = the argmax position).  No full-resolution gradient
// for the weights and no weight-gradient conv (MIOpen's needs two NCHW <-> NHWC transposes).
// One block per `per` images; per image the Cin input planes (zero border) and the routed gradient
// g and argmax offset of all C channels are staged in LDS, then thread t owns the (co, ci) pairs
// t % Q + 256 p... (Q = C Cin pairs; with Q < 256 the S = 256 / Q threads of a pair split its
// positions and are summed in LDS at the end).  Block partials part[bx][m], m = C Cin 9 + C,
// summed over blocks in a fixed order by wgrad_sum_kernel: deterministic.
template <int NP>
__global__ __launch_bounds__(256) void conv3x3_pool_wgrad_kernel(const float* __restrict__ gy,
                                                                 const float* __restrict__ y,
                                                                 const uint8_t* __restrict__ idx,
                                                                 const float* __restrict__ x, int N, int C, int Cin,
                                                                 int Ho, int Wo, int per, float* __restrict__ part) {
  extern __shared__ float sm[];
  // channel stride of the staged input: odd, so the 16+ ci lanes reading one offset hit distinct banks
  const int H = 2 * Ho, W = 2 * Wo, Hp = H + 2, Wp = W + 2, P = Ho * Wo, HWp = (Hp * Wp) | 1;
  const int Q = C * Cin, S = Q >= 256 ? 1 : 256 / Q;
  float* zl = sm;                                   // [Cin][HWp]
  float* gl = zl + Cin * HWp;                       // [C][P]
  int* ol = reinterpret_cast<int*>(gl + C * P);     // [C][P] padded offset of the argmax
  const int t = threadIdx.x, split = Q >= 256 ? 0 : t / Q;
  const bool active = Q >= 256 || t < Q * S;
  const int n0 = blockIdx.x * per, n1 = min(N, n0 + per);
  for (int e = t; e < Cin * HWp; e += 256) zl[e] = 0.f;
  float acc[NP][9], bacc[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    bacc[p] = 0.f;
#pragma unroll
    for (int q = 0; q < 9; ++q) acc[p][q] = 0.f;
  }
  for (int n = n0; n < n1; ++n) {
    __syncthreads();  // the previous image's reads are done (and the border is zero)
    const float* xn = x + (int64_t)n * Cin * H * W;
#pragma unroll 4
    for (int e = t; e < Cin * H * W; e += 256) {
      const int ci = e / (H * W), r = (e / W) % H, c = e % W;
      zl[ci * HWp + (r + 1) * Wp + c + 1] = xn[e];
    }
    const int64_t b0 = (int64_t)n * C * P;
#pragma unroll 4
    for (int e = t; e < C * P; e += 256) {  // unconditional loads: no load waits on another
      const float yv = y[b0 + e], gv = gy[b0 + e];
      const int k = idx[b0 + e], r = e % P, i = r / Wo, j = r % Wo;
      gl[e] = yv > 0.f ? gv : 0.f;
      ol[e] = (2 * i + (k >> 1)) * Wp + 2 * j + (k & 1);  // padded coords of tap (0, 0)
    }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int pr = (Q >= 256 ? t : t % Q) + 256 * p;
      if (active && pr < Q) {
        const int co = pr / Cin, ci = pr % Cin;
        const float* zc = zl + ci * HWp;
        for (int r = split; r < P; r += S) {
          const float g = gl[co * P + r];
          if (g == 0.f) continue;
          const float* z0 = zc + ol[co * P + r];
          bacc[p] += g;
#pragma unroll
          for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) acc[p][3 * ky + kx] += g * z0[ky * Wp + kx];
        }
      }
    }
  }
  // sum the S position splits of each pair in LDS (reusing the staging area), then write partials
  __syncthreads();
  const int m = Q * 9 + C;
  float* pb = part + (int64_t)blockIdx.x * m;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    if (S > 1) {
#pragma unroll
      for (int q = 0; q < 9; ++q) sm[q * 256 + t] = acc[p][q];
      sm[9 * 256 + t] = bacc[p];
      __syncthreads();
      if (t < Q) {
        for (int sp = 1; sp < S; ++sp) {
#pragma unroll
          for (int q = 0; q < 9; ++q) acc[p][q] += sm[q * 256 + sp * Q + t];
          bacc[p] += sm[9 * 256 + sp * Q + t];
        }
      }
      __syncthreads();
    }
    const int pr = t + 256 * p;
    if (t < Q && pr < Q) {
      const int co = pr / Cin, ci = pr % Cin;
#pragma unroll
      for (int q = 0; q < 9; ++q) pb[pr * 9 + q] = acc[p][q];
      if (ci == 0) pb[Q * 9 + co] = bacc[p];
    }
  }
}

// out[q] = sum_b part[b][q] (fixed order): 64 columns x 4 row slices per block, slices summed in LDS;
// q < nw -> dw[q], else db[q - nw]
__global__ __launch_bounds__(256) void wgrad_sum_kernel(const float* __restrict__ part, int nb, int m, int nw,
                                                        float* __restrict__ dw, float* __restrict__ db) {
  __shared__ float red[4][64];
  const int c = threadIdx.x & 63, sl = threadIdx.x >> 6, q = blockIdx.x * 64 + c;
  float s = 0.f;
  if (q < m) {
#pragma unroll 8
    for (int b = sl; b < nb; b += 4) s += part[(int64_t)b * m + q];
  }
  red[sl][c] = s;
  __syncthreads();
  if (sl == 0 && q < m) {
    const float v = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
    if (q < nw) dw[q] = v;
    else db[q - nw] = v;
  }
}


// Input gradient of the same conv + relu + pool (the second encoder conv's, VAE.py:48-50), from the pooled
// gradient: gx[ci][a][b] = sum_{co, ky, kx} g0[co][a + 1 - ky][b + 1 - kx] W[co][ci][ky][kx], g0 the routed
// full-resolution gradient (gy at each window's argmax where y > 0, 0 elsewhere).  One block per image, one
// thread per output pixel with all CI input channels in registers (pairs: packed fp32 FMAs).  g0 is formed in
// LDS with a zero border straight from (gy, y, idx) -- never written to HBM -- CC channels per stage (a
// smaller LDS stage: more blocks per CU); the 9 taps of a co are read from LDS once for the CI channels, and
// W's addresses are uniform across the block (scalar loads).  Replaces relu_maxpool2_bwd's full-resolution
// write plus MIOpen's backward-data conv and its NCHW <-> NHWC transposes.
template <int CI>
__global__ __launch_bounds__(1024) void conv3x3_pool_dgrad_kernel(const float* __restrict__ gy,
                                                                  const float* __restrict__ y,
                                                                  const uint8_t* __restrict__ idx,
                                                                  const float* __restrict__ w, int C, int Ho, int Wo,
                                                                  int CC, float* __restrict__ gx) {
  extern __shared__ float sm[];
  const int H = 2 * Ho, W = 2 * Wo, Wp = W + 2, HWp = (H + 2) * Wp, P = Ho * Wo;
  const int t = threadIdx.x, nthr = blockDim.x;
  const int64_t n = blockIdx.x;
  for (int e = t; e < CC * HWp; e += nthr) sm[e] = 0.f;  // (the border stays zero: each stage rewrites the interior)
  const int64_t b0 = n * C * P;
  const bool act = t < H * W;
  const int a = t / W, b = t % W;
  vo_f32x2 acc[CI / 2];
#pragma unroll
  for (int c = 0; c < CI / 2; ++c) acc[c] = vo_f32x2{0.f, 0.f};
  // tap (ky, kx) of output (a, b) reads g0 at padded (a + 2 - ky, b + 2 - kx)
  const float* g0 = sm + a * Wp + b;
  for (int c0 = 0; c0 < C; c0 += CC) {
    const int cc = min(CC, C - c0);
    __syncthreads();  // the previous stage's reads (and the zeroing) are done
    for (int e = t; e < cc * P; e += nthr) {
      const int c = e / P, r = e % P, i = r / Wo, j = r % Wo;
      const int64_t s = b0 + (int64_t)c0 * P + e;
      const float yv = y[s], gv = gy[s];
      const int k = idx[s];
      const float g = yv > 0.f ? gv : 0.f;
      float* q = sm + c * HWp + (2 * i + 1) * Wp + 2 * j + 1;
      q[0] = k == 0 ? g : 0.f;
      q[1] = k == 1 ? g : 0.f;
      q[Wp] = k == 2 ? g : 0.f;
      q[Wp + 1] = k == 3 ? g : 0.f;
    }
    __syncthreads();
    if (act) {
      for (int co = 0; co < cc; ++co) {
        const float* gc = g0 + co * HWp;
        const float* wc = w + (int64_t)(c0 + co) * CI * 9;
        float gt[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) gt[k] = gc[(2 - k / 3) * Wp + 2 - k % 3];
#pragma unroll
        for (int k = 0; k < 9; ++k) {
          const vo_f32x2 g2{gt[k], gt[k]};
#pragma unroll
          for (int c = 0; c < CI / 2; ++c) {
            const vo_f32x2 w2{wc[(2 * c) * 9 + k], wc[(2 * c + 1) * 9 + k]};
            acc[c] = __builtin_elementwise_fma(g2, w2, acc[c]);
          }
        }
      }
    }
  }
  if (act) {
    float* gxn = gx + n * CI * H * W + t;
#pragma unroll
    for (int c = 0; c < CI / 2; ++c) {
      gxn[(int64_t)(2 * c) * H * W] = acc[c][0];
      gxn[(int64_t)(2 * c + 1) * H * W] = acc[c][1];
    }
  }
}

// The same input gradient with one thread per horizontal pixel pair (a, b), (a, b + 1) (b even): the packed
// FMAs pair the two pixels (g from two adjacent LDS words, W's scalar broadcast to both halves) instead of two
// input channels, so W's per-tap scalar loads serve twice the FMAs and no SGPR pairs need assembling.
template <int CI>
__global__ __launch_bounds__(512) void conv3x3_pool_dgrad2_kernel(const float* __restrict__ gy,
                                                                  const float* __restrict__ y,
                                                                  const uint8_t* __restrict__ idx,
                                                                  const float* __restrict__ w, int C, int Ho, int Wo,
                                                                  float* __restrict__ gx) {
  extern __shared__ float sm[];
  const int H = 2 * Ho, W = 2 * Wo, Wp = W + 2, HWp = (H + 2) * Wp, P = Ho * Wo;
  const int t = threadIdx.x, nthr = blockDim.x;
  const int64_t n = blockIdx.x;
  for (int e = t; e < (H + 2) * Wp; e += nthr) {  // the zero border of every channel plane
    const int r = e / Wp, c = e % Wp;
    if (r == 0 || r == H + 1 || c == 0 || c == W + 1)
      for (int co = 0; co < C; ++co) sm[co * HWp + e] = 0.f;
  }
  const int64_t b0 = n * C * P;
  for (int e = t; e < C * P; e += nthr) {
    const int c = e / P, r = e % P, i = r / Wo, j = r % Wo;
    const float yv = y[b0 + e], gv = gy[b0 + e];
    const int k = idx[b0 + e];
    const float g = yv > 0.f ? gv : 0.f;
    float* q = sm + c * HWp + (2 * i + 1) * Wp + 2 * j + 1;
    q[0] = k == 0 ? g : 0.f;
    q[1] = k == 1 ? g : 0.f;
    q[Wp] = k == 2 ? g : 0.f;
    q[Wp + 1] = k == 3 ? g : 0.f;
  }
  __syncthreads();
  const int a = t / Wo, b = 2 * (t % Wo);
  if (t >= H * Wo) return;  // (after the only barrier)
  vo_f32x2 acc[CI];
#pragma unroll
  for (int c = 0; c < CI; ++c) acc[c] = vo_f32x2{0.f, 0.f};
  // tap (ky, kx) of pixel (a, b + d) reads g0 at padded (a + 2 - ky, b + d + 2 - kx)
  const float* g0 = sm + a * Wp + b;
  for (int co = 0; co < C; ++co) {
    const float* gc = g0 + co * HWp;
    const float* wc = w + (int64_t)co * CI * 9;
    vo_f32x2 gp[9];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const vo_f32x2 lo = *reinterpret_cast<const vo_f32x2*>(gc + (2 - ky) * Wp);
      const vo_f32x2 hi = *reinterpret_cast<const vo_f32x2*>(gc + (2 - ky) * Wp + 2);
      gp[3 * ky + 0] = hi;
      gp[3 * ky + 1] = vo_f32x2{lo[1], hi[0]};
      gp[3 * ky + 2] = lo;
    }
#pragma unroll
    for (int c = 0; c < CI; ++c) {
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        const float wv = wc[c * 9 + k];
        acc[c] = __builtin_elementwise_fma(gp[k], vo_f32x2{wv, wv}, acc[c]);
      }
    }
  }
  float* gxn = gx + n * CI * H * W + a * W + b;
#pragma unroll
  for (int c = 0; c < CI; ++c) *reinterpret_cast<vo_f32x2*>(gxn + (int64_t)c * H * W) = acc[c];
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

int lvae_conv1_relu_maxpool2_fwd_f32(const float* x, const float* w, const float* bias, int N, int C, int H, int W,
                                     float* y, uint8_t* idx, void* stream) {
  if (!x || !w || !bias || !y || !idx) return -1;
  if (N < 0 || C <= 0 || H < 2 || W < 2 || (H & 1) || (W & 1)) return -2;
  const int64_t total = (int64_t)N * (H / 2) * (W / 2);
  if (total == 0) return 0;
  conv1_relu_maxpool2_fwd_kernel<<<cdiv(total, 256), 256, 0, (hipStream_t)stream>>>(x, w, bias, N, C, H / 2, W / 2, y,
                                                                                     idx);
  LVAE_CHECK_LAUNCH();
  return 0;
}

static int deconv2_blocks(int N, int, int) { return (int)cdiv(N, imgs_per_block(N)); }

size_t lvae_deconv2_sigmoid_workspace_size(int N, int Cin, int Hi, int Wi) {
  return N <= 0 || Cin <= 0 ? 0 : sizeof(float) * ((size_t)Cin * 16 + 1) * (size_t)deconv2_blocks(N, Hi, Wi);
}

int lvae_deconv2_sigmoid_fwd_f32(const float* z, const float* w, const float* bias, int N, int Cin, int Hi, int Wi,
                                 float* out, void* stream) {
  if (!z || !w || !bias || !out) return -1;
  if (N < 0 || Cin <= 0 || Cin > 16 || Hi <= 0 || Wi <= 0) return -2;
  const int64_t total = (int64_t)N * 4 * Hi * Wi;
  if (total == 0) return 0;
  const size_t lds = sizeof(float) * Cin * (((Hi + 2) * (Wi + 2)) | 1);
  if (lds > 64 * 1024) return -3;
  deconv2_sigmoid_fwd_kernel<<<cdiv(N, imgs_per_block(N)), 256, lds, (hipStream_t)stream>>>(
      z, w, bias, N, Cin, Hi, Wi, imgs_per_block(N), out);
  LVAE_CHECK_LAUNCH();
  return 0;
}

int lvae_deconv2_sigmoid_bwd_f32(const float* g, const float* out, const float* z, const float* w, int N, int Cin,
                                 int Hi, int Wi, float* gz, float* dw, float* db, void* workspace, void* stream) {
  if (!g || !out || !z || !w || !gz || !dw || !db || !workspace) return -1;
  if (N < 0 || Cin <= 0 || Cin > 16 || Hi <= 0 || Wi <= 0) return -2;
  hipStream_t st = (hipStream_t)stream;
  if (N == 0) {
    (void)zero_async(dw, sizeof(float) * Cin * 16, st);
    (void)zero_async(db, sizeof(float), st);
    return 0;
  }
  const int nb = deconv2_blocks(N, Hi, Wi), m = Cin * 16 + 1;
  float* part = (float*)workspace;
  const size_t lds = sizeof(float) * ((size_t)(2 * Hi + 2) * (2 * Wi + 2) + (size_t)Cin * Hi * Wi);
  if (lds > 64 * 1024) return -3;
  deconv2_sigmoid_bwd_kernel<<<nb, 256, lds, st>>>(g, out, z, w, N, Cin, Hi, Wi, imgs_per_block(N), gz, part);
  wgrad_sum_kernel<<<cdiv(m, 64), 256, 0, st>>>(part, nb, m, Cin * 16, dw, db);
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

static size_t conv3x3_pool_wgrad_lds(int C, int Cin, int H, int W) {
  const size_t stage = (size_t)Cin * (((H + 2) * (W + 2)) | 1) + 2 * (size_t)C * (H / 2) * (W / 2);
  return sizeof(float) * (stage > 2560 ? stage : 2560);
}

// images per block of conv3x3_pool_wgrad_kernel: imgs_per_block, or LVAE_WGRAD_PER (A/B runs; read once, so the
// workspace size query and the launch agree)
static int wgrad_per(int N) {
  static const int v = getenv("LVAE_WGRAD_PER") ? atoi(getenv("LVAE_WGRAD_PER")) : 0;
  return v > 0 ? v : imgs_per_block(N);
}

size_t lvae_conv3x3_pool_wgrad_workspace_size(int N, int C, int Cin) {
  return N <= 0 || C <= 0 || Cin <= 0 ? 0 : sizeof(float) * ((size_t)C * Cin * 9 + C) * (size_t)cdiv(N, wgrad_per(N));
}

int lvae_conv3x3_pool_wgrad_f32(const float* gy, const float* y, const uint8_t* idx, const float* x, int N, int C,
                                int Cin, int H, int W, float* dw, float* db, void* workspace, void* stream) {
  if (!gy || !y || !idx || !x || !dw || !db || !workspace) return -1;
  if (N < 0 || C <= 0 || Cin <= 0 || H < 2 || W < 2 || (H & 1) || (W & 1)) return -2;
  const int Q = C * Cin, NP = (Q + 255) / 256;
  if (NP > 4) return -3;
  const size_t lds = conv3x3_pool_wgrad_lds(C, Cin, H, W);
  if (lds > 64 * 1024) return -4;
  hipStream_t st = (hipStream_t)stream;
  if (N == 0) {
    (void)zero_async(dw, sizeof(float) * Q * 9, st);
    (void)zero_async(db, sizeof(float) * C, st);
    return 0;
  }
  const int per = wgrad_per(N), nb = (int)cdiv(N, per), m = Q * 9 + C;
  float* part = (float*)workspace;
  const int Ho = H / 2, Wo = W / 2;
  switch (NP) {
    case 1: conv3x3_pool_wgrad_kernel<1><<<nb, 256, lds, st>>>(gy, y, idx, x, N, C, Cin, Ho, Wo, per, part); break;
    case 2: conv3x3_pool_wgrad_kernel<2><<<nb, 256, lds, st>>>(gy, y, idx, x, N, C, Cin, Ho, Wo, per, part); break;
    case 3: conv3x3_pool_wgrad_kernel<3><<<nb, 256, lds, st>>>(gy, y, idx, x, N, C, Cin, Ho, Wo, per, part); break;
    default: conv3x3_pool_wgrad_kernel<4><<<nb, 256, lds, st>>>(gy, y, idx, x, N, C, Cin, Ho, Wo, per, part); break;
  }
  wgrad_sum_kernel<<<cdiv(m, 64), 256, 0, st>>>(part, nb, m, Q * 9, dw, db);
  LVAE_CHECK_LAUNCH();
  return 0;
}

// channels per LDS stage of conv3x3_pool_dgrad_kernel: LVAE_DGRAD_CC (A/B runs), default 0 = all C in one stage
// (at the headline shape 243-256 us vs 257-269 with 16-channel stages and 268-278 with 8: the smaller stage's
// extra blocks per CU do not pay for its extra barriers; profiles/r5_conv_dgrad_ab.txt)
static int dgrad_cc(int C) {
  static const int v = getenv("LVAE_DGRAD_CC") ? atoi(getenv("LVAE_DGRAD_CC")) : 0;
  return v <= 0 || v > C ? C : v;
}

size_t lvae_conv3x3_pool_dgrad_lds(int C, int H, int W) {
  return sizeof(float) * (size_t)dgrad_cc(C) * (H + 2) * (W + 2);
}

int lvae_conv3x3_pool_dgrad_f32(const float* gy, const float* y, const uint8_t* idx, const float* w, int N, int C,
                                int Cin, int H, int W, float* gx, void* stream) {
  if (!gy || !y || !idx || !w || !gx) return -1;
  if (N < 0 || C <= 0 || Cin <= 0 || H < 2 || W < 2 || (H & 1) || (W & 1)) return -2;
  if (Cin != 16) return -3;
  const size_t lds = lvae_conv3x3_pool_dgrad_lds(C, H, W);
  if (lds > 64 * 1024 || H * W > 1024) return -4;
  if (N == 0) return 0;
  // LVAE_DGRAD_PAIR=0: one thread per pixel (channel-paired FMAs) instead of per pixel pair (pixel-paired: 209-221
  // vs 244-256 us at the headline shape; the step is unchanged, the weight-gradient kernel beside it is the longer
  // of the two; profiles/r5_conv_dgrad_ab.txt)
  static const bool pair = !getenv("LVAE_DGRAD_PAIR") || atoi(getenv("LVAE_DGRAD_PAIR")) != 0;
  if (pair && dgrad_cc(C) == C) {
    const int nthr = (int)cdiv((int64_t)H * W / 2, 64) * 64;
    conv3x3_pool_dgrad2_kernel<16><<<N, nthr, lds, (hipStream_t)stream>>>(gy, y, idx, w, C, H / 2, W / 2, gx);
  } else {
    const int nthr = (int)cdiv((int64_t)H * W, 64) * 64;
    conv3x3_pool_dgrad_kernel<16><<<N, nthr, lds, (hipStream_t)stream>>>(gy, y, idx, w, C, H / 2, W / 2,
                                                                         dgrad_cc(C), gx);
  }
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
    (void)zero_async(db, sizeof(float) * C, st);
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
