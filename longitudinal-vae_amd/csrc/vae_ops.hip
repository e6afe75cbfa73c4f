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

// ---- The second encoder conv end to end (VAE.py:48-50): conv3x3 (padding 1, CI input channels) + bias + relu +
// 2x2 max pool, C = 16 k output channels, H = W input, in one pass.  Replaces MIOpen's conv (an implicit GEMM over
// NHWC: NCHW -> NHWC transposes of the input and the weights and one back for its output) and
// relu_maxpool2_bias_fwd's pass over the full-resolution output (written and read once: 170 MB at 4096 images).
// IPB images per block are staged in LDS with a zero border.  Work item = (image, pooled position, group of 16
// output channels); 64 consecutive items of a wave share the group, so W's addresses are uniform across the wave
// (scalar loads, broadcast into the packed FMAs).  An item reads the 4 x 4 input patch under its window once per
// input channel and keeps the window's 2 x 2 conv outputs of its 16 channels in packed accumulators (a window row's
// two columns in one pair): per output sum_ci sum_ky sum_kx x w (this order) + b, then relu + first strict maximum
// (scan order) exactly as relu_maxpool2_bias_fwd_kernel.
template <int CI, int H, int IPB>
__global__ __launch_bounds__(256) void conv3x3_relu_pool_fwd_kernel(const float* __restrict__ x,
                                                                    const float* __restrict__ w,
                                                                    const float* __restrict__ bias, int N, int C,
                                                                    float* __restrict__ y, uint8_t* __restrict__ idx) {
  constexpr int W = H, Wp = W + 2, HWp = (H + 2) * Wp, Ho = H / 2, Wo = W / 2, P = Ho * Wo, HW = H * W;
  __shared__ float xl[IPB * CI * HWp];
  const int t = threadIdx.x, n0 = blockIdx.x * IPB, ni = min(IPB, N - n0);
  for (int e = t; e < IPB * CI * HWp; e += 256) xl[e] = 0.f;
  __syncthreads();
  const float* xb = x + (int64_t)n0 * CI * HW;
  for (int e = t; e < ni * CI * HW; e += 256) {
    const int pl = e / HW, r = e - pl * HW, rr = r / W;
    xl[pl * HWp + (rr + 1) * Wp + (r - rr * W) + 1] = xb[e];
  }
  __syncthreads();
  const int ntask = ni * P, nchunk = (ntask + 63) >> 6, ngrp = C >> 4, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);  // (uniform: W's loads scalar)
  for (int ch = wave; ch < nchunk * ngrp; ch += 4) {
    const int grp = ch % ngrp, task = (ch / ngrp) * 64 + lane;
    const int tk = task < ntask ? task : ntask - 1;
    const int img = tk / P, r = tk - img * P, i = r / Wo, j = r - i * Wo;
    const float* xp = xl + img * CI * HWp + 2 * i * Wp + 2 * j;  // padded (2 i, 2 j) = input (2 i - 1, 2 j - 1)
    const float* wg = w + (int64_t)grp * 16 * CI * 9;
    vo_f32x2 acc[16][2];
#pragma unroll
    for (int co = 0; co < 16; ++co) acc[co][0] = acc[co][1] = vo_f32x2{0.f, 0.f};
    for (int ci = 0; ci < CI; ++ci) {
      const float* xc = xp + ci * HWp;
      float p[4][4];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) p[a][b] = xc[a * Wp + b];
#pragma unroll
      for (int co = 0; co < 16; ++co) {
        const float* wc = wg + (co * CI + ci) * 9;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            const float wv = wc[3 * ky + kx];
            acc[co][0] = __builtin_elementwise_fma(vo_f32x2{p[ky][kx], p[ky][kx + 1]}, vo_f32x2{wv, wv}, acc[co][0]);
            acc[co][1] =
                __builtin_elementwise_fma(vo_f32x2{p[ky + 1][kx], p[ky + 1][kx + 1]}, vo_f32x2{wv, wv}, acc[co][1]);
          }
      }
    }
    if (task < ntask) {
#pragma unroll
      for (int co = 0; co < 16; ++co) {
        const int c = grp * 16 + co;
        const float bc = bias[c];
        float m = acc[co][0][0] + bc;
        uint8_t k = 0;
        if (acc[co][0][1] + bc > m) m = acc[co][0][1] + bc, k = 1;
        if (acc[co][1][0] + bc > m) m = acc[co][1][0] + bc, k = 2;
        if (acc[co][1][1] + bc > m) m = acc[co][1][1] + bc, k = 3;
        const int64_t o = ((int64_t)(n0 + img) * C + c) * P + r;
        y[o] = m > 0.f ? m : 0.f;
        idx[o] = k;
      }
    }
  }
}

// ---- The decoder's first transposed conv (VAE.py:73, 122): relu(ConvTranspose2d(CI, CO, 4, stride 2, padding 1)(x)
// + b), x [N, CI, HI, HI] -> [N, CO, 2 HI, 2 HI], in one pass (MIOpen's transposed conv with its transposes, then
// bias_relu_fwd, before).  Output (2 iy + a, 2 ix + b) takes input rows iy, iy - 1 (a = 0: ky 1, 3) or iy + 1, iy
// (a = 1: ky 0, 2), columns likewise: 4 taps per input channel (deconv2_sigmoid_fwd_kernel's indexing).  IPB images
// per block in LDS with a zero border; item = (image, input position, group of 8 output channels), the group
// uniform across a wave (W's row of 16 taps per (ci, co) by scalar loads); the item's 2 x 2 output block of its 8
// channels in packed accumulators (the two columns of an output row in one pair).  relu as bias_relu_fwd: v < 0 ->
// 0, NaN kept.
template <int CI, int CO, int HI, int IPB>
__global__ __launch_bounds__(256) void deconv4s2_relu_fwd_kernel(const float* __restrict__ x,
                                                                 const float* __restrict__ w,
                                                                 const float* __restrict__ bias, int N,
                                                                 float* __restrict__ y) {
  constexpr int Wp = HI + 2, HWp = (HI + 2) * Wp, P = HI * HI, Wo = 2 * HI, PO = 4 * P, NG = CO / 8;
  __shared__ float xl[IPB * CI * HWp];
  const int t = threadIdx.x, n0 = blockIdx.x * IPB, ni = min(IPB, N - n0);
  for (int e = t; e < IPB * CI * HWp; e += 256) xl[e] = 0.f;
  __syncthreads();
  const float* xb = x + (int64_t)n0 * CI * P;
  for (int e = t; e < ni * CI * P; e += 256) {
    const int pl = e / P, r = e - pl * P, rr = r / HI;
    xl[pl * HWp + (rr + 1) * Wp + (r - rr * HI) + 1] = xb[e];
  }
  __syncthreads();
  const int ntask = ni * P, nchunk = (ntask + 63) >> 6, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);  // (uniform: W's loads scalar)
  for (int ch = wave; ch < nchunk * NG; ch += 4) {
    const int grp = ch % NG, task = (ch / NG) * 64 + lane;
    const int tk = task < ntask ? task : ntask - 1;
    const int img = tk / P, q = tk - img * P, iy = q / HI, ix = q - iy * HI;
    const float* xp = xl + img * CI * HWp + iy * Wp + ix;  // padded (iy, ix) = input (iy - 1, ix - 1)
    vo_f32x2 acc[8][2];
#pragma unroll
    for (int co = 0; co < 8; ++co) acc[co][0] = acc[co][1] = vo_f32x2{0.f, 0.f};
    for (int ci = 0; ci < CI; ++ci) {
      const float* xc = xp + ci * HWp;
      float v[3][3];
#pragma unroll
      for (int u = 0; u < 3; ++u)
#pragma unroll
        for (int c = 0; c < 3; ++c) v[u][c] = xc[u * Wp + c];
#pragma unroll
      for (int co = 0; co < 8; ++co) {
        const float* wc = w + ((int64_t)ci * CO + grp * 8 + co) * 16;
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const int ky = a == 0 ? 1 + 2 * u : 2 * u, ry = a == 0 ? 1 - u : 2 - u;
#pragma unroll
            for (int c = 0; c < 2; ++c)  // b = 0: (kx 1 + 2 c, col 1 - c); b = 1: (kx 2 c, col 2 - c)
              acc[co][a] = __builtin_elementwise_fma(vo_f32x2{v[ry][1 - c], v[ry][2 - c]},
                                                     vo_f32x2{wc[ky * 4 + 1 + 2 * c], wc[ky * 4 + 2 * c]}, acc[co][a]);
          }
      }
    }
    if (task < ntask) {
#pragma unroll
      for (int co = 0; co < 8; ++co) {
        const int c = grp * 8 + co;
        const float bc = bias[c];
        float* yo = y + ((int64_t)(n0 + img) * CO + c) * PO + (2 * iy) * Wo + 2 * ix;
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          vo_f32x2 r2 = acc[co][a] + vo_f32x2{bc, bc};
          r2[0] = r2[0] < 0.f ? 0.f : r2[0];
          r2[1] = r2[1] < 0.f ? 0.f : r2[1];
          *reinterpret_cast<vo_f32x2*>(yo + a * Wo) = r2;
        }
      }
    }
  }
}

// Its backward from d y and y: g = d y [y > 0] (act_bwd's mask: y <= 0 -> 0), then in one pass per block of `per`
// images (IPB at a time in LDS: g with a zero border, x):
//   dx[ci][iy][ix] = sum_co sum_{ky,kx} W[ci][co][ky][kx] g[co][2 iy - 1 + ky][2 ix - 1 + kx]   (written per image)
//   dW[ci][co][ky][kx] = sum_n sum_{iy,ix} x[ci][iy][ix] g[co][2 iy - 1 + ky][2 ix - 1 + kx]     (block partials)
//   db[co] = sum g                                                                                (block partials)
// dx items = (image, input position, group of 8 input channels), the group uniform across a wave (W by scalar
// loads), two channels per packed FMA.  dW: thread (co = t & 15, ci 4 ((t >> 4) & 7) + 0..3, position parity
// t >> 7) keeps its 4 x 16 taps in packed accumulators over the block's images (tap pairs per FMA); the two
// parities are separate partial rows.  Partials part[2 block + parity][CI CO 16 + CO], summed in a fixed order by
// wgrad_sum_kernel: deterministic.  Replaces act_bwd (mask + bias sum), MIOpen's backward-data and backward-weights
// convs and their five NCHW <-> NHWC transposes.
template <int CI, int CO, int HI, int IPB>
__global__ __launch_bounds__(256) void deconv4s2_relu_bwd_kernel(const float* __restrict__ gy,
                                                                 const float* __restrict__ y,
                                                                 const float* __restrict__ x,
                                                                 const float* __restrict__ w, int N, int per,
                                                                 float* __restrict__ dx, float* __restrict__ part) {
  static_assert(CI == 32 && CO == 16, "the dW thread map: 16 output x 8 groups of 4 input channels x 2 parities");
  constexpr int P = HI * HI, Wo = 2 * HI, PO = 4 * P, Gp = Wo + 2, GP = ((2 * HI + 2) * Gp) | 1, NG = CI / 8;
  __shared__ float gl[IPB * CO * GP];  // (odd plane stride: the 16 co lanes of a dW read hit distinct banks)
  __shared__ float xs[IPB * CI * P];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);  // (uniform: W's loads scalar)
  const int wco = t & 15, wcg = (t >> 4) & 7, par = t >> 7;
  const int nb0 = blockIdx.x * per, nb1 = min(N, nb0 + per);
  for (int e = t; e < IPB * CO * GP; e += 256) gl[e] = 0.f;  // (the borders stay zero: each group rewrites the interior)
  vo_f32x2 dacc[4][8];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int p = 0; p < 8; ++p) dacc[k][p] = vo_f32x2{0.f, 0.f};
  float bacc = 0.f;
  for (int g0 = nb0; g0 < nb1; g0 += IPB) {
    const int ni = min(IPB, nb1 - g0);
    __syncthreads();  // the previous group's readers are done
    const int64_t ob = (int64_t)g0 * CO * PO;
    for (int e = t; e < ni * CO * PO; e += 256) {
      const int pl = e / PO, r = e - pl * PO, rr = r / Wo;
      const float yv = y[ob + e], gv = gy[ob + e];
      gl[pl * GP + (rr + 1) * Gp + (r - rr * Wo) + 1] = yv <= 0.f ? 0.f : gv;
    }
    const float* xb = x + (int64_t)g0 * CI * P;
    for (int e = t; e < ni * CI * P; e += 256) xs[e] = xb[e];
    __syncthreads();
    // dx
    const int ntask = ni * P, nchunk = (ntask + 63) >> 6;
    for (int ch = wave; ch < nchunk * NG; ch += 4) {
      const int grp = ch % NG, task = (ch / NG) * 64 + lane;
      const int tk = task < ntask ? task : ntask - 1;
      const int img = tk / P, q = tk - img * P, iy = q / HI, ix = q - iy * HI;
      const float* gp = gl + img * CO * GP + (2 * iy) * Gp + 2 * ix;  // padded (2 iy, 2 ix) = (2 iy - 1, 2 ix - 1)
      vo_f32x2 xa[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) xa[k] = vo_f32x2{0.f, 0.f};
      for (int co = 0; co < CO; ++co) {
        float pt[16];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int c = 0; c < 4; ++c) pt[4 * a + c] = gp[co * GP + a * Gp + c];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float* w0 = w + ((int64_t)(grp * 8 + 2 * k) * CO + co) * 16;  // W[ci][co][:], W[ci + 1][co][:]
#pragma unroll
          for (int tp = 0; tp < 16; ++tp)
            xa[k] = __builtin_elementwise_fma(vo_f32x2{pt[tp], pt[tp]}, vo_f32x2{w0[tp], w0[CO * 16 + tp]}, xa[k]);
        }
      }
      if (task < ntask) {
        float* dxo = dx + ((int64_t)(g0 + img) * CI + grp * 8) * P + q;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          dxo[(2 * k) * P] = xa[k][0];
          dxo[(2 * k + 1) * P] = xa[k][1];
        }
      }
    }
    // dW, db
    for (int img = 0; img < ni; ++img) {
      const float* xi = xs + (img * CI + 4 * wcg) * P;
      const float* gi = gl + (img * CO + wco) * GP;
      for (int q = par; q < P; q += 2) {
        const int iy = q / HI, ix = q - iy * HI;
        float pt[16];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int c = 0; c < 4; ++c) pt[4 * a + c] = gi[(2 * iy + a) * Gp + 2 * ix + c];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float xv = xi[k * P + q];
#pragma unroll
          for (int p = 0; p < 8; ++p)
            dacc[k][p] = __builtin_elementwise_fma(vo_f32x2{pt[2 * p], pt[2 * p + 1]}, vo_f32x2{xv, xv}, dacc[k][p]);
        }
      }
      if (wcg == 0)
        for (int r = par; r < PO; r += 2) {
          const int rr = r / Wo;
          bacc += gi[(rr + 1) * Gp + (r - rr * Wo) + 1];
        }
    }
  }
  constexpr int M = CI * CO * 16 + CO;
  float* pb = part + (int64_t)(2 * blockIdx.x + par) * M;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float* pw = pb + ((4 * wcg + k) * CO + wco) * 16;
#pragma unroll
    for (int p = 0; p < 8; ++p) *reinterpret_cast<vo_f32x2*>(pw + 2 * p) = dacc[k][p];
  }
  if (wcg == 0) pb[CI * CO * 16 + wco] = bacc;
}

// The same backward on the f32 MFMA (v_mfma_f32_32x32x2_f32: a k-ordered f32 fma chain, the VALU's numerics at
// 2.3x its practical rate).  One image at a time in LDS: g (masked, zero border), x (positions padded to 96 with
// zeros), and W^T [k = 16 co + tap][ci] loaded once per block.  With G [k][pos] = g[co][2 iy - 1 + ky][2 ix - 1 + kx]
// (the im2col of g, gathered from LDS straight into the MFMA operands):
//   dx^T [pos][ci] = sum_k G^T [pos][k] W^T [k][ci]   -- 3 tiles of 32 positions (81 valid), K = 256: waves 0..2;
//   dW [ci][k]     = sum_pos x [ci][pos] G^T [pos][k] -- 8 tiles of 32 k, K = the positions of all the block's
//                    images (accumulated in registers): one tile on each of waves 0..2, five on wave 3.
// Per image 169 MFMAs on waves 0..2 and 205 on wave 3.  db from the staged g (16 pixel slices per channel, summed in
// a fixed order at the end).  Block partials part[block][CI CO 16 + CO], wgrad_sum_kernel as before.
typedef float vo_f32x16 __attribute__((ext_vector_type(16)));
__global__ __launch_bounds__(256) void deconv4s2_relu_bwd_mfma_kernel(const float* __restrict__ gy,
                                                                      const float* __restrict__ y,
                                                                      const float* __restrict__ x,
                                                                      const float* __restrict__ w, int N, int per,
                                                                      float* __restrict__ dx, float* __restrict__ part) {
  constexpr int CI = 32, CO = 16, HI = 9, P = HI * HI, Wo = 2 * HI, PO = 4 * P, Gp = Wo + 2;
  constexpr int GP = ((2 * HI + 2) * Gp) | 1;  // (odd plane stride)
  constexpr int XS = 97;                       // x plane stride: >= 82 positions, odd (the 32 ci lanes: distinct banks)
  constexpr int K = CO * 16;
  __shared__ float gl[CO * GP];
  __shared__ float xs[CI * XS];
  __shared__ float wt[K * CI];  // W^T [k][ci]
  __shared__ float red[256];
  const int t = threadIdx.x, lane = t & 63, l32 = lane & 31, hi = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int nb0 = blockIdx.x * per, nb1 = min(N, nb0 + per);
  for (int e = t; e < CO * GP; e += 256) gl[e] = 0.f;
  for (int e = t; e < CI * XS; e += 256) xs[e] = 0.f;
  for (int e = t; e < K * CI; e += 256) {  // w [ci][k] -> wt [k][ci]
    const int ci = e / K, k = e - ci * K;
    wt[k * CI + ci] = w[e];
  }
  vo_f32x16 dwacc[5];
#pragma unroll
  for (int j = 0; j < 5; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) dwacc[j][r] = 0.f;
  const int ntile = wave == 3 ? 5 : 1, tile0 = wave == 3 ? 3 : wave;
  float bacc = 0.f;
  const int bco = t & 15, bsl = t >> 4;
  // the next image's y, d y and x in registers, loaded under the current image's MFMAs
  constexpr int NG = (CO * PO + 255) / 256, NX = (CI * P + 255) / 256;
  float pg[NG], px[NX];
  auto fetch = [&](int n) {
    const int64_t ob = (int64_t)n * CO * PO;
#pragma unroll
    for (int k = 0; k < NG; ++k) {
      const int e = t + 256 * k;
      if (e < CO * PO) {
        const float yv = y[ob + e], gv = gy[ob + e];
        pg[k] = yv <= 0.f ? 0.f : gv;
      }
    }
    const float* xn = x + (int64_t)n * CI * P;
#pragma unroll
    for (int k = 0; k < NX; ++k) {
      const int e = t + 256 * k;
      if (e < CI * P) px[k] = xn[e];
    }
  };
  if (nb0 < nb1) fetch(nb0);
  for (int n = nb0; n < nb1; ++n) {
    __syncthreads();  // the previous image's readers are done (and the zeroing / W^T staged)
#pragma unroll
    for (int k = 0; k < NG; ++k) {
      const int e = t + 256 * k;
      if (e < CO * PO) {
        const int co = e / PO, r = e - co * PO, rr = r / Wo;
        gl[co * GP + (rr + 1) * Gp + (r - rr * Wo) + 1] = pg[k];
      }
    }
#pragma unroll
    for (int k = 0; k < NX; ++k) {
      const int e = t + 256 * k;
      if (e < CI * P) {
        const int ci = e / P;
        xs[ci * XS + (e - ci * P)] = px[k];
      }
    }
    if (n + 1 < nb1) fetch(n + 1);
    __syncthreads();
    for (int r = bsl; r < PO; r += 16) {  // db: channel bco, pixel slice bsl
      const int rr = r / Wo;
      bacc += gl[bco * GP + (rr + 1) * Gp + (r - rr * Wo) + 1];
    }
    // dW: K = this image's positions, 2 per step (pos 81 of the last step: x is 0 there)
#pragma unroll 2
    for (int s = 0; s < (P + 1) / 2; ++s) {
      const int pos = 2 * s + hi, pc = pos < P ? pos : P - 1, iy = pc / HI, ix = pc - iy * HI;
      const float a = xs[l32 * XS + pos];
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        if (j < ntile) {
          const int kk = (tile0 + j) * 32 + l32, co = kk >> 4, ky = (kk >> 2) & 3, kx = kk & 3;
          const float b = gl[co * GP + (2 * iy + ky) * Gp + 2 * ix + kx];
          dwacc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, pos < P ? b : 0.f, dwacc[j], 0, 0, 0);
        }
      }
    }
    // dx: waves 0..2, positions 32 wave + 0..31
    if (wave < 3) {
      const int pos = 32 * wave + l32, pv = pos < P, pc = pv ? pos : P - 1, iy = pc / HI, ix = pc - iy * HI;
      const float* gq = gl + (2 * iy) * Gp + 2 * ix;
      vo_f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll 4
      for (int s = 0; s < K / 2; ++s) {
        const int k = 2 * s + hi, co = k >> 4, ky = (k >> 2) & 3, kx = k & 3;
        const float a = gq[co * GP + ky * Gp + kx];
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(pv ? a : 0.f, wt[k * CI + l32], acc, 0, 0, 0);
      }
      float* dxn = dx + (int64_t)n * CI * P + l32 * P;  // column = ci (the lane), rows = positions
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int pr = 32 * wave + (r & 3) + 8 * (r >> 2) + 4 * hi;
        if (pr < P) dxn[pr] = acc[r];
      }
    }
  }
  constexpr int M = CI * K + CO;
  float* pb = part + (int64_t)blockIdx.x * M;
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    if (j < ntile) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ci = (r & 3) + 8 * (r >> 2) + 4 * hi;
        pb[ci * K + (tile0 + j) * 32 + l32] = dwacc[j][r];
      }
    }
  }
  red[t] = bacc;
  __syncthreads();
  if (t < CO) {
    float s = 0.f;
    for (int sl = 0; sl < 16; ++sl) s += red[sl * 16 + t];
    pb[CI * K + t] = s;
  }
}

// The second encoder conv's weight and bias gradients on the f32 MFMA (v_mfma_f32_16x16x4_f32), dense over the
// routed full-resolution gradient g0 (gy at each window's argmax where y > 0, 0 at the other three positions):
//   dW [co][k = 9 ci + 3 ky + kx] = sum_n sum_pos g0[co][pos] x[ci][pos + (ky - 1, kx - 1)],  db[co] = sum g0.
// conv3x3_pool_wgrad_kernel reads one x patch per nonzero g0 with no reuse (LDS-bound: one read per FMA); here
// every operand read feeds 16 MACs and the 3 zeros of a window ride along (4x the MACs at 2.3x the rate, a fraction
// of the LDS traffic).  Per image in LDS: g0 [co][324] and x with a zero border; the next image's pooled gradient,
// y, idx and x prefetched into registers under the MFMAs.  Every wave owns all 2 x 9 tiles (16 co x 16 k) over its
// quarter of the positions (steps of 4, s = wave mod 4): 2 A reads + 9 B gathers per 18 MFMAs, no branches; the
// four quarters are separate partial rows.  Partials part[4 block + wave][C 144 + C] (conv3x3_pool_wgrad_kernel's
// row layout), summed in a fixed order by wgrad_sum_kernel.
__global__ __launch_bounds__(256) void conv3x3_pool_wgrad_mfma_kernel(const float* __restrict__ gy,
                                                                      const float* __restrict__ y,
                                                                      const uint8_t* __restrict__ idx,
                                                                      const float* __restrict__ x, int N, int per,
                                                                      float* __restrict__ part) {
  constexpr int CI = 16, C = 32, H = 18, W = 18, Ho = 9, Wo = 9, P = Ho * Wo, PF = H * W, Wp = W + 2;
  constexpr int XP = ((H + 2) * Wp) | 1, GS = PF | 1, K2 = CI * 9, NT = K2 / 16;
  __shared__ float g0[C * GS];
  __shared__ float xl[CI * XP];
  __shared__ float red[256];
  const int t = threadIdx.x, lane = t & 63, l16 = lane & 15, kq = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int nb0 = blockIdx.x * per, nb1 = min(N, nb0 + per);
  for (int e = t; e < CI * XP; e += 256) xl[e] = 0.f;  // (the border stays zero)
  typedef float f32x4_t __attribute__((ext_vector_type(4)));
  f32x4_t acc[2][NT];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[m][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // B gather offsets (k = 16 j + l16 -> ci, ky, kx): padded (a + ky, b + kx) of plane ci
  int boff[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int k = 16 * j + l16, ci = k / 9, r9 = k - 9 * ci;
    boff[j] = ci * XP + (r9 / 3) * Wp + (r9 % 3);
  }
  float bacc = 0.f;
  const int bco = t & 31, bsl = t >> 5;
  constexpr int NGP = (C * P + 255) / 256, NXP = (CI * PF + 255) / 256;
  float pg[NGP], px[NXP];
  int pk[NGP];
  auto fetch = [&](int n) {
    const int64_t ob = (int64_t)n * C * P;
#pragma unroll
    for (int k = 0; k < NGP; ++k) {
      const int e = t + 256 * k;
      if (e < C * P) {
        const float yv = y[ob + e], gv = gy[ob + e];
        pg[k] = yv > 0.f ? gv : 0.f;
        pk[k] = idx[ob + e];
      }
    }
    const float* xn = x + (int64_t)n * CI * PF;
#pragma unroll
    for (int k = 0; k < NXP; ++k) {
      const int e = t + 256 * k;
      if (e < CI * PF) px[k] = xn[e];
    }
  };
  if (nb0 < nb1) fetch(nb0);
  for (int n = nb0; n < nb1; ++n) {
    __syncthreads();  // the previous image's readers are done (and the zeroing)
#pragma unroll
    for (int k = 0; k < NGP; ++k) {
      const int e = t + 256 * k;
      if (e < C * P) {
        const int co = e / P, r = e - co * P, i = r / Wo, j = r - i * Wo;
        float* q = g0 + co * GS + (2 * i) * W + 2 * j;
        q[0] = pk[k] == 0 ? pg[k] : 0.f;
        q[1] = pk[k] == 1 ? pg[k] : 0.f;
        q[W] = pk[k] == 2 ? pg[k] : 0.f;
        q[W + 1] = pk[k] == 3 ? pg[k] : 0.f;
      }
    }
#pragma unroll
    for (int k = 0; k < NXP; ++k) {
      const int e = t + 256 * k;
      if (e < CI * PF) {
        const int ci = e / PF, r = e - ci * PF, rr = r / W;
        xl[ci * XP + (rr + 1) * Wp + (r - rr * W) + 1] = px[k];
      }
    }
    if (n + 1 < nb1) fetch(n + 1);
    __syncthreads();
    for (int r = bsl; r < PF; r += 8) bacc += g0[bco * GS + r];  // db: channel bco, slice bsl
#pragma unroll 2
    for (int s = wave; s < PF / 4; s += 4) {
      const int pos = 4 * s + kq, a = pos / W, b = pos - a * W;
      const float a0 = g0[l16 * GS + pos], a1 = g0[(16 + l16) * GS + pos];
      const float* xb = xl + a * Wp + b;
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const float bv = xb[boff[j]];
        acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, bv, acc[0][j], 0, 0, 0);
        acc[1][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, bv, acc[1][j], 0, 0, 0);
      }
    }
  }
  constexpr int M = C * K2 + C;
  float* pb = part + (int64_t)(4 * blockIdx.x + wave) * M;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) pb[(16 * m + kq * 4 + r) * K2 + 16 * j + l16] = acc[m][j][r];
  red[t] = bacc;
  __syncthreads();
  if (t < C) {  // db into wave 0's row; the other rows' db slots zero
    float s = 0.f;
    for (int sl = 0; sl < 8; ++sl) s += red[sl * 32 + t];
    pb[C * K2 + t] = s;
  } else if (t >= 64 && (t & 63) < C) {
    pb[C * K2 + (t & 63)] = 0.f;
  }
}

// The second encoder conv's input gradient on the f32 MFMA (v_mfma_f32_16x16x4_f32), dense over the routed
// full-resolution gradient g0 (as conv3x3_pool_wgrad_mfma_kernel's):
//   gx^T [pos][ci] = sum_{k = 9 co + 3 ky + kx} g0[co][pos + (1 - ky, 1 - kx)] W[co][ci][ky][kx]   (K = 288).
// One image per iteration in LDS: g0 with a zero border and W^T [k][ci] (once per block); the next image's pooled
// gradient, y and idx prefetched into registers.  Position tiles of 16 (324 -> 21, padded to 24: 6 per wave, the
// same k per lane for the wave's 6 tiles: one W^T read and one offset computation per 6 MFMAs).  Output rows
// 16 tile + 4 (lane >> 4) + 0..3: four consecutive positions of one channel per lane (one 16-byte store).
__global__ __launch_bounds__(256) void conv3x3_pool_dgrad_mfma_kernel(const float* __restrict__ gy,
                                                                      const float* __restrict__ y,
                                                                      const uint8_t* __restrict__ idx,
                                                                      const float* __restrict__ w, int N, int per,
                                                                      float* __restrict__ gx) {
  constexpr int CI = 16, C = 32, H = 18, W = 18, Ho = 9, Wo = 9, P = Ho * Wo, PF = H * W, Wp = W + 2;
  constexpr int GP = ((H + 2) * Wp) | 1, K = C * 9, TPW = 6;
  __shared__ float g0[C * GP];
  __shared__ float wt[K * CI];  // W^T [k][ci]
  const int t = threadIdx.x, lane = t & 63, l16 = lane & 15, kq = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int nb0 = blockIdx.x * per, nb1 = min(N, nb0 + per);
  for (int e = t; e < C * GP; e += 256) g0[e] = 0.f;  // (the border stays zero)
  for (int e = t; e < C * CI * 9; e += 256) {       // w [co][ci][tap] -> wt [9 co + tap][ci]
    const int co = e / (CI * 9), r = e - co * CI * 9, ci = r / 9, tap = r - 9 * ci;
    wt[(9 * co + tap) * CI + ci] = w[e];
  }
  // the wave's position tiles: 16 (wave + 4 j) + l16 (A rows); padded (a + 2, b + 2) - (ky, kx) is the read
  int aoff[TPW];
  bool aval[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int pos = 16 * (wave + 4 * j) + l16, pc = pos < PF ? pos : PF - 1, a = pc / W, b = pc - a * W;
    aoff[j] = (a + 2) * Wp + b + 2;
    aval[j] = pos < PF;
  }
  constexpr int NGP = (C * P + 255) / 256;
  float pg[NGP];
  int pk[NGP];
  auto fetch = [&](int n) {
    const int64_t ob = (int64_t)n * C * P;
#pragma unroll
    for (int k = 0; k < NGP; ++k) {
      const int e = t + 256 * k;
      if (e < C * P) {
        const float yv = y[ob + e], gv = gy[ob + e];
        pg[k] = yv > 0.f ? gv : 0.f;
        pk[k] = idx[ob + e];
      }
    }
  };
  if (nb0 < nb1) fetch(nb0);
  typedef float f32x4_t __attribute__((ext_vector_type(4)));
  for (int n = nb0; n < nb1; ++n) {
    __syncthreads();  // the previous image's readers are done (and the zeroing / W^T staged)
#pragma unroll
    for (int k = 0; k < NGP; ++k) {
      const int e = t + 256 * k;
      if (e < C * P) {
        const int co = e / P, r = e - co * P, i = r / Wo, j = r - i * Wo;
        float* q = g0 + co * GP + (2 * i + 1) * Wp + 2 * j + 1;
        q[0] = pk[k] == 0 ? pg[k] : 0.f;
        q[1] = pk[k] == 1 ? pg[k] : 0.f;
        q[Wp] = pk[k] == 2 ? pg[k] : 0.f;
        q[Wp + 1] = pk[k] == 3 ? pg[k] : 0.f;
      }
    }
    if (n + 1 < nb1) fetch(n + 1);
    __syncthreads();
    f32x4_t acc[TPW];
#pragma unroll
    for (int j = 0; j < TPW; ++j) acc[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int s = 0; s < K / 4; ++s) {
      const int k = 4 * s + kq, co = (k * 57) >> 9, r9 = k - 9 * co, ky = (r9 * 11) >> 5, kx = r9 - 3 * ky;
      const float* gk = g0 + co * GP - ky * Wp - kx;
      const float bv = wt[k * CI + l16];
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
        const float av = gk[aoff[j]];
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(aval[j] ? av : 0.f, bv, acc[j], 0, 0, 0);
      }
    }
    float* gxn = gx + ((int64_t)n * CI + l16) * PF;  // column = ci (lane & 15)
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int p0 = 16 * (wave + 4 * j) + 4 * kq;
      if (p0 < PF) *reinterpret_cast<f32x4_t*>(gxn + p0) = acc[j];
    }
  }
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

// the second encoder conv's shape takes the dense f32-MFMA form (LVAE_WGRAD_MFMA=0: the sparse VALU form; read
// once, so the workspace size query and the launch agree): 4 partial rows per block of 2 wgrad_per images
static bool wgrad_mfma(int C, int Cin, int H, int W) {
  static const bool on = !getenv("LVAE_WGRAD_MFMA") || atoi(getenv("LVAE_WGRAD_MFMA")) != 0;
  return on && Cin == 16 && C == 32 && H == 18 && W == 18;
}

size_t lvae_conv3x3_pool_wgrad_workspace_size(int N, int C, int Cin) {
  if (N <= 0 || C <= 0 || Cin <= 0) return 0;
  const size_t rows = (size_t)cdiv(N, wgrad_per(N)), rows2 = 4 * (size_t)cdiv(N, 2 * wgrad_per(N));
  // (the MFMA form's rows when the shape can take it: H, W are not arguments here)
  return sizeof(float) * ((size_t)C * Cin * 9 + C) * (wgrad_mfma(C, Cin, 18, 18) && rows2 > rows ? rows2 : rows);
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
  // the second encoder conv's shape: the dense f32-MFMA form (LVAE_WGRAD_MFMA=0: the sparse VALU form), twice the
  // images per block (fewer partial rows than the workspace holds)
  if (wgrad_mfma(C, Cin, H, W)) {
    const int nb2 = (int)cdiv(N, 2 * per);
    conv3x3_pool_wgrad_mfma_kernel<<<nb2, 256, 0, st>>>(gy, y, idx, x, N, 2 * per, part);
    wgrad_sum_kernel<<<cdiv(m, 64), 256, 0, st>>>(part, 4 * nb2, m, Q * 9, dw, db);
    LVAE_CHECK_LAUNCH();
    return 0;
  }
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
  // the second encoder conv's shape: the dense f32-MFMA form (LVAE_DGRAD_MFMA=0: the VALU kernels below)
  static const bool mfma = !getenv("LVAE_DGRAD_MFMA") || atoi(getenv("LVAE_DGRAD_MFMA")) != 0;
  if (mfma && C == 32 && H == 18 && W == 18) {
    const int per = N >= 4096 ? 8 : N >= 2048 ? 4 : N >= 1024 ? 2 : 1;
    conv3x3_pool_dgrad_mfma_kernel<<<cdiv(N, per), 256, 0, (hipStream_t)stream>>>(gy, y, idx, w, N, per, gx);
  } else if (pair && dgrad_cc(C) == C) {
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

// The fused second-conv forward: Cin 16, H = W = 18 (the ConvVAE's 36 x 36 images after the first pool), C a
// multiple of 16; -3 for other shapes (the caller keeps MIOpen's conv + relu_maxpool2_bias_fwd for them).
int lvae_conv3x3_relu_maxpool2_fwd_f32(const float* x, const float* w, const float* bias, int N, int Cin, int C, int H,
                                       int W, float* y, uint8_t* idx, void* stream) {
  if (!x || !w || !bias || !y || !idx) return -1;
  if (N < 0 || Cin <= 0 || C <= 0 || H < 2 || W < 2 || (H & 1) || (W & 1)) return -2;
  if (Cin != 16 || H != 18 || W != 18 || C % 16) return -3;
  if (N == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  // (3 images a block: 243 of 256 lanes busy; below 2048 images, one: more blocks to fill the GPU.
  // LVAE_CONV2_IPB = 1 / 2 / 3 forces one, for A/B runs)
  static const int ipb_env = getenv("LVAE_CONV2_IPB") ? atoi(getenv("LVAE_CONV2_IPB")) : 0;
  const int ipb = ipb_env >= 1 && ipb_env <= 3 ? ipb_env : N >= 2048 ? 3 : 1;
  if (ipb == 3)
    conv3x3_relu_pool_fwd_kernel<16, 18, 3><<<cdiv(N, 3), 256, 0, st>>>(x, w, bias, N, C, y, idx);
  else if (ipb == 2)
    conv3x3_relu_pool_fwd_kernel<16, 18, 2><<<cdiv(N, 2), 256, 0, st>>>(x, w, bias, N, C, y, idx);
  else
    conv3x3_relu_pool_fwd_kernel<16, 18, 1><<<N, 256, 0, st>>>(x, w, bias, N, C, y, idx);
  LVAE_CHECK_LAUNCH();
  return 0;
}

// The fused first decoder transposed conv: Cin 32, Cout 16, Hi = Wi = 9, kernel 4, stride 2, padding 1 (-3 otherwise)
int lvae_deconv4s2_relu_fwd_f32(const float* x, const float* w, const float* bias, int N, int Cin, int Cout, int Hi,
                                int Wi, float* y, void* stream) {
  if (!x || !w || !bias || !y) return -1;
  if (N < 0 || Cin <= 0 || Cout <= 0 || Hi <= 0 || Wi <= 0) return -2;
  if (Cin != 32 || Cout != 16 || Hi != 9 || Wi != 9) return -3;
  if (N == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  static const int ipb_env = getenv("LVAE_DECONV_IPB") ? atoi(getenv("LVAE_DECONV_IPB")) : 0;  // (A/B runs)
  const int ipb = ipb_env >= 1 && ipb_env <= 3 ? ipb_env : N >= 2048 ? 3 : 1;
  if (ipb == 3)
    deconv4s2_relu_fwd_kernel<32, 16, 9, 3><<<cdiv(N, 3), 256, 0, st>>>(x, w, bias, N, y);
  else if (ipb == 2)
    deconv4s2_relu_fwd_kernel<32, 16, 9, 2><<<cdiv(N, 2), 256, 0, st>>>(x, w, bias, N, y);
  else
    deconv4s2_relu_fwd_kernel<32, 16, 9, 1><<<N, 256, 0, st>>>(x, w, bias, N, y);
  LVAE_CHECK_LAUNCH();
  return 0;
}

// images per block of the backward (a multiple of its 2 images in LDS): 8 at 4096+ images (512 blocks, 2 per CU),
// fewer below so that the grid still covers the GPU
static int deconv4s2_per(int N) { return N >= 4096 ? 8 : N >= 2048 ? 4 : 2; }

size_t lvae_deconv4s2_relu_bwd_workspace_size(int N, int Cin, int Cout) {
  if (N <= 0 || Cin <= 0 || Cout <= 0) return 0;
  return sizeof(float) * 2 * (size_t)cdiv(N, deconv4s2_per(N)) * ((size_t)Cin * Cout * 16 + Cout);
}

int lvae_deconv4s2_relu_bwd_f32(const float* gy, const float* y, const float* x, const float* w, int N, int Cin,
                                int Cout, int Hi, int Wi, float* dx, float* dw, float* db, void* workspace,
                                void* stream) {
  if (!gy || !y || !x || !w || !dx || !dw || !db || !workspace) return -1;
  if (N < 0 || Cin <= 0 || Cout <= 0 || Hi <= 0 || Wi <= 0) return -2;
  if (Cin != 32 || Cout != 16 || Hi != 9 || Wi != 9) return -3;
  hipStream_t st = (hipStream_t)stream;
  if (N == 0) {
    (void)zero_async(dw, sizeof(float) * Cin * Cout * 16, st);
    (void)zero_async(db, sizeof(float) * Cout, st);
    return 0;
  }
  const int per = deconv4s2_per(N), nb = (int)cdiv(N, per), m = Cin * Cout * 16 + Cout;
  float* part = (float*)workspace;
  // LVAE_DECONV_MFMA=0: the VALU form (deconv4s2_relu_bwd_kernel, two partial rows per block)
  static const bool mfma = !getenv("LVAE_DECONV_MFMA") || atoi(getenv("LVAE_DECONV_MFMA")) != 0;
  if (mfma) {
    deconv4s2_relu_bwd_mfma_kernel<<<nb, 256, 0, st>>>(gy, y, x, w, N, per, dx, part);
    wgrad_sum_kernel<<<cdiv(m, 64), 256, 0, st>>>(part, nb, m, Cin * Cout * 16, dw, db);
  } else {
    deconv4s2_relu_bwd_kernel<32, 16, 9, 2><<<nb, 256, 0, st>>>(gy, y, x, w, N, per, dx, part);
    wgrad_sum_kernel<<<cdiv(m, 64), 256, 0, st>>>(part, 2 * nb, m, Cin * Cout * 16, dw, db);
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
