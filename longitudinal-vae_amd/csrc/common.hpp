// common.hpp -- shared device helpers for the lvae_hip library (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lvae_hip.h"

#define LVAE_CHECK_LAUNCH()                                   \
  do {                                                        \
    if (hipGetLastError() != hipSuccess) return LVAE_ERR_LAUNCH; \
  } while (0)

#define LVAE_TRY(expr)            \
  do {                            \
    int _rc = (expr);             \
    if (_rc != 0) return _rc;     \
  } while (0)

namespace lvae {

constexpr int kWave = 64;

inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }
inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// Zero `bytes` bytes at p (4-byte aligned) on st with a kernel.  The library never calls hipMemsetAsync: a memset
// captured into a HIP graph by stream capture was found not to zero its target on the replays after the first
// (ROCm 7.0 runtime; scripts/dp_replay_diag.py: the natural-gradient update's info array kept stale bytes in
// the data-parallel step's second graph), while kernel nodes replay exactly.
static __global__ __launch_bounds__(256) void lvae_zero_kernel(uint32_t* __restrict__ p, int64_t words,
                                                               uint8_t* __restrict__ tail, int ntail) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e < words) p[e] = 0u;
  if (e < ntail) tail[e] = 0;
}
// dst[0..words) = src[0..words) (4-byte words): small device-to-device copies as a kernel node, like zero_async
static __global__ __launch_bounds__(256) void lvae_copy_words_kernel(uint32_t* __restrict__ dst,
                                                                     const uint32_t* __restrict__ src, int64_t words) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e < words) dst[e] = src[e];
}
static inline int copy_words_async(void* dst, const void* src, size_t bytes, hipStream_t st) {
  const int64_t words = (int64_t)(bytes / 4);
  if (words <= 0) return 0;
  lvae_copy_words_kernel<<<(unsigned)((words + 255) / 256), 256, 0, st>>>((uint32_t*)dst, (const uint32_t*)src, words);
  return hipGetLastError() == hipSuccess ? 0 : LVAE_ERR_LAUNCH;
}
static inline int zero_async(void* p, size_t bytes, hipStream_t st) {
  if (!p || !bytes) return 0;
  const int64_t words = (int64_t)(bytes / 4);
  const int ntail = (int)(bytes & 3);
  const int64_t n = words > ntail ? words : ntail;
  lvae_zero_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>((uint32_t*)p, words, (uint8_t*)p + 4 * words, ntail);
  return hipGetLastError() == hipSuccess ? 0 : LVAE_ERR_LAUNCH;
}

// Split scale of the fp32-accurate f16 GEMMs (mfma_x3.hpp, x3_dma.hpp): x sc = hi + lo in fp16.
// The power of two 2^floor(log2(2^14 / bound)), clamped to [2^-40, 2^40] (bound 0 or inf / NaN ->
// 1): every |x| <= bound splits without overflow, and the largest entries keep 2^13..2^14 -- the
// split is then accurate to ~2^-22 of max|x| whatever the magnitude of the operand.
__device__ inline float x3_scale(float bound) {
  if (!(bound > 0.0f) || !(bound < 3.0e38f)) return 1.0f;
  int e;
  (void)frexpf(bound, &e);  // bound in [2^(e-1), 2^e)
  e = 14 - e;
  e = e < -40 ? -40 : (e > 40 ? 40 : e);
  return ldexpf(1.0f, e);
}

// ------------------------------------------------------------------------------------------
// wave / block reductions (wave64)
// ------------------------------------------------------------------------------------------
__device__ inline double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ inline float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// sum over a block of NT threads; red must hold NT/64 doubles; result valid in all threads.
template <int NT>
__device__ inline double block_sum(double v, double* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) s += red[i];
  return s;
}

// ------------------------------------------------------------------------------------------
// Additive kernel evaluation.  Templates on the maximum component / factor counts keep every
// accumulator slot compile-time indexed (runtime-indexed register arrays spill to scratch).
// ------------------------------------------------------------------------------------------
struct DevSpec {
  int32_t n_comp, n_params;
  int32_t n_fac[LVAE_MAX_COMP];
  int32_t scale_idx[LVAE_MAX_COMP];
  int32_t kind[LVAE_MAX_COMP][LVAE_MAX_FAC];
  int32_t dim[LVAE_MAX_COMP][LVAE_MAX_FAC];
  int32_t param_idx[LVAE_MAX_COMP][LVAE_MAX_FAC];
};

inline DevSpec to_dev(const lvae_kernel_spec* s) {
  DevSpec d;
  static_assert(sizeof(DevSpec) == sizeof(lvae_kernel_spec), "spec layout");
  __builtin_memcpy(&d, s, sizeof(d));
  return d;
}

// smallest template bucket that holds the spec; returns 0 if the spec is out of range.
inline int spec_bucket(const lvae_kernel_spec* s) {
  if (s->n_comp < 0 || s->n_comp > LVAE_MAX_COMP || s->n_params > 64) return 0;
  int maxf = 0;
  for (int r = 0; r < s->n_comp; ++r) {
    if (s->n_fac[r] < 1 || s->n_fac[r] > LVAE_MAX_FAC) return 0;
    maxf = s->n_fac[r] > maxf ? s->n_fac[r] : maxf;
  }
  if (s->n_comp <= 8 && maxf <= 2) return 1;
  return 2;
}

// One kernel evaluation k(xi, xj) for latent dim parameters p[] (already in LDS / regs).
// xi, xj: covariate rows (double).  Returns sum_r s_r prod_f phi_rf.
template <int MC, int MF, typename T>
__device__ inline T kernel_eval(const DevSpec& s, const double* __restrict__ xi, const double* __restrict__ xj,
                                const T* __restrict__ p) {
  T sum = T(0);
#pragma unroll
  for (int r = 0; r < MC; ++r) {
    if (r < s.n_comp) {
    T prod = p[s.scale_idx[r]];
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      if (f < s.n_fac[r]) {
      const int d = s.dim[r][f];
      const double a = xi[d], b = xj[d];
      switch (s.kind[r][f]) {
        case LVAE_CAT: prod = (a - b == 0.0) ? prod : T(0); break;
        case LVAE_BIN: prod = (a + b == 2.0) ? prod : T(0); break;
        case LVAE_RBF: {
          const T diff = T(a - b), ell = p[s.param_idx[r][f]];
          prod *= exp(-(diff * diff) / (T(2) * ell * ell));
          break;
        }
        case LVAE_PER: {
          const T ad = T(fabs(a - b)), ell = p[s.param_idx[r][f]], per = p[s.param_idx[r][f] + 1];
          const T sn = sin(T(M_PI) * ad / per);
          prod *= exp(T(-2) * sn * sn / (ell * ell));
          break;
        }
        default: prod *= T(a * b); break;  // LVAE_LIN
      }
      }
    }
    sum += prod;
    }
  }
  return sum;
}

// Accumulate g * d k(xi,xj) / d p into per-(component, factor) slots:
//   acc_s[r]      += g * d/d scale_r
//   acc_f[r][f][0] += g * d/d first param of factor f (lengthscale), [1] the period (PER)
template <int MC, int MF, typename T, typename A>
__device__ inline void kernel_grad_acc(const DevSpec& s, const double* __restrict__ xi,
                                       const double* __restrict__ xj, const T* __restrict__ p, T g,
                                       A (&acc_s)[MC], A (&acc_f)[MC][MF][2]) {
#pragma unroll
  for (int r = 0; r < MC; ++r) {
    if (r < s.n_comp) {
    T prod = T(1);
    T dlog[MF][2];
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      dlog[f][0] = T(0);
      dlog[f][1] = T(0);
      if (f >= s.n_fac[r]) continue;
      const int d = s.dim[r][f];
      const double a = xi[d], b = xj[d];
      switch (s.kind[r][f]) {
        case LVAE_CAT: prod = (a - b == 0.0) ? prod : T(0); break;
        case LVAE_BIN: prod = (a + b == 2.0) ? prod : T(0); break;
        case LVAE_RBF: {
          const T diff = T(a - b), ell = p[s.param_idx[r][f]];
          const T d2 = diff * diff;
          prod *= exp(-d2 / (T(2) * ell * ell));
          dlog[f][0] = d2 / (ell * ell * ell);
          break;
        }
        case LVAE_PER: {
          const T ad = T(fabs(a - b)), ell = p[s.param_idx[r][f]], per = p[s.param_idx[r][f] + 1];
          const T u = T(M_PI) * ad / per;
          const T sn = sin(u);
          prod *= exp(T(-2) * sn * sn / (ell * ell));
          dlog[f][0] = T(4) * sn * sn / (ell * ell * ell);
          dlog[f][1] = T(2) * T(M_PI) * ad * sin(T(2) * u) / (ell * ell * per * per);
          break;
        }
        default: prod *= T(a * b); break;
      }
    }
    const T gp = g * prod;  // g * d k / d scale_r
    acc_s[r] += A(gp);
    const T gc = gp * p[s.scale_idx[r]];
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      acc_f[r][f][0] += A(gc * dlog[f][0]);
      acc_f[r][f][1] += A(gc * dlog[f][1]);
    }
    }
  }
}

// Map the per-slot accumulators to parameter indices: out[p] for p < n_params.
// Called by one thread per (reduced) slot set; slots are summed by the caller first.
template <int MC, int MF>
__device__ inline int slot_param(const DevSpec& s, int slot) {
  // slot layout: [0, MC) scales; then MC + (r*MF + f)*2 + j
  if (slot < MC) return slot < s.n_comp ? s.scale_idx[slot] : -1;
  const int q = slot - MC, r = q / (MF * 2), f = (q / 2) % MF, j = q & 1;
  if (r >= s.n_comp || f >= s.n_fac[r]) return -1;
  const int k = s.kind[r][f];
  if (k == LVAE_RBF && j == 0) return s.param_idx[r][f];
  if (k == LVAE_PER) return s.param_idx[r][f] + j;
  return -1;
}

}  // namespace lvae
