// kl_refine.hip -- fp64 refinement of diag(K^-1) for ill-conditioned latent dims of the exact KL.
//
// The reference inverts K with an fp64 cholesky_solve(I) (elbo_functions.py:27-31); its diagonal feeds
// the trace term tr(K^-1 V) of the KL and d kl / d log v = (v diag K^-1 - 1) / 2.  The Cholesky inverse
// X of chol_inv.hip is fp32-grade: diag X carries ~cond(K) 2^-24 relative error.  One Newton step on
// the inverse, X' = 2 X - X K X, squares that error (the error of X lies in K's small-eigenvalue
// directions, where K shrinks it); only the diagonal of X' is needed:
//     d'_j = 2 X_jj - sum_k X_kj (K X)_kj
// with K evaluated from the covariates in fp64, X's fp32 entries exact in fp64, and K X accumulated in
// fp64 on v_mfma_f64_16x16x4f64 -- 2 np^3 flop per refined dim, so it runs only where it is needed:
//
//   gate   est_l = (sum_r s_r + noise_l) * max_i (K^-1)_ii (the first factor bounds max_i K_ii; the fp32
//          inverse's diagonal before refinement): a cheap
//          proxy of the diagonal's error -- first order, dX_ii = -x_i^T dK x_i with |dK| ~ 2^-24 |K|.  On
//          the -m gpu suite's draws the x3 inverse's dlogv error is 0.9-3.1e-6 x est_l (headline
//          workload est <= 6.2, error <= 1.8e-5; cond 7.9e4 / noise 1e-3 draws est 47-209, error
//          1.1-3.7e-4; CPU calibration of the same draws: scripts/refine_calib.py).  Dims with est_l > tau
//          (LVAE_KL_REFINE_TAU, default 16: an unrefined dim stays below ~5e-5) are refined;
//          LVAE_KL_REFINE=0 never runs these launches, =1 refines every dim.  (The size of alpha's fp64
//          refinement step was tried first: it follows mu's spectrum, not the diagonal's error, and
//          flagged every dim of the bench's step.)
//   fill   K_l in fp64 for the flagged dims ([L, np, np], rows / columns < n; the others exit at once)
//   gemm   128 x 128 tiles of Y = K X per flagged dim, each contracted at once with the same tile of
//          X: part[l][I][j] = sum_{k in row block I} X_kj Y_kj (Y never stored; deterministic)
//   diag   d'_j = 2 d_j - sum_I part[l][I][j] in a fixed order, over kdiag
// Unflagged dims cost the gate and three launches whose workgroups read one flag and exit.
#include <stdlib.h>

#include "common.hpp"
#include "blkinv.hpp"

namespace lvae {

constexpr int kRfT = 64;      // fill tile edge
constexpr int kRfQ = 32;      // staged covariate columns (the Gram kernels' limit)
constexpr int kRgT = 128;     // gemm output tile edge
constexpr int kRgK = 32;      // k chunk
constexpr int kRgAs = kRgK + 1;   // LDS row strides (doubles)
constexpr int kRgBs = kRgT + 2;
constexpr int kRfMaxL = 256;  // latent dims the flag lists hold
constexpr int kRfFillWG = 2048, kRgGemmWG = 512;  // grid sizes (the gemm: 2 resident per CU, 68 KB LDS)

// est_l and flag_l; grid L, 256 threads.  max_i K_ii is bounded by sum_r s_r + noise_l (every factor is
// <= 1 at zero distance and every gate passes or zeroes the component): exact for kernels without Bin
// gates, conservative (a larger est) otherwise, and no kernel evaluations on the caller's stream
// A linear factor x_i[d] x_j[d] (the C5 extension) is not <= 1: its component's scale is multiplied by
// max_i x_i[d]^2, the factor's largest diagonal value (taken here from the covariates, per LIN factor).
__device__ inline double gate_block_max(double v, double* mred) {
  const int tid = threadIdx.x;
  __syncthreads();  // the previous reduction's readers are done
  mred[tid] = v;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) mred[tid] = fmax(mred[tid], mred[tid + o]);
    __syncthreads();
  }
  return mred[0];
}

__global__ __launch_bounds__(256) void kl_refine_gate_kernel(DevSpec s, const double* __restrict__ x, int ldx,
                                                             const double* __restrict__ params,
                                                             const double* __restrict__ noise,
                                                             const double* __restrict__ kdiag, int n, int np_,
                                                             int mode, double tau, double* __restrict__ est,
                                                             int* __restrict__ flag) {
  __shared__ double mred[256];
  const int l = blockIdx.x, tid = threadIdx.x;
  const double* d = kdiag + (int64_t)l * np_;
  double mx = 0.0;
  for (int i = tid; i < n; i += 256) mx = fmax(mx, d[i]);
  const double dmax = gate_block_max(mx, mred);
  double ks = noise[l];
  for (int r = 0; r < s.n_comp; ++r) {  // (uniform loops)
    double sc = params[(int64_t)l * s.n_params + s.scale_idx[r]];
    for (int f = 0; f < s.n_fac[r]; ++f) {
      if (s.kind[r][f] != LVAE_LIN) continue;
      const int dd = s.dim[r][f];
      double m2 = 0.0;
      for (int i = tid; i < n; i += 256) {
        const double xv = x[(int64_t)i * ldx + dd];
        m2 = fmax(m2, xv * xv);
      }
      sc *= gate_block_max(m2, mred);
    }
    ks += sc;
  }
  if (tid == 0) {
    const double e = ks * dmax;
    est[l] = e;
    flag[l] = mode == 1 ? 1 : (mode == 2 && e > tau ? 1 : 0);
  }
}

// the flagged dims in order into list (LDS); returns their count (every thread)
__device__ inline int refine_list(const int* __restrict__ flag, int L, int* list) {
  __shared__ int cnt;
  if (threadIdx.x == 0) {
    int c = 0;
    for (int l = 0; l < L; ++l)
      if (flag[l]) list[c++] = l;
    cnt = c;
  }
  __syncthreads();
  return cnt;
}

// K_l (fp64, + noise_l on the diagonal, rows / columns < n) for the flagged dims: a 1-D grid over the
// (flagged dim, 64-tile) items -- no items, every workgroup exits after reading the flags
template <int MC, int MF>
__global__ __launch_bounds__(256) void kl_refine_fill_kernel(DevSpec s, const double* __restrict__ x, int ldx,
                                                             int n, int np_, int L, int qs,
                                                             const double* __restrict__ params,
                                                             const double* __restrict__ noise,
                                                             const int* __restrict__ flag, double* __restrict__ K,
                                                             int r0, int cap) {
  __shared__ int list[kRfMaxL];
  __shared__ double sx1[kRfT * kRfQ];
  __shared__ double sx2[kRfT * kRfQ];
  __shared__ double sp[64];
  const int cnt = min(max(refine_list(flag, L, list) - r0, 0), cap);  // this round's flagged dims
  const int tid = threadIdx.x, ntf = (n + kRfT - 1) / kRfT, per = ntf * ntf;
  for (int it = blockIdx.x; it < cnt * per; it += gridDim.x) {
    const int slot = it / per, l = list[r0 + slot], t = it % per, i0 = (t / ntf) * kRfT, j0 = (t % ntf) * kRfT;
    __syncthreads();  // the previous item's LDS readers are done
    if (tid < s.n_params) sp[tid] = params[(int64_t)l * s.n_params + tid];
    for (int e = tid; e < kRfT * qs; e += 256) {
      const int r = e / qs, q = e % qs;
      sx1[r * kRfQ + q] = (i0 + r < n) ? x[(int64_t)(i0 + r) * ldx + q] : 0.0;
      sx2[r * kRfQ + q] = (j0 + r < n) ? x[(int64_t)(j0 + r) * ldx + q] : 0.0;
    }
    __syncthreads();
    const int jj = tid & 63, j = j0 + jj;
    const double nz = noise[l];
    double* o = K + (int64_t)slot * np_ * np_;
#pragma unroll 4
    for (int k = 0; k < kRfT / 4; ++k) {
      const int ii = (tid >> 6) + 4 * k, i = i0 + ii;
      if (i >= n || j >= n) continue;
      double v = kernel_eval<MC, MF, double>(s, &sx1[ii * kRfQ], &sx2[jj * kRfQ], sp);
      if (i == j) v += nz;
      o[(int64_t)i * np_ + j] = v;
    }
  }
}

// X (symmetric, lower 64-tiles of the fp32 K^-1 valid) at (k, j) as fp64
__device__ inline double refine_x(const float* __restrict__ X, int np_, int k, int j) {
  return (k >> 6) >= (j >> 6) ? (double)X[(int64_t)k * np_ + j] : (double)X[(int64_t)j * np_ + k];
}

// 128 x 128 tiles of the flagged dims' Y = K X, contracted with X: a 1-D grid over the (flagged dim,
// tile) items (tiles with rows and columns < n); 4 waves, a 64 x 64 quadrant each
__global__ __launch_bounds__(256) void kl_refine_gemm_kernel(const double* __restrict__ K,
                                                             const float* __restrict__ Kinv, int n, int np_,
                                                             int L, const int* __restrict__ flag,
                                                             double* __restrict__ part, int r0, int cap) {
  __shared__ int list[kRfMaxL];
  __shared__ double As[kRgT * kRgAs];
  __shared__ double Bs[kRgK * kRgBs];
  __shared__ double red[kRgT];
  const int cnt = min(max(refine_list(flag, L, list) - r0, 0), cap);
  const int nt = np_ / kRgT, ntn = (n + kRgT - 1) / kRgT, per = ntn * ntn;
  for (int it = blockIdx.x; it < cnt * per; it += gridDim.x) {
    const int slot = it / per, l = list[r0 + slot], t = it % per;
    const int I = t / ntn, J = t % ntn;
    const int i0 = I * kRgT, j0 = J * kRgT;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wr = (w >> 1) * 64, wc = (w & 1) * 64, li = lane & 15, lk = lane >> 4;
    const double* Kl = K + (int64_t)slot * np_ * np_;
    const float* Xl = Kinv + (int64_t)l * np_ * np_;
    bi_f64x4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] = bi_f64x4{0.0, 0.0, 0.0, 0.0};
    // the next chunk's K / X values are loaded into registers while this chunk's MFMAs run
    double ra[kRgT * kRgK / 256];
    float rb[kRgK * kRgT / 256];
    auto load = [&](int k0) {
#pragma unroll
      for (int q = 0; q < kRgT * kRgK / 256; ++q) {
        const int e = tid + 256 * q, r = e >> 5, c = e & 31;
        const int i = i0 + r, k = k0 + c;
        ra[q] = (i < n && k < n) ? Kl[(int64_t)i * np_ + k] : 0.0;
      }
      // X rows k0.. k0 + 31, columns j0 + 64 h ..: a lower 64-tile row-major (lanes along j), an upper one
      // from its transpose (lanes along k: 128-byte row pieces)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const bool low = (k0 >> 6) >= ((j0 >> 6) + h);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int e = tid + 256 * q;
          const int r = low ? e >> 6 : e & 31, c = low ? e & 63 : e >> 5;
          const int k = k0 + r, j = j0 + 64 * h + c;
          rb[8 * h + q] = (k < n && j < n) ? (low ? Xl[(int64_t)k * np_ + j] : Xl[(int64_t)j * np_ + k]) : 0.0f;
        }
      }
    };
    load(0);
    for (int k0 = 0; k0 < n; k0 += kRgK) {
      __syncthreads();  // the previous chunk's readers are done
#pragma unroll
      for (int q = 0; q < kRgT * kRgK / 256; ++q) {
        const int e = tid + 256 * q;
        As[(e >> 5) * kRgAs + (e & 31)] = ra[q];
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const bool low = (k0 >> 6) >= ((j0 >> 6) + h);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int e = tid + 256 * q;
          const int r = low ? e >> 6 : e & 31, c = low ? e & 63 : e >> 5;
          Bs[r * kRgBs + 64 * h + c] = (double)rb[8 * h + q];
        }
      }
      __syncthreads();
      if (k0 + kRgK < n) load(k0 + kRgK);
#pragma unroll 2
      for (int kk = 0; kk < kRgK; kk += 4) {
        double a[4], b[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) a[m] = As[(wr + 16 * m + li) * kRgAs + kk + lk];
#pragma unroll
        for (int m = 0; m < 4; ++m) b[m] = Bs[(kk + lk) * kRgBs + wc + 16 * m + li];
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
      }
    }
    // contraction with the same tile of X: column sums over this wave's 64 rows (accumulator row
    // (lane >> 4) + 4 r of each 16 x 16 block, column lane & 15), then over the two row halves
    double cs[4];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int j = j0 + wc + 16 * ni + li;
      double s = 0.0;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int k = i0 + wr + 16 * mi + lk + 4 * r;
          const double xv = (k < n && j < n) ? refine_x(Xl, np_, k, j) : 0.0;
          s += xv * acc[mi][ni][r];
        }
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      cs[ni] = s;
    }
    if (wr == 64 && lane < 16) {
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) red[wc + 16 * ni + li] = cs[ni];
    }
    __syncthreads();
    if (wr == 0 && lane < 16) {
      double* pr = part + ((int64_t)l * nt + I) * np_ + j0;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) pr[wc + 16 * ni + li] = cs[ni] + red[wc + 16 * ni + li];
    }
  }
}

// d'_j = 2 d_j - sum_I part[l][I][j] (fixed order); grid (np / 256, L)
__global__ __launch_bounds__(256) void kl_refine_diag_kernel(const double* __restrict__ part, int n, int np_,
                                                             const int* __restrict__ flag,
                                                             double* __restrict__ kdiag) {
  const int l = blockIdx.y, j = blockIdx.x * 256 + threadIdx.x;
  if (!flag[l] || j >= n) return;
  const int nt = np_ / kRgT, nI = (n + kRgT - 1) / kRgT;
  const double* p = part + (int64_t)l * nt * np_ + j;
  double s = 0.0;
  for (int I = 0; I < nI; ++I) s += p[(int64_t)I * np_];
  double* d = kdiag + (int64_t)l * np_ + j;
  *d = 2.0 * *d - s;
}

// read per call (a getenv each: A/B runs and tests switch them inside one process)
static int refine_mode() {
  const char* v = getenv("LVAE_KL_REFINE");
  return v ? (atoi(v) == 0 ? 0 : (atoi(v) == 1 ? 1 : 2)) : 2;
}

static double refine_tau() {
  const char* v = getenv("LVAE_KL_REFINE_TAU");
  return v ? atof(v) : 16.0;
}

// K64 holds kl_refine_cap(L) = ceil(L / 2) dims: the flagged dims go in (at most) two rounds through the caller's
// buffer -- the KL workspace lends the factor's Y^T planes (L np^2 fp16 pairs, dead after lauum until the backward
// writes S there) plus np^2 floats for odd L, instead of a dedicated L np^2 fp64 buffer
int kl_refine_cap(int L) { return (L + 1) / 2; }
size_t kl_refine_bytes(int np_, int L) { return (size_t)kl_refine_cap(L) * np_ * np_ * sizeof(double); }

size_t kl_refine_part_bytes(int np_, int L) { return (size_t)L * (np_ / kRgT) * np_ * sizeof(double); }

// the gate alone: est, flag from kdiag (mode 0: both zero)
int kl_refine_gate(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int np_, int L, const double* params,
                   const double* noise, const double* kdiag, double* est, int* flag, hipStream_t st) {
  const int mode = refine_mode();
  if (mode == 0) {  // off: only the state lvae_kl_closed_refine_state reports
    if (zero_async(est, (size_t)L * sizeof(double), st) != 0 ||
        zero_async(flag, (size_t)L * sizeof(int), st) != 0)
      return LVAE_ERR_LAUNCH;
    return 0;
  }
  if (!spec_bucket(spec) || L > kRfMaxL) return -1;
  kl_refine_gate_kernel<<<L, 256, 0, st>>>(to_dev(spec), x, ldx, params, noise, kdiag, n, np_, mode, refine_tau(), est,
                                           flag);
  LVAE_CHECK_LAUNCH();
  return 0;
}

// the refinement of the flagged dims' diag K^-1 (kdiag) from the fp32 K^-1 in Kinv (the gate ran before)
int kl_refine_apply(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int np_, int L, const double* params,
                    const double* noise, const float* Kinv, double* kdiag, double* K64, double* part, const int* flag,
                    hipStream_t st) {
  if (refine_mode() == 0) return 0;
  const int bucket = spec_bucket(spec);
  int qs = 0;
  for (int r = 0; r < spec->n_comp; ++r)
    for (int f = 0; f < spec->n_fac[r]; ++f) qs = spec->dim[r][f] + 1 > qs ? spec->dim[r][f] + 1 : qs;
  if (!bucket || qs > kRfQ || qs > ldx || np_ % kRgT || L > kRfMaxL) return -1;
  const DevSpec ds = to_dev(spec);
  const int cap = kl_refine_cap(L);
  for (int r0 = 0; r0 < L; r0 += cap) {  // (rounds with no flagged dims: launches that read the flags and exit)
    if (bucket == 1)
      kl_refine_fill_kernel<8, 2><<<kRfFillWG, 256, 0, st>>>(ds, x, ldx, n, np_, L, qs, params, noise, flag, K64,
                                                             r0, cap);
    else
      kl_refine_fill_kernel<16, 4><<<kRfFillWG, 256, 0, st>>>(ds, x, ldx, n, np_, L, qs, params, noise, flag, K64,
                                                              r0, cap);
    kl_refine_gemm_kernel<<<kRgGemmWG, 256, 0, st>>>(K64, Kinv, n, np_, L, flag, part, r0, cap);
  }
  kl_refine_diag_kernel<<<dim3(np_ / 256, L), 256, 0, st>>>(part, n, np_, flag, kdiag);
  LVAE_CHECK_LAUNCH();
  return 0;
}

int kl_refine_diag(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int np_, int L,
                   const double* params, const double* noise, const float* Kinv, double* kdiag, double* K64,
                   double* part, double* est, int* flag, hipStream_t st) {
  LVAE_TRY(kl_refine_gate(spec, x, ldx, n, np_, L, params, noise, kdiag, est, flag, st));
  return kl_refine_apply(spec, x, ldx, n, np_, L, params, noise, Kinv, kdiag, K64, part, flag, st);
}

}  // namespace lvae
