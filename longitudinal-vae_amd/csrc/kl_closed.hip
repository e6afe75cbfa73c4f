// kl_closed.hip -- exact GP-prior KL of the Longitudinal-VAE (elbo_functions.py:8-34), forward and
// analytic backward, batched over the L latent dims (replaces the Python loop at training.py:515-522).
//
// factor (needs only the covariates and hyper-parameters: launched before the encoder has run):
//   K_l = Gram_l(x, x) + noise_l I                (kl_gram_fill, f32, padded to np; table / fp32 / fp64
//                                                   covariate paths chosen on the device, gram.hip)
//   Y = L^-1, log|K|                               (ci_factor_f32: blocked Cholesky + trtri, f16 x3 MFMA,
//                                                   chol_inv.hip)
//   the binned residual's plan                     (kl_resid_bins_plan, on the side stream behind the
//                                                   pivot chain; integer-coded covariates only)
// reduce (needs mu, log v), early form (the default for L > 2 dims per call, kl_early):
//   a0 = Y^T (Y mu), d = diag K^-1                 (kl_ymv_kernel: triangular mat-vecs over the Y / Y^T planes,
//                                                   d = the row sums of squares of Y^T; no K^-1)
//   r = mu - K a0, a = a0 + Y^T (Y r)              (fp64 residual as below, then two more mat-vecs)
//   the refinement gate on d; the flagged dims' K^-1 alone + their fp64 diag; kl_l
//   -> lauum (K^-1 = Y^T Y, B planes) runs in the backward's hyper-parameter half, after d kl / d (mu, log v)
// reduce, K^-1 form (pipelined factors, L <= 2: K^-1 is accumulated in the factor; LVAE_KL_EARLY=0):
//   K^-1 = Y^T Y, the partials of a0 = K^-1 mu,    (ci_lauum_f32 with the KL epilogue: one pass over the
//   and B = K^-1 diag(sqrt v) as fp16 hi / lo       K^-1 tiles while they are in registers; B only when a
//   planes, one power-of-two scale per dim          backward follows)
//   a0, d = diag K^-1                              (kl_alpha0_kernel: fixed-order sum of the partials)
//   r = mu - K a0                                  (kl_gram_resid: fp64 Gram-free residual, binned
//                                                   O(N W) (kl_resid_bins.hip) or tiled O(N^2), gram.hip)
//   a = a0 + K^-1 r                                (kl_alpha_sym_kernel over the lower tiles of K^-1, f64
//                                                   accumulation: one step of iterative refinement)
//   kl_l = 1/2 (sum v d + mu.a - n + logdet - sum log v)
// backward (dL/dkl_l = g_l):
//   S = K^-1 V K^-1 = B B^T                        (syrk_tiles_f32, f16 x3 MFMA, lower tiles; K^-1 itself
//                                                   is kept as its lower tiles only)
//   G = 1/2 (K^-1 - S - a a^T) -> dtheta, dnoise   (kl_gram_bwd, fused, never materialised)
//   dmu = g a,  dlogv = g/2 (v d - 1)
// One reduce per factor: the backward's S overwrites the Y^T planes.
#include "common.hpp"
#include "side_stream.hpp"
#include "prof.hpp"
#include "x3_c16.hpp"  // c16_off: the chunk-major Y / Y^T planes

#include <atomic>


#ifndef LVAE_ALPHA_WG
#define LVAE_ALPHA_WG 4096
#endif

namespace lvae {

int kl_gram_fill(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int np_, int L,
                 const double* params, const double* noise, float* K, int* covflag, hipStream_t st);
size_t kl_gram_bwd_partials_bytes(int np_, int L);
int kl_gram_bwd(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int np_, int L,
                const double* params, const float* Kinv, const float* S, const float* Sx, int nsplit,
                const double* alpha, const double* kdiag, const float* v, const double* gkl, double* part,
                double* dparams, double* dnoise, const int* covflag, void* hbws, const int* hbon, hipStream_t st);
int syrk_x3_splits(int np_, int L);
int syrk_tiles_f32(int np_, int L, const float* bsc, const _Float16* planes, float* S, float* Sx, hipStream_t st,
                   const int* skip);
size_t kl_hyper_bytes(int np_, int L);
struct HbDev;
HbDev* kl_hyper_dev(void* base, int np_, int L);
int kl_hyper_plan(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int np_, int L, void* wsbase,
                  const int* covflag, hipStream_t st);
int ci_factor_f32(int np_, int L, float* A, void* scratch, _Float16* YT, float* Kinv, double* logdet,
                  int32_t* info, hipStream_t st, float* lout = nullptr);
int ci_lauum_f32(int np_, int L, void* scratch, const _Float16* YT, float* Kinv, const double* mu, const float* sv,
                 float* apart, _Float16* Bh, float* bsc, hipStream_t st, const int* hbon);
size_t ci_scratch_bytes(int np_, int L);
size_t kl_resid_partials_bytes(int np_, int L);
int kl_gram_resid(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int np_, int L,
                  const double* params, const double* noise, const double* alpha0, const double* muc, double* part,
                  double* res, void* rbws, hipStream_t st);
size_t kl_resid_bins_bytes(int np_, int L, int ncomp);
bool kl_resid_bins_enabled(const lvae_kernel_spec* spec, int n);
int kl_resid_bins_plan(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int np_, int L, void* wsbuf,
                       hipStream_t st);
size_t kl_refine_bytes(int np_, int L);
int kl_refine_gate(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int np_, int L, const double* params,
                   const double* noise, const double* kdiag, double* est, int* flag, hipStream_t st);
int kl_refine_apply(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int np_, int L, const double* params,
                    const double* noise, const float* Kinv, double* kdiag, double* K64, double* part, const int* flag,
                    hipStream_t st);
int ci_lauum_flagged_f32(int np_, int L, void* scratch, const _Float16* YT, float* Kinv, const int* flag, hipStream_t st);
const float* ci_ysc_ptr(void* scratch, int np_, int L);
int ci_pipe_mode_of(int np_, int L);
size_t kl_refine_part_bytes(int np_, int L);
int kl_refine_diag(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int np_, int L,
                   const double* params, const double* noise, const float* Kinv, double* kdiag, double* K64,
                   double* part, double* est, int* flag, hipStream_t st);

struct KLWorkspace {
  float *A, *Kinv, *v, *sv;
  float* Sx;         // K-split partials 1.. of the S GEMM (syrk_x3_splits(np, L) - 1 matrices; few dims only)
  _Float16* planes;  // 2 L np^2 halves: the factor's Y^T planes, then (backward) S = K^-1 V K^-1 in fp32
  _Float16* Bp;      // the planes of B = K^-1 diag(sqrt v) (reduce -> backward): = A, dead after trtri
  float* bsc;        // [L] their split scale per dim
  float* apart;      // [L, nt, np] the partials of K^-1 mu (lauum epilogue)
  char* chol;        // ci_factor_f32 scratch
  double *mu, *alpha, *res, *kdiag, *logdet, *part, *rpart;
  int* covflag;      // 1: integer covariates (the Gram kernels' fp32 covariate path; set by the factor)
  char* rb;          // the binned residual's plan / bin sums (kl_resid_bins.hip)
  double* K64;       // [ceil(L / 2), np, np] fp64 K of the dims whose diag K^-1 is refined (kl_refine.hip), two
                     // rounds: = the Y^T planes (dead between lauum and the backward's S) + np^2 floats for odd L
  char* hb;          // the binned hyper-gradient's plan, point bins / runs and slab partials (kl_hyper.hip)
  const int* hbon;   // its device flag: on -> the lauum writes K^-1's mirror, the S GEMM and the table adjoint exit
  double* rest;      // [L] the refinement gate's estimate (sum_r s_r + noise) max (K^-1)_ii
  int* rflag;        // [L] 1: diag K^-1 refined
  double* ypart;     // early reduce: [2][L][nt][np] fp64 partials of the triangular mat-vecs over the Y planes
  double* yvec;      // early reduce: [L][np] t = Y mu, then u = Y r
  double* K64e;      // early reduce: the refinement's fp64 K (the Y^T planes are still needed by the late lauum)
  size_t bytes, bytes_base;
  KLWorkspace(char* base, int np_, int L) {
    size_t off = 0;
    auto take = [&](size_t b) {
      char* p = base ? base + off : nullptr;
      off += align256(b);
      return p;
    };
    const size_t mat = (size_t)L * np_ * np_ * sizeof(float);
    A = (float*)take(mat);
    Bp = reinterpret_cast<_Float16*>(A);
    Kinv = (float*)take(mat);
    planes = (_Float16*)take(mat);
    K64 = reinterpret_cast<double*>(planes);
    take(kl_refine_bytes(np_, L) - mat);  // (odd L: the second half of the last K64 slot, right after the planes)
    v = (float*)take((size_t)L * np_ * sizeof(float));
    sv = (float*)take((size_t)L * np_ * sizeof(float));
    bsc = (float*)take((size_t)L * sizeof(float));
    apart = (float*)take((size_t)L * (np_ / 256) * np_ * sizeof(float));  // nt = np / 256 slots
    mu = (double*)take((size_t)L * np_ * sizeof(double));
    alpha = (double*)take((size_t)L * np_ * sizeof(double));
    res = (double*)take((size_t)L * np_ * sizeof(double));
    kdiag = (double*)take((size_t)L * np_ * sizeof(double));
    logdet = (double*)take((size_t)L * sizeof(double));
    chol = take(ci_scratch_bytes(np_, L));
    part = (double*)take(kl_gram_bwd_partials_bytes(np_, L));
    rpart = (double*)take(kl_resid_partials_bytes(np_, L));
    covflag = (int*)take(sizeof(int));
    rb = take(kl_resid_bins_bytes(np_, L, LVAE_MAX_COMP));
    Sx = (float*)take(mat * (size_t)(syrk_x3_splits(np_, L) - 1));
    hb = take(kl_hyper_bytes(np_, L));
    hbon = base ? reinterpret_cast<const int*>(kl_hyper_dev(hb, np_, L)) : nullptr;  // (HbDev::on: its first member)
    rest = (double*)take((size_t)L * sizeof(double));
    rflag = (int*)take((size_t)L * sizeof(int));
    bytes_base = off;  // (the early reduce's buffers below: sized only when it is on, lvae_kl_closed_workspace_size)
    ypart = (double*)take(2 * (size_t)L * (np_ / 256) * np_ * sizeof(double));
    yvec = (double*)take((size_t)L * np_ * sizeof(double));
    K64e = (double*)take(kl_refine_bytes(np_, L));
    bytes = off;
  }
};

// mu / v / sqrt v into contiguous per-dim vectors (zero on the padding)
__global__ void kl_prep_kernel(const double* __restrict__ mu, const double* __restrict__ logv, int ld, int n, int np_,
                               int L, double* __restrict__ muc, float* __restrict__ v, float* __restrict__ sv) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x, l = blockIdx.y;
  if (i >= np_) return;
  const bool in = i < n;
  muc[(int64_t)l * np_ + i] = in ? mu[(int64_t)i * ld + l] : 0.0;
  const double vv = in ? exp(logv[(int64_t)i * ld + l]) : 0.0;
  v[(int64_t)l * np_ + i] = (float)vv;
  sv[(int64_t)l * np_ + i] = (float)sqrt(vv);
}

// a0 = sum_s apart[l][s] (fixed order, fp64) and d = diag K^-1; grid (np / 256, L)
__global__ __launch_bounds__(256) void kl_alpha0_kernel(const float* __restrict__ apart, const float* __restrict__ Kinv,
                                                        int np_, double* __restrict__ alpha,
                                                        double* __restrict__ kdiag) {
  const int l = blockIdx.y, nt = np_ / 256;
  const int p = blockIdx.x * 256 + threadIdx.x;
  const float* ap = apart + (int64_t)l * nt * np_ + p;
  double s = 0.0;
  for (int q = 0; q < nt; ++q) s += (double)ap[(int64_t)q * np_];
  const int64_t o = (int64_t)l * np_ + p;
  alpha[o] = s;
  kdiag[o] = (double)Kinv[(int64_t)l * np_ * np_ + (int64_t)p * np_ + p];
}

// alpha = base + K^-1 u (one wave per row, fp64 accumulation of the fp32 K^-1 row times the fp64 u)
__global__ __launch_bounds__(256) void kl_alpha_kernel(const float* __restrict__ Kinv, const double* __restrict__ u,
                                                       int np_, const double* base, double* alpha) {
  const int l = blockIdx.y, lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= np_) return;
  const float* row = Kinv + (int64_t)l * np_ * np_ + (int64_t)i * np_;
  const double* m = u + (int64_t)l * np_;
  double acc = 0.0;
  for (int j = lane * 4; j < np_; j += 256) {
    const float4 k4 = *reinterpret_cast<const float4*>(row + j);
    acc += (double)k4.x * m[j] + (double)k4.y * m[j + 1] + (double)k4.z * m[j + 2] + (double)k4.w * m[j + 3];
  }
  acc = wave_sum(acc);
  if (lane == 0) {
    const int64_t o = (int64_t)l * np_ + i;
    alpha[o] = base[o] + acc;
  }
}

// The same product over the lower 64-tiles only (K^-1 is symmetric; half the bytes): tile (I, J), I >= J,
// gives its row sums K_IJ u_J to rows of block I and, off the diagonal, its column sums K_IJ^T u_I to rows
// of block J, each written once to part[l][other block][row]; kl_alpha_reduce adds them in a fixed order
// (deterministic).  Grid (G, L), the tiles t = g, g + G, ...; thread (tr, tc) reads rows 4 tr + a,
// columns 4 tc .. 4 tc + 3 (float4: 16 lanes per 256-byte row segment).
__device__ inline void alpha_tri_index(int t, int& I, int& J) {
  int r = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
  while ((r + 1) * (r + 2) / 2 <= t) ++r;
  while (r * (r + 1) / 2 > t) --r;
  I = r;
  J = t - r * (r + 1) / 2;
}
__global__ __launch_bounds__(256) void kl_alpha_sym_kernel(const float* __restrict__ Kinv,
                                                           const double* __restrict__ u, int np_,
                                                           double* __restrict__ part, int ntiles) {
  __shared__ double cred[4][64];
  const int G = gridDim.x, l = blockIdx.y, tid = threadIdx.x, tr = tid >> 4, tc = tid & 15, wv = tid >> 6;
  const int nt = np_ / 64;
  const float* K = Kinv + (int64_t)l * np_ * np_;
  const double* ul = u + (int64_t)l * np_;
  for (int t = blockIdx.x; t < ntiles; t += G) {
    int I, J;
    alpha_tri_index(t, I, J);
    const int i0 = I * 64, j0 = J * 64;
    float4 k[4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
      k[a] = *reinterpret_cast<const float4*>(K + (int64_t)(i0 + 4 * tr + a) * np_ + j0 + 4 * tc);
    double uj[4], ui[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) uj[c] = ul[j0 + 4 * tc + c];
#pragma unroll
    for (int a = 0; a < 4; ++a) ui[a] = ul[i0 + 4 * tr + a];
    double rs[4], cs[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      rs[a] = (double)k[a].x * uj[0] + (double)k[a].y * uj[1] + (double)k[a].z * uj[2] + (double)k[a].w * uj[3];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) rs[a] += __shfl_xor(rs[a], o, 64);
    }
    if (tc == 0) {
      double* pr = part + ((int64_t)l * nt + J) * np_ + i0 + 4 * tr;
#pragma unroll
      for (int a = 0; a < 4; ++a) pr[a] = rs[a];
    }
    if (I != J) {  // (uniform)
      cs[0] = (double)k[0].x * ui[0] + (double)k[1].x * ui[1] + (double)k[2].x * ui[2] + (double)k[3].x * ui[3];
      cs[1] = (double)k[0].y * ui[0] + (double)k[1].y * ui[1] + (double)k[2].y * ui[2] + (double)k[3].y * ui[3];
      cs[2] = (double)k[0].z * ui[0] + (double)k[1].z * ui[1] + (double)k[2].z * ui[2] + (double)k[3].z * ui[3];
      cs[3] = (double)k[0].w * ui[0] + (double)k[1].w * ui[1] + (double)k[2].w * ui[2] + (double)k[3].w * ui[3];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        cs[c] += __shfl_xor(cs[c], 16, 64);
        cs[c] += __shfl_xor(cs[c], 32, 64);
      }
      __syncthreads();  // the previous tile's readers of cred are done
      if ((tid & 63) < 16) {
#pragma unroll
        for (int c = 0; c < 4; ++c) cred[wv][4 * tc + c] = cs[c];
      }
      __syncthreads();
      if (tid < 64)
        part[((int64_t)l * nt + I) * np_ + j0 + tid] = ((cred[0][tid] + cred[1][tid]) + cred[2][tid]) + cred[3][tid];
    }
  }
}

// alpha[l][i] = base[l][i] + sum_s part[l][s][i] (fixed order).  Grid (np / 256, L).
__global__ __launch_bounds__(256) void kl_alpha_reduce(const double* __restrict__ part, const double* base, int np_,
                                                       double* alpha) {
  const int i = blockIdx.x * 256 + threadIdx.x, l = blockIdx.y, nt = np_ / 64;
  if (i >= np_) return;
  double acc = 0.0;
  const double* pl = part + (int64_t)l * nt * np_ + i;
  for (int s = 0; s < nt; s += 4) {  // (nt = np / 64: a multiple of 4) loads first, adds in order
    const double v0 = pl[(int64_t)s * np_], v1 = pl[(int64_t)(s + 1) * np_];
    const double v2 = pl[(int64_t)(s + 2) * np_], v3 = pl[(int64_t)(s + 3) * np_];
    acc += v0;
    acc += v1;
    acc += v2;
    acc += v3;
  }
  const int64_t o = (int64_t)l * np_ + i;
  alpha[o] = base[o] + acc;
}

// ---- the early reduce: K^-1 mu and diag K^-1 from Y = L^-1 before lauum (K^-1 = Y^T Y) ----------------------------
// y = P x over one triangle of 256-tiles of a chunk-major plane pair (hi, lo; x3_c16.hpp): the Y planes' lower
// tiles (R, C), C <= R (UPPER false: y = Y x), or the Y^T planes' upper tiles (R, C), C >= R (y = Y^T x); the
// value of an entry is (hi + lo) / ysc(max(R, C), min(R, C)).  One 256-thread workgroup per (tile, dim), a thread
// per row of the tile: every 16-deep chunk is one contiguous 8 KB run (256 rows x 32 B per plane), each row's
// 16 halves un-swizzled (the two 8-half groups swapped when bit 3 of the row is set).  fp64 accumulation; the
// tile's row sums go to part[l][C][row] (SUMSQ: the row sums of squares to part2 -- diag K^-1 = the row sums
// of squares of Y^T), summed in a fixed order by kl_ymv_reduce.  HBM-bound: 4 B per element read once.
template <bool UPPER, bool SUMSQ>
__global__ __launch_bounds__(256) void kl_ymv_kernel(const _Float16* __restrict__ hi, const _Float16* __restrict__ lo,
                                                     const float* __restrict__ ysc, int np_, const double* __restrict__ x,
                                                     double* __restrict__ part, double* __restrict__ part2) {
  __shared__ double xs[256];
  const int l = blockIdx.y, tid = threadIdx.x, nt = np_ / 256;
  int R, C;
  alpha_tri_index(blockIdx.x, R, C);  // (R >= C)
  if (UPPER) {
    const int t = R;
    R = C;
    C = t;
  }
  xs[tid] = x[(int64_t)l * np_ + C * 256 + tid];
  const float s = ysc[((int64_t)l * nt + max(R, C)) * nt + min(R, C)];
  __syncthreads();
  const int row = R * 256 + tid;
  const bool sw = (tid >> 3) & 1;  // this row's two 8-half groups are stored swapped
  // chunk 0 of column block C, this row (c16_off's layout without the swizzle: the row's 16 halves whole)
  const int64_t base = (int64_t)l * np_ * np_ + ((int64_t)R * (np_ >> 4) + C * 16) * kC16Part + tid * 16;
  const uint4* ph = reinterpret_cast<const uint4*>(hi + base);
  const uint4* pl = reinterpret_cast<const uint4*>(lo + base);
  constexpr int kChunkU4 = kC16Part / 8;  // uint4 per chunk (8 halves each)
  double acc = 0.0, sq = 0.0;
#pragma unroll 4
  for (int c = 0; c < 16; ++c) {
    const uint4 h0 = ph[c * kChunkU4], h1 = ph[c * kChunkU4 + 1];
    const uint4 l0 = pl[c * kChunkU4], l1 = pl[c * kChunkU4 + 1];
    // un-swizzle by whole 8-half groups (selects, no runtime-indexed register arrays: those go to scratch)
    _Float16 hv[16], lv[16];
    *reinterpret_cast<uint4*>(hv) = sw ? h1 : h0;
    *reinterpret_cast<uint4*>(hv + 8) = sw ? h0 : h1;
    *reinterpret_cast<uint4*>(lv) = sw ? l1 : l0;
    *reinterpret_cast<uint4*>(lv + 8) = sw ? l0 : l1;
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      const double v = (double)((float)hv[kk] + (float)lv[kk]);
      acc += v * xs[c * 16 + kk];
      if (SUMSQ) sq += v * v;
    }
  }
  const double inv = 1.0 / (double)s;
  part[((int64_t)l * nt + C) * np_ + row] = acc * inv;
  if (SUMSQ) part2[((int64_t)l * nt + C) * np_ + row] = sq * inv * inv;
}

// out[l][i] = (base ? base[l][i] : 0) + sum over the triangle's column blocks C of part[l][C][i] (fixed order: C
// ascending); lower: C = 0 .. R, upper: C = R .. nt - 1 (R = i's row block).  Grid (np / 256, L).
template <bool UPPER>
__global__ __launch_bounds__(256) void kl_ymv_reduce(const double* __restrict__ part, const double* base, int np_,
                                                     double* out) {
  const int i = blockIdx.x * 256 + threadIdx.x, l = blockIdx.y, nt = np_ / 256, R = blockIdx.x;
  const double* p = part + (int64_t)l * nt * np_ + i;
  double acc = 0.0;
  for (int C = UPPER ? R : 0; C <= (UPPER ? nt - 1 : R); ++C) acc += p[(int64_t)C * np_];
  const int64_t o = (int64_t)l * np_ + i;
  out[o] = (base ? base[o] : 0.0) + acc;
}

__global__ __launch_bounds__(256) void kl_finalize_kernel(const double* __restrict__ muc, const double* __restrict__ logv,
                                                          int ld, const double* __restrict__ alpha,
                                                          const double* __restrict__ kdiag,
                                                          const double* __restrict__ logdet, int n, int np_,
                                                          double* __restrict__ kl) {
  __shared__ double red[4];
  const int l = blockIdx.x, tid = threadIdx.x;
  double quad = 0.0, tr = 0.0, slv = 0.0;
  for (int i = tid; i < n; i += 256) {
    const double lv = logv[(int64_t)i * ld + l];
    quad += muc[(int64_t)l * np_ + i] * alpha[(int64_t)l * np_ + i];
    tr += exp(lv) * kdiag[(int64_t)l * np_ + i];
    slv += lv;
  }
  quad = block_sum<256>(quad, red);
  tr = block_sum<256>(tr, red);
  slv = block_sum<256>(slv, red);
  if (tid == 0) kl[l] = 0.5 * (tr + quad - (double)n + logdet[l] - slv);
}

__global__ void kl_bwd_elem_kernel(const double* __restrict__ logv, int ld, int n, int np_, int L,
                                   const double* __restrict__ alpha, const double* __restrict__ kdiag,
                                   const double* __restrict__ gkl, double* __restrict__ dmu,
                                   double* __restrict__ dlogv) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)n * L) return;
  const int i = (int)(e / L), l = (int)(e % L);
  const double g = gkl[l];
  dmu[(int64_t)i * ld + l] = g * alpha[(int64_t)l * np_ + i];
  dlogv[(int64_t)i * ld + l] = 0.5 * g * (exp(logv[(int64_t)i * ld + l]) * kdiag[(int64_t)l * np_ + i] - 1.0);
}

}  // namespace lvae

using namespace lvae;

extern "C" {

int lvae_kl_closed_padded_n(int n) { return ((n + 255) / 256) * 256; }

static bool kl_early_env() {
  const char* e = getenv("LVAE_KL_EARLY");
  return e && atoi(e) != 0;
}
static std::atomic<bool> g_kl_early_sized{false};  // LVAE_KL_EARLY at the last workspace-size query

// (kl_hyper.hip's state query: where the workspace keeps the binned hyper-gradient's region)
size_t kl_hyper_offset_in_kl_ws(int np_, int L) {
  char* const fake = reinterpret_cast<char*>(uintptr_t(1) << 20);  // (offsets only: any aligned base)
  KLWorkspace ws(fake, np_, L);
  return (size_t)(ws.hb - fake);
}

size_t lvae_kl_closed_workspace_size(int n, int L) {
  const int np_ = lvae_kl_closed_padded_n(n);
  const KLWorkspace ws(nullptr, np_, L);
  // the early reduce's buffers (the workspace's tail, ~0.3-0.6 GB) only when LVAE_KL_EARLY is on at this call; the
  // decision is kept for the calls on the workspace sized here (kl_early)
  const bool early = kl_early_env();
  g_kl_early_sized.store(early);
  return early ? ws.bytes : ws.bytes_base;
}

int lvae_kl_closed_factor_f32(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int L,
                              const double* params, const double* noise, int32_t* info, void* workspace,
                              void* stream) {
  if (!spec) return -1;
  if (!x) return -2;
  if (n <= 0) return -4;
  if (L <= 0) return -5;
  if (!params) return -6;
  if (!noise) return -7;
  if (!workspace || ((uintptr_t)workspace & 255)) return -9;
  hipStream_t st = (hipStream_t)stream;
  const int np_ = lvae_kl_closed_padded_n(n);
  KLWorkspace ws((char*)workspace, np_, L);
  // the binned residual's plan (x only) goes on the side stream behind the Cholesky's pivot chain, beside
  // the trailing updates / trtri; the reduce waits for it (event rb)
  const bool rb_on = kl_resid_bins_enabled(spec, n);
  std::unique_lock<std::recursive_mutex> lock(side_mutex(), std::defer_lock);
  SideStream* sd = nullptr;
  auto ok = [](hipError_t e) { return e == hipSuccess; };
  if (rb_on) {
    lock.lock();
    LVAE_TRY(side_stream(sd));
  }
  {
    ProfScope ps(LVAE_PH_GRAM, st);
    LVAE_TRY(kl_gram_fill(spec, x, ldx, n, np_, L, params, noise, ws.A, ws.covflag, st));
  }
  // (after the fill: the side stream's plans read x and the fill's covariate flag)
  if (rb_on && !ok(hipEventRecord(sd->rbx, st))) return LVAE_ERR_LAUNCH;
  // the binned hyper-gradient's plan (covariates and the fill's covariate flag; the reduce's lauum and the
  // backward read its flag): beside trtri on the side stream with the residual's plan when that runs (behind the
  // last pivot, so after the fill), else here
  if (!rb_on) LVAE_TRY(kl_hyper_plan(spec, x, ldx, n, np_, L, ws.hb, ws.covflag, st));
  // Y = L^-1 and log|K|: blocked Cholesky + trtri (chol_inv.hip; phases POTRF / POTRI inside); lauum
  // runs in the reduce
  LVAE_TRY(ci_factor_f32(np_, L, ws.A, ws.chol, ws.planes, ws.Kinv, ws.logdet, info, st));
  if (rb_on) {
    if (!ok(hipStreamWaitEvent(sd->s, sd->rbx, 0))) return LVAE_ERR_LAUNCH;
    LVAE_TRY(kl_resid_bins_plan(spec, x, ldx, n, np_, L, ws.rb, sd->s));
    LVAE_TRY(kl_hyper_plan(spec, x, ldx, n, np_, L, ws.hb, ws.covflag, sd->s));
    if (!ok(hipEventRecord(sd->rb, sd->s))) return LVAE_ERR_LAUNCH;
    // join the side stream back before returning (the header's contract): the wait sits behind the
    // trtri launches already on `st`, so the plan still runs beside them; each call is self-contained
    // (separate graph captures, a caller that syncs `st` and frees the workspace after the factor)
    if (!ok(hipStreamWaitEvent(st, sd->rb, 0))) return LVAE_ERR_LAUNCH;
  }
  LVAE_CHECK_LAUNCH();
  return 0;
}

// The early reduce (opt-in, LVAE_KL_EARLY=1; non-pipelined factors only, L > 2 dims per call): K^-1 mu and
// diag K^-1 straight from Y = L^-1 while the Y and Y^T planes are fresh, before any lauum, so that d kl / d (mu,
// log v) -- and the encoder's backward -- need no K^-1; lauum moves into the backward's hyper-parameter half.
// Measured (r6, same box, headline step): d kl / d (mu, log v) 0.7 ms earlier, but the step 9.32-9.37 vs 9.20-9.25
// ms: the encoder backward then runs beside lauum + the slab pass, whose grids hold every CU, and the four
// mat-vec passes (~0.45 ms) add to a step that is bound by its total GPU work (profiles/r6_kl_early_ab.txt).
// The variable is read when the workspace is sized (tests compare both routes in one process) and that decision
// holds for the forward and the backward on it: the early buffers exist only in a workspace sized with it on.
static bool kl_early(int np_, int L) { return g_kl_early_sized.load() && ci_pipe_mode_of(np_, L) == 0; }

// t = Y x (lower) or a = base + Y^T x (upper, + the row sums of squares of Y^T: diag K^-1 into sumsq)
static void kl_ymv(const KLWorkspace& ws, const float* ysc, int np_, int L, bool upper, const double* x,
                   const double* base, double* out, double* sumsq, hipStream_t st) {
  const int nt = np_ / 256, ntri = nt * (nt + 1) / 2;
  const int64_t full = (int64_t)L * np_ * np_;
  double* p2 = ws.ypart + (int64_t)L * nt * np_;
  if (!upper) {
    const _Float16* yh = reinterpret_cast<const _Float16*>(ws.A);  // the Y planes (A is dead after potrf)
    kl_ymv_kernel<false, false><<<dim3(ntri, L), 256, 0, st>>>(yh, yh + full, ysc, np_, x, ws.ypart, nullptr);
    kl_ymv_reduce<false><<<dim3(nt, L), 256, 0, st>>>(ws.ypart, base, np_, out);
  } else {
    const _Float16* th = ws.planes;  // the Y^T planes
    if (sumsq) {
      kl_ymv_kernel<true, true><<<dim3(ntri, L), 256, 0, st>>>(th, th + full, ysc, np_, x, ws.ypart, p2);
      kl_ymv_reduce<true><<<dim3(nt, L), 256, 0, st>>>(p2, nullptr, np_, sumsq);
    } else {
      kl_ymv_kernel<true, false><<<dim3(ntri, L), 256, 0, st>>>(th, th + full, ysc, np_, x, ws.ypart, nullptr);
    }
    kl_ymv_reduce<true><<<dim3(nt, L), 256, 0, st>>>(ws.ypart, base, np_, out);
  }
}

int lvae_kl_closed_reduce_f32(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int L,
                              const double* params, const double* noise, const double* mu, const double* logv,
                              int ld_mu, double* kl, void* workspace, int need_bwd, void* stream) {
  if (!spec) return -1;
  if (!x) return -2;
  if (n <= 0) return -4;
  if (L <= 0) return -5;
  if (!params) return -6;
  if (!noise) return -7;
  if (!mu || !logv || ld_mu < L) return -8;
  if (!kl) return -11;
  if (!workspace || ((uintptr_t)workspace & 255)) return -12;
  hipStream_t st = (hipStream_t)stream;
  const int np_ = lvae_kl_closed_padded_n(n);
  KLWorkspace ws((char*)workspace, np_, L);
  ProfScope ps(LVAE_PH_KL_REDUCE, st);
  kl_prep_kernel<<<dim3(cdiv(np_, 256), L), 256, 0, st>>>(mu, logv, ld_mu, n, np_, L, ws.mu, ws.v, ws.sv);
  const bool rb_on = kl_resid_bins_enabled(spec, n);  // (the plan: the factor call's, joined on `st`)
  if (kl_early(np_, L)) {
    // a0 = Y^T (Y mu) and d = diag K^-1 (the row sums of squares of Y^T); r = mu - K a0 in fp64 from the
    // covariates; a = a0 + Y^T (Y r); the refinement gate on d, and for the flagged dims (if any) their K^-1 alone
    // (the other dims' lauum workgroups exit) and the fp64 diag refinement; the KL.  No K^-1 for unflagged dims.
    const float* ysc = ci_ysc_ptr(ws.chol, np_, L);
    kl_ymv(ws, ysc, np_, L, false, ws.mu, nullptr, ws.yvec, nullptr, st);
    kl_ymv(ws, ysc, np_, L, true, ws.yvec, nullptr, ws.alpha, ws.kdiag, st);
    LVAE_TRY(kl_gram_resid(spec, x, ldx, n, np_, L, params, noise, ws.alpha, ws.mu, ws.rpart, ws.res,
                           rb_on ? ws.rb : nullptr, st));
    kl_ymv(ws, ysc, np_, L, false, ws.res, nullptr, ws.yvec, nullptr, st);
    kl_ymv(ws, ysc, np_, L, true, ws.yvec, ws.alpha, ws.alpha, nullptr, st);
    LVAE_TRY(kl_refine_gate(spec, x, ldx, n, np_, L, params, noise, ws.kdiag, ws.rest, ws.rflag, st));
    LVAE_TRY(ci_lauum_flagged_f32(np_, L, ws.chol, ws.planes, ws.Kinv, ws.rflag, st));
    LVAE_TRY(kl_refine_apply(spec, x, ldx, n, np_, L, params, noise, ws.Kinv, ws.kdiag, ws.K64e, ws.rpart, ws.rflag,
                             st));
    kl_finalize_kernel<<<L, 256, 0, st>>>(ws.mu, logv, ld_mu, ws.alpha, ws.kdiag, ws.logdet, n, np_, kl);
    LVAE_CHECK_LAUNCH();
    return 0;
  }
  // K^-1 (+ the partials of a0 = K^-1 mu, + the B planes); a0, d; r = mu - K a0 in fp64 from the
  // covariates; a = a0 + K^-1 r
  LVAE_TRY(ci_lauum_f32(np_, L, ws.chol, ws.planes, ws.Kinv, ws.mu, ws.sv, ws.apart, need_bwd ? ws.Bp : nullptr,
                        ws.bsc, st, ws.hbon));
  kl_alpha0_kernel<<<dim3(np_ / 256, L), 256, 0, st>>>(ws.apart, ws.Kinv, np_, ws.alpha, ws.kdiag);
  LVAE_TRY(kl_gram_resid(spec, x, ldx, n, np_, L, params, noise, ws.alpha, ws.mu, ws.rpart, ws.res,
                         rb_on ? ws.rb : nullptr, st));
  {  // alpha = a0 + K^-1 r over the lower tiles of K^-1 (the residual's partials buffer is free again)
    const int nt64 = np_ / 64, ntiles = nt64 * (nt64 + 1) / 2;
    int G = (LVAE_ALPHA_WG + L - 1) / L;  // workgroups in all (~16 resident per CU: more loads in flight)
    G = G < ntiles ? G : ntiles;
    kl_alpha_sym_kernel<<<dim3(G, L), 256, 0, st>>>(ws.Kinv, ws.res, np_, ws.rpart, ntiles);
    kl_alpha_reduce<<<dim3(np_ / 256, L), 256, 0, st>>>(ws.rpart, ws.alpha, np_, ws.alpha);
  }
  // diag K^-1 in fp64 for the dims whose (sum_r s_r + noise) max (K^-1)_ii says the fp32 inverse's diagonal is not
  // enough (kl_refine.hip; the partials buffer is free again)
  LVAE_TRY(kl_refine_diag(spec, x, ldx, n, np_, L, params, noise, ws.Kinv, ws.kdiag, ws.K64, ws.rpart, ws.rest,
                          ws.rflag, st));
  kl_finalize_kernel<<<L, 256, 0, st>>>(ws.mu, logv, ld_mu, ws.alpha, ws.kdiag, ws.logdet, n, np_, kl);
  LVAE_CHECK_LAUNCH();
  return 0;
}

int lvae_kl_closed_fwd_f32(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int L, const double* params,
                           const double* noise, const double* mu, const double* logv, int ld_mu, double* kl,
                           int32_t* info, void* workspace, int need_bwd, void* stream) {
  if (!spec) return -1;
  if (!x) return -2;
  if (n <= 0) return -4;
  if (L <= 0) return -5;
  if (!params) return -6;
  if (!noise) return -7;
  if (!mu || !logv || ld_mu < L) return -8;
  if (!kl) return -11;
  if (!workspace || ((uintptr_t)workspace & 255)) return -13;
  LVAE_TRY(lvae_kl_closed_factor_f32(spec, x, ldx, n, L, params, noise, info, workspace, stream));
  return lvae_kl_closed_reduce_f32(spec, x, ldx, n, L, params, noise, mu, logv, ld_mu, kl, workspace, need_bwd, stream);
}

// d kl / d (params, noise): S = K^-1 V K^-1, then the fused Gram adjoint
int lvae_kl_closed_bwd_hyper_f32(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int L,
                                 const double* params, const double* gkl, double* dparams, double* dnoise,
                                 void* workspace, void* stream) {
  if (!spec) return -1;
  if (!workspace || ((uintptr_t)workspace & 255)) return -15;
  hipStream_t st = (hipStream_t)stream;
  const int np_ = lvae_kl_closed_padded_n(n);
  KLWorkspace ws((char*)workspace, np_, L);
  if (kl_early(np_, L)) {
    // the early reduce left K^-1 to this half: lauum now (+ the B planes for the S GEMM when the binned route is off;
    // the a0 partials it also writes are unused), beside the encoder's backward on the caller's other stream
    ProfScope ps(LVAE_PH_KL_REDUCE, st);
    LVAE_TRY(ci_lauum_f32(np_, L, ws.chol, ws.planes, ws.Kinv, ws.mu, ws.sv, ws.apart, ws.Bp, ws.bsc, st, ws.hbon));
  }
  // S = K^-1 V K^-1 = B B^T into the (no longer needed) Y^T plane buffer, from the fp16 hi / lo planes
  // of B = K^-1 diag(sqrt v) the forward wrote (need_bwd; np is a multiple of 256: lvae_kl_closed_padded_n)
  float* S = reinterpret_cast<float*>(ws.planes);
  {
    ProfScope ps(LVAE_PH_SYRK, st);
    LVAE_TRY(syrk_tiles_f32(np_, L, ws.bsc, ws.Bp, S, ws.Sx, st, ws.hbon));
  }
  {
    ProfScope ps(LVAE_PH_GRAM_BWD, st);
    LVAE_TRY(kl_gram_bwd(spec, x, ldx, n, np_, L, params, ws.Kinv, S, ws.Sx, syrk_x3_splits(np_, L), ws.alpha,
                         ws.kdiag, ws.v, gkl, ws.part, dparams, dnoise, ws.covflag, ws.hb, ws.hbon, st));
  }
  LVAE_CHECK_LAUNCH();
  return 0;
}

// d kl / d (mu, logv): elementwise from K^-1 mu and diag K^-1 (the forward's)
int lvae_kl_closed_bwd_latent_f32(int n, int L, const double* logv, int ld_mu, const double* gkl, double* dmu,
                                  double* dlogv, void* workspace, void* stream) {
  if (n <= 0) return -4;
  if (L <= 0) return -5;
  if (!logv || ld_mu < L) return -8;
  if (!gkl || !dmu || !dlogv) return -10;
  if (!workspace || ((uintptr_t)workspace & 255)) return -15;
  hipStream_t st = (hipStream_t)stream;
  const int np_ = lvae_kl_closed_padded_n(n);
  KLWorkspace ws((char*)workspace, np_, L);
  ProfScope ps(LVAE_PH_BWD_ELEM, st);
  const int64_t tot = (int64_t)n * L;
  kl_bwd_elem_kernel<<<cdiv(tot, 256), 256, 0, st>>>(logv, ld_mu, n, np_, L, ws.alpha, ws.kdiag, gkl, dmu, dlogv);
  LVAE_CHECK_LAUNCH();
  return 0;
}

int lvae_kl_closed_bwd_f32(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int L, const double* params,
                           const double* mu, const double* logv, int ld_mu, const double* gkl, double* dmu,
                           double* dlogv, double* dparams, double* dnoise, void* workspace, void* stream) {
  (void)mu;
  LVAE_TRY(lvae_kl_closed_bwd_latent_f32(n, L, logv, ld_mu, gkl, dmu, dlogv, workspace, stream));
  return lvae_kl_closed_bwd_hyper_f32(spec, x, ldx, n, L, params, gkl, dparams, dnoise, workspace, stream);
}

int lvae_kl_closed_refine_state(int n, int L, const void* workspace, double* est, int32_t* flag, void* stream) {
  if (n <= 0) return -1;
  if (L <= 0) return -2;
  if (!workspace || ((uintptr_t)workspace & 255)) return -3;
  if (!est || !flag) return -4;
  const int np_ = lvae_kl_closed_padded_n(n);
  KLWorkspace ws((char*)workspace, np_, L);
  hipStream_t st = (hipStream_t)stream;
  if (copy_words_async(est, ws.rest, (size_t)L * sizeof(double), st) != 0 ||
      copy_words_async(flag, ws.rflag, (size_t)L * sizeof(int32_t), st) != 0)
    return LVAE_ERR_LAUNCH;
  return 0;
}

const char* lvae_version(void) { return "lvae_hip 0.1.0 gfx950"; }

}  // extern "C"
