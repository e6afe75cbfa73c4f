// small.hip -- batched small fp64 linear algebra for the Hensman SVI path (Regime A, fp64 required:
// K0zz has a 1e-6 jitter and cond ~1e8, fp32 Cholesky fails -- SURVEY.md §0).
//
//   spd_inv_small : one workgroup per matrix (n <= 128): 16-block Cholesky + block triangular solves in
//                   MFMA f64 accumulators (blkinv.hpp) -> A^-1, log|A| and LAPACK-style info.
//                   Replaces torch.cholesky + cholesky_solve(I) at elbo_functions.py:176-186 and
//                   training.py:130-134 (M = 120 -> 128: 8 waves x 8 tiles, 8 + 8 + 8 block steps).
//   gemm_small    : C = alpha op(A) op(B) + beta C over a two-level batch; 32x32 output tile per
//                   workgroup on v_mfma_f64_16x16x4f64, K staged through LDS in one pass (K <= 128).
#include "common.hpp"
#include "blkinv.hpp"

namespace lvae {

constexpr int kSmallMax = 128;

// Two independent batches in one launch (blocks [0, nb0) take set 0, the rest set 1): the
// Hensman forward inverts K0zz and H together, halving the serial inverse launches per step.
struct InvSet {
  const double* A;
  int64_t stride;
  double* Ainv;
  int64_t stride_out;
  double* logdet;
  int32_t* info;
};

template <int TS, int TPW>
__global__ __launch_bounds__(64 * TS * TS / TPW) void spd_inv_small_kernel(int n, int nb0, InvSet s0, InvSet s1) {
  const bool first = (int)blockIdx.x < nb0;
  const InvSet& s = first ? s0 : s1;
  const int b = first ? blockIdx.x : blockIdx.x - nb0;
  blk_inverse<double, TS, TPW>(n, s.A + (int64_t)b * s.stride, n, s.Ainv + (int64_t)b * s.stride_out, n,
                                 s.logdet + b, 0, s.info + b, 0);
}

constexpr int kGS = 32;   // output tile edge
constexpr int kGK = 128;  // K staged per pass (every Hensman product has K <= 128: one pass)

// 32 x 32 output tile per 256-thread workgroup, one 16 x 16 quarter per wave on v_mfma_f64_16x16x4f64
// (C[(lane >> 4) + 4 r][lane & 15], blkinv.hpp); op(A) and op(B) staged for the whole K (<= 128 per pass)
// in one round of loads, then kc / 4 MFMAs per wave -- one global-latency round trip per launch instead
// of one per 32-deep chunk.
__global__ __launch_bounds__(256) void gemm_small_kernel(int ta, int tb, int m, int n, int k, double alpha,
                                                         const double* __restrict__ A, int lda, int64_t sa1,
                                                         int64_t sa2, const double* __restrict__ B, int ldb,
                                                         int64_t sb1, int64_t sb2, double beta,
                                                         double* __restrict__ C, int ldc, int64_t sc1, int64_t sc2,
                                                         int nb2) {
  __shared__ double As[kGS][kGK + 1];  // [i][kk]
  __shared__ double Bs[kGK][kGS + 1];  // [kk][j]
  const int bz = blockIdx.z, b1 = bz / nb2, b2 = bz % nb2;
  const double* a = A + b1 * sa1 + b2 * sa2;
  const double* bb = B + b1 * sb1 + b2 * sb2;
  double* c = C + b1 * sc1 + b2 * sc2;
  const int i0 = blockIdx.y * kGS, j0 = blockIdx.x * kGS;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, li = lane & 15, lk = lane >> 4;
  const int wr = (w >> 1) * 16, wc = (w & 1) * 16;
  bi_f64x4 acc = {0.0, 0.0, 0.0, 0.0};
  for (int k0 = 0; k0 < k; k0 += kGK) {
    const int kc = k - k0 < kGK ? k - k0 : kGK, kc4 = (kc + 3) & ~3;  // zero-padded to whole MFMA steps
    // op(A)[i0 + r][k0 + q]: q fastest when A is row-major in k (ta = 0), r fastest when transposed
#pragma unroll
    for (int u = 0; u < kGS * kGK / 256; ++u) {  // (constant trip count: the loads issue together)
      const int e = tid + 256 * u;
      const int r = ta ? (e & (kGS - 1)) : (e >> 7), q = ta ? (e >> 5) : (e & (kGK - 1));
      if (q < kc4) {
        const int i = i0 + r, kk = k0 + q;
        double v = 0.0;
        if (i < m && q < kc) v = ta ? a[(int64_t)kk * lda + i] : a[(int64_t)i * lda + kk];
        As[r][q] = v;
      }
    }
    // op(B)[k0 + r][j0 + q]: q fastest for row-major B (tb = 0)
#pragma unroll
    for (int u = 0; u < kGK * kGS / 256; ++u) {
      const int e = tid + 256 * u;
      const int r = tb ? (e & (kGK - 1)) : (e >> 5), q = tb ? (e >> 7) : (e & (kGS - 1));
      if (r < kc4) {
        const int kk = k0 + r, j = j0 + q;
        double v = 0.0;
        if (r < kc && j < n) v = tb ? bb[(int64_t)j * ldb + kk] : bb[(int64_t)kk * ldb + j];
        Bs[r][q] = v;
      }
    }
    __syncthreads();
    for (int kk = 0; kk < kc4; kk += 4)
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(As[wr + li][kk + lk], Bs[kk + lk][wc + li], acc, 0, 0, 0);
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = i0 + wr + lk + 4 * r, j = j0 + wc + li;
    if (i < m && j < n) {
      double* p = c + (int64_t)i * ldc + j;
      *p = (beta == 0.0) ? alpha * acc[r] : alpha * acc[r] + beta * *p;
    }
  }
}

int spd_inv_small2_f64(int n, int nb0, const double* A0, int64_t stride0, double* Ainv0, int64_t stride_out0,
                       double* logdet0, int32_t* info0, int nb1, const double* A1, int64_t stride1, double* Ainv1,
                       int64_t stride_out1, double* logdet1, int32_t* info1, hipStream_t st) {
  if (n < 1 || n > kSmallMax) return -1;
  if (nb0 < 0 || nb1 < 0) return -2;
  const int batch = nb0 + nb1;
  if (batch == 0) return 0;
  const InvSet s0{A0, stride0, Ainv0, stride_out0, logdet0, info0};
  const InvSet s1{A1, stride1, Ainv1, stride_out1, logdet1, info1};
  if (n <= 16)
    spd_inv_small_kernel<1, 1><<<batch, 64, 0, st>>>(n, nb0, s0, s1);
  else if (n <= 32)
    spd_inv_small_kernel<2, 2><<<batch, 128, 0, st>>>(n, nb0, s0, s1);
  else if (n <= 64)
    spd_inv_small_kernel<4, 2><<<batch, 512, 0, st>>>(n, nb0, s0, s1);
  else
    spd_inv_small_kernel<8, 8><<<batch, 512, 0, st>>>(n, nb0, s0, s1);
  LVAE_CHECK_LAUNCH();
  return 0;
}

int spd_inv_small_f64(int n, int batch, const double* A, int64_t stride, double* Ainv, int64_t stride_out,
                      double* logdet, int32_t* info, hipStream_t st) {
  return spd_inv_small2_f64(n, batch, A, stride, Ainv, stride_out, logdet, info, 0, A, stride, Ainv, stride_out,
                            logdet, info, st);
}

int gemm_small_f64(int ta, int tb, int m, int n, int k, double alpha, const double* A, int lda, int64_t sa1,
                   int64_t sa2, const double* B, int ldb, int64_t sb1, int64_t sb2, double beta, double* C, int ldc,
                   int64_t sc1, int64_t sc2, int nb1, int nb2, hipStream_t st) {
  if (m < 0 || n < 0 || k < 0) return -3;
  if (nb1 < 1 || nb2 < 1) return -20;
  if (m == 0 || n == 0) return 0;
  dim3 grid(cdiv(n, kGS), cdiv(m, kGS), nb1 * nb2);
  gemm_small_kernel<<<grid, 256, 0, st>>>(ta, tb, m, n, k, alpha, A, lda, sa1, sa2, B, ldb, sb1, sb2, beta, C, ldc,
                                          sc1, sc2, nb2);
  LVAE_CHECK_LAUNCH();
  return 0;
}

}  // namespace lvae

extern "C" {
int lvae_spd_inv_small_f64(int n, int batch, const double* A, int64_t stride, double* Ainv, int64_t stride_out,
                           double* logdet, int32_t* info, void* stream) {
  return lvae::spd_inv_small_f64(n, batch, A, stride, Ainv, stride_out, logdet, info, (hipStream_t)stream);
}

int lvae_gemm_small_f64(int ta, int tb, int m, int n, int k, double alpha, const double* A, int lda, int64_t sa1,
                        int64_t sa2, const double* B, int ldb, int64_t sb1, int64_t sb2, double beta, double* C,
                        int ldc, int64_t sc1, int64_t sc2, int nb1, int nb2, void* stream) {
  return lvae::gemm_small_f64(ta, tb, m, n, k, alpha, A, lda, sa1, sa2, B, ldb, sb1, sb2, beta, C, ldc, sc1, sc2,
                              nb1, nb2, (hipStream_t)stream);
}
}
