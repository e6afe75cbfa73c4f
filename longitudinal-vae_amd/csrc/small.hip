// small.hip -- batched small fp64 linear algebra for the Hensman SVI path (Regime A, fp64 required:
// K0zz has a 1e-6 jitter and cond ~1e8, fp32 Cholesky fails -- SURVEY.md §0).
//
//   spd_inv_small : one workgroup per matrix (n <= 128): 16-block Cholesky + block triangular solves in
//                   MFMA f64 accumulators (blkinv.hpp) -> A^-1, log|A| and LAPACK-style info.
//                   Replaces torch.cholesky + cholesky_solve(I) at elbo_functions.py:176-186 and
//                   training.py:130-134 (M = 120 -> 128: 8 waves x 8 tiles, 8 + 8 + 8 block steps).
//   gemm_small    : C = alpha op(A) op(B) + beta C over a two-level batch; 32x32 output tile per
//                   workgroup, K staged through LDS in chunks of 32.
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

constexpr int kGS = 32;

__global__ __launch_bounds__(256) void gemm_small_kernel(int ta, int tb, int m, int n, int k, double alpha,
                                                         const double* __restrict__ A, int lda, int64_t sa1,
                                                         int64_t sa2, const double* __restrict__ B, int ldb,
                                                         int64_t sb1, int64_t sb2, double beta,
                                                         double* __restrict__ C, int ldc, int64_t sc1, int64_t sc2,
                                                         int nb2) {
  __shared__ double As[kGS][kGS + 1];  // [i][kk]
  __shared__ double Bs[kGS][kGS + 1];  // [kk][j]
  const int bz = blockIdx.z, b1 = bz / nb2, b2 = bz % nb2;
  const double* a = A + b1 * sa1 + b2 * sa2;
  const double* bb = B + b1 * sb1 + b2 * sb2;
  double* c = C + b1 * sc1 + b2 * sc2;
  const int i0 = blockIdx.y * kGS, j0 = blockIdx.x * kGS;
  const int tid = threadIdx.x, tj = tid & 31, ti = tid >> 5;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  for (int k0 = 0; k0 < k; k0 += kGS) {
    for (int e = tid; e < kGS * kGS; e += 256) {
      const int r = e >> 5, q = e & 31;
      // As[r][q] = op(A)[i0 + r][k0 + q];  Bs[r][q] = op(B)[k0 + r][j0 + q]
      {
        const int i = i0 + r, kk = k0 + q;
        double v = 0.0;
        if (i < m && kk < k) v = ta ? a[(int64_t)kk * lda + i] : a[(int64_t)i * lda + kk];
        As[r][q] = v;
      }
      {
        const int kk = k0 + r, j = j0 + q;
        double v = 0.0;
        if (kk < k && j < n) v = tb ? bb[(int64_t)j * ldb + kk] : bb[(int64_t)kk * ldb + j];
        Bs[r][q] = v;
      }
    }
    __syncthreads();
#pragma unroll 8
    for (int q = 0; q < kGS; ++q) {
      const double bv = Bs[q][tj];
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] += As[ti + 8 * u][q] * bv;
    }
    __syncthreads();
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = i0 + ti + 8 * u, j = j0 + tj;
    if (i < m && j < n) {
      double* p = c + (int64_t)i * ldc + j;
      *p = (beta == 0.0) ? alpha * acc[u] : alpha * acc[u] + beta * *p;
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
