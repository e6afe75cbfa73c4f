// small.hip -- batched small fp64 linear algebra for the Hensman SVI path (Regime A, fp64 required:
// K0zz has a 1e-6 jitter and cond ~1e8, fp32 Cholesky fails -- SURVEY.md §0).
//
//   spd_inv_small : one workgroup per matrix (n <= 128): Cholesky in LDS, in-place L^-1, then
//                   A^-1 = L^-T L^-1 straight to global; log|A| and LAPACK-style info.
//                   Replaces torch.cholesky + cholesky_solve(I) at elbo_functions.py:176-186 and
//                   training.py:130-134 (M = 120 -> 120*121*8 B = 116 KB of LDS).
//   gemm_small    : C = alpha op(A) op(B) + beta C over a two-level batch; 32x32 output tile per
//                   workgroup, K staged through LDS in chunks of 32.
#include "common.hpp"

namespace lvae {

constexpr int kSmallMax = 128;

__global__ __launch_bounds__(256) void spd_inv_small_kernel(int n, const double* __restrict__ A, int64_t stride,
                                                            double* __restrict__ Ainv, int64_t stride_out,
                                                            double* __restrict__ logdet,
                                                            int32_t* __restrict__ info) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int ld = n + 1;
  double* Ls = sm;  // [n][n+1]
  __shared__ double red[4];
  __shared__ int fail;
  const int b = blockIdx.x, tid = threadIdx.x;
  const double* a = A + (int64_t)b * stride;
  for (int e = tid; e < n * n; e += 256) {
    const int i = e / n, j = e - i * n;
    Ls[i * ld + j] = a[e];
  }
  if (tid == 0) fail = 0;
  __syncthreads();
  // right-looking Cholesky, one column per step
  for (int j = 0; j < n; ++j) {
    const double d = Ls[j * ld + j];
    if (!(d > 0.0) || !isfinite(d)) {
      if (tid == 0 && fail == 0) fail = j + 1;
    }
    const double piv = sqrt(d);
    __syncthreads();
    for (int i = j + 1 + tid; i < n; i += 256) Ls[i * ld + j] /= piv;
    if (tid == 0) Ls[j * ld + j] = piv;
    __syncthreads();
    const int R = n - j - 1;
    for (int e = tid; e < R * R; e += 256) {
      const int ii = e / R, jj = e - ii * R;
      if (jj <= ii) {
        const int i = j + 1 + ii, c = j + 1 + jj;
        Ls[i * ld + c] -= Ls[i * ld + j] * Ls[c * ld + j];
      }
    }
    __syncthreads();
  }
  // log|A|
  double ls = 0.0;
  for (int j = tid; j < n; j += 256) ls += log(Ls[j * ld + j]);
  ls = block_sum<256>(ls, red);
  if (tid == 0) {
    logdet[b] = 2.0 * ls;
    info[b] = fail;
  }
  // in-place inverse of the lower factor (LAPACK trti2 order: last column first)
  for (int j = n - 1; j >= 0; --j) {
    __syncthreads();
    const double wjj = 1.0 / Ls[j * ld + j];
    // x = L[j+1:, j];  W[j+1:, j] = -wjj * W[j+1:, j+1:] x  (W[j+1:, j+1:] already inverted)
    double y[1];
    const int R = n - j - 1;
    double acc = 0.0;
    const int i = j + 1 + tid;
    if (tid < R) {
      for (int k = j + 1; k <= i; ++k) acc += Ls[i * ld + k] * Ls[k * ld + j];
    }
    y[0] = acc;
    __syncthreads();
    if (tid < R) Ls[i * ld + j] = -wjj * y[0];
    if (tid == 0) Ls[j * ld + j] = wjj;
  }
  __syncthreads();
  // A^-1 = W^T W : (i, j) = sum_{k >= max(i,j)} W[k][i] W[k][j]
  double* o = Ainv + (int64_t)b * stride_out;
  for (int e = tid; e < n * n; e += 256) {
    const int i = e / n, j = e - i * n;
    const int k0 = i > j ? i : j;
    double acc = 0.0;
    for (int k = k0; k < n; ++k) acc += Ls[k * ld + i] * Ls[k * ld + j];
    o[e] = acc;
  }
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

int spd_inv_small_f64(int n, int batch, const double* A, int64_t stride, double* Ainv, int64_t stride_out,
                      double* logdet, int32_t* info, hipStream_t st) {
  if (n < 1 || n > kSmallMax) return -1;
  if (batch < 0) return -2;
  if (batch == 0) return 0;
  const size_t lds = (size_t)n * (n + 1) * sizeof(double);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)spd_inv_small_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)(kSmallMax * (kSmallMax + 1) * sizeof(double)));
    attr = true;
  }
  spd_inv_small_kernel<<<batch, 256, lds, st>>>(n, A, stride, Ainv, stride_out, logdet, info);
  LVAE_CHECK_LAUNCH();
  return 0;
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
