// potrf.hip -- the standalone N x N factor / solve entry points of the C ABI, the reference's
//   LK1 = torch.cholesky(K1);  torch.cholesky_solve(B, LK1);  2 sum log diag(LK1)      (elbo_functions.py:26-29)
// as LAPACK-shaped calls over L batched matrices:
//   lvae_potrf_f64   blocked right-looking Cholesky in fp64: 64-wide block columns; per pass one launch factors
//                    the diagonal block and inverts its factor (16 x 16 pivots in f64 MFMA accumulators), one
//                    solves the panel as the product L_ik = A_ik L_kk^-T (the trtri-based trsm of MAGMA /
//                    rocSOLVER), one applies the trailing update A_IJ -= L_Ik L_Jk^T -- all on
//                    v_mfma_f64_16x16x4f64
//   lvae_potrf_f32   the exact KL's own factorisation (chol_inv.hip: 256-wide blocks, pivots in LDS on fp32
//                    MFMA, panels / trailing updates on the f16 cores with the 3-product split), stopped after
//                    potrf and exported as an fp32 L
//   lvae_trsm_*      op(L)^-1 B over 64-column chunks of B: one workgroup per (chunk, matrix) sweeps the block
//                    rows in dependency order, R = B_k - sum_j op(L)_kj X_j and X_k = op(L_kk^-1) R, both on
//                    the f64 MFMA (the 64 x 64 diagonal-block inverses first, one workgroup each, as the
//                    blocked trsm of rocBLAS / LAPACK's trtri-based solve do); f32 operands are computed in fp64
//   lvae_potrs_*     trsm(L) then trsm(L^T)
#include "blkinv.hpp"
#include "pv_lds.hpp"  // kSwB

namespace lvae {

// chol_inv.hip
size_t ci_scratch_bytes(int np_, int L);
int ci_potrf_f32(int np_, int L, float* A, void* scratch, double* logdet, int32_t* info, hipStream_t st);

constexpr int kPB = 64;        // block edge
constexpr int kPBL = kPB + 1;  // LDS pitch (doubles)

__device__ inline void p64_tri(int t, int& I, int& J) {  // t -> (I, J), J <= I, row-major lower triangle
  int r = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
  while ((r + 1) * (r + 2) / 2 <= t) ++r;
  while (r * (r + 1) / 2 > t) --r;
  I = r;
  J = t - r * (r + 1) / 2;
}

// 64 x 64 x 64 product on the f64 MFMA: wave w owns rows 16 w .. 16 w + 15 of the tile, acc[cb] its 16 x 16
// block of columns 16 cb ..; A operand As[row][kk], B operand Bs[kk][col] (v_mfma_f64_16x16x4f64, lane
// (li = lane & 15, lk = lane >> 4): A[li][lk], B[lk][li]; acc[cb][r] = C[lk + 4 r][li])
__device__ inline void p64_mma(const double* __restrict__ As, const double* __restrict__ Bs, bi_f64x4 (&acc)[4]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, li = lane & 15, lk = lane >> 4;
#pragma unroll 4
  for (int kk = 0; kk < kPB; kk += 4) {
    const double a = As[(16 * w + li) * kPBL + kk + lk];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
      acc[cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, Bs[(kk + lk) * kPBL + 16 * cb + li], acc[cb], 0, 0, 0);
  }
}

// pass k, the diagonal block (one 256-thread workgroup per matrix): L_kk and Y_kk = L_kk^-1 by the 16-block
// Cholesky in f64 MFMA accumulators (blkinv.hpp, MODE 1: no thread-serial pivots, the 16 x 16 pivots in
// registers).  L_kk goes to A's lower part, Y_kk's strict lower part transposed into A_kk's strict upper part
// (the panel launch's operand, zeroed by the next pass's diagonal launch; the last block writes no Y).  Also
// zeroes the strict upper part right of the block, adds 2 sum log L_jj to logdet[l] and sets info[l]
// LAPACK-style.  Only this launch writes A_kk: the panel launch after it reads it (the former
// fused diagonal + panel launch had one workgroup overwrite A_kk while others of the same launch still read it).
__global__ __launch_bounds__(256) void p64_diag_kernel(double* __restrict__ A, int64_t lda, int64_t sa, int n, int k,
                                                       double* __restrict__ logdet, int32_t* __restrict__ info) {
  const int l = blockIdx.x, tid = threadIdx.x, nt = (n + kPB - 1) / kPB;
  double* Al = A + (int64_t)l * sa;
  const int k0 = k * kPB, nbk = min(kPB, n - k0);
  if (k > 0) {  // the previous diagonal block's Y^T (its panel launch is done)
    const int p0 = k0 - kPB;
    for (int e = tid; e < kPB * kPB; e += 256) {
      const int r = e >> 6, c = e & 63;
      if (c > r) Al[(int64_t)(p0 + r) * lda + p0 + c] = 0.0;
    }
  }
  for (int r = 0; r < nbk; ++r)  // the strict upper part right of the diagonal block
    for (int c = k0 + nbk + tid; c < n; c += 256) Al[(int64_t)(k0 + r) * lda + c] = 0.0;
  double* D = Al + (int64_t)k0 * lda + k0;
  const bool last = k + 1 == nt;
  if (last) {  // no panel reads Y: the strict upper part of the block is zero
    for (int e = tid; e < nbk * nbk; e += 256) {
      const int r = e / nbk, c = e % nbk;
      if (c > r) D[(int64_t)r * lda + c] = 0.0;
    }
    __syncthreads();
  }
  blk_inverse<double, 4, 4, 1>(nbk, D, lda, last ? nullptr : D, lda, logdet + l, 1, info + l, k0, D, lda);
}

// pass k, the panel: L_ik = A_ik Y_kk^T for the block rows i > k, one workgroup per (block, matrix) on the f64
// MFMA; Y_kk^T's strict upper part from A_kk's strict upper triangle, its diagonal 1 / L_jj
__global__ __launch_bounds__(256) void p64_panel_kernel(double* __restrict__ A, int64_t lda, int64_t sa, int n, int k) {
  __shared__ double As[kPB * kPBL];  // A_ik [row][kk]
  __shared__ double Bs[kPB * kPBL];  // Y_kk^T [kk][col]
  const int l = blockIdx.y, tid = threadIdx.x;
  double* Al = A + (int64_t)l * sa;
  const int k0 = k * kPB, nbk = min(kPB, n - k0), i0 = (k + 1 + blockIdx.x) * kPB, nbi = min(kPB, n - i0);
  for (int e = tid; e < kPB * kPB; e += 256) {
    const int r = e >> 6, c = e & 63;
    As[r * kPBL + c] = (r < nbi && c < nbk) ? Al[(int64_t)(i0 + r) * lda + k0 + c] : 0.0;
    const double y = Al[(int64_t)(k0 + min(r, nbk - 1)) * lda + k0 + min(c, nbk - 1)];
    Bs[r * kPBL + c] = (r < nbk && c < nbk && c >= r) ? (c > r ? y : 1.0 / y) : 0.0;
  }
  __syncthreads();
  bi_f64x4 acc[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) acc[cb] = bi_f64x4{0.0, 0.0, 0.0, 0.0};
  p64_mma(As, Bs, acc);
  const int lane = tid & 63, w = tid >> 6, li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * w + lk + 4 * r, col = 16 * cb + li;
      if (row < nbi && col < nbk) Al[(int64_t)(i0 + row) * lda + k0 + col] = acc[cb][r];
    }
}

// trailing update of pass k: A_IJ -= L_Ik L_Jk^T for the lower tiles k < J <= I, one workgroup per tile
__global__ __launch_bounds__(256) void p64_update_kernel(double* __restrict__ A, int64_t lda, int64_t sa, int n, int k) {
  __shared__ double As[kPB * kPBL];  // L_Ik [row][kk]
  __shared__ double Bs[kPB * kPBL];  // L_Jk^T [kk][col]
  const int l = blockIdx.y, tid = threadIdx.x;
  int I, J;
  p64_tri(blockIdx.x, I, J);
  I += k + 1;
  J += k + 1;
  double* Al = A + (int64_t)l * sa;
  const int k0 = k * kPB, I0 = I * kPB, J0 = J * kPB;
  for (int e = tid; e < kPB * kPB; e += 256) {
    const int r = e >> 6, c = e & 63;
    const bool kc = k0 + c < n;
    As[r * kPBL + c] = (I0 + r < n && kc) ? Al[(int64_t)(I0 + r) * lda + k0 + c] : 0.0;
    Bs[c * kPBL + r] = (J0 + r < n && kc) ? Al[(int64_t)(J0 + r) * lda + k0 + c] : 0.0;
  }
  __syncthreads();
  bi_f64x4 acc[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) acc[cb] = bi_f64x4{0.0, 0.0, 0.0, 0.0};
  p64_mma(As, Bs, acc);
  const int lane = tid & 63, w = tid >> 6, li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = I0 + 16 * w + lk + 4 * r, j = J0 + 16 * cb + li;
      if (i < n && j < n && j <= i) Al[(int64_t)i * lda + j] -= acc[cb][r];
    }
}

// dst lower triangle <- src lower triangle (an out-of-place potrf_f64 factors in dst)
template <typename T>
__global__ __launch_bounds__(256) void p64_copy_lower_kernel(const T* __restrict__ src, int64_t lds_, int64_t ss,
                                                             T* __restrict__ dst, int64_t ldd, int64_t sd, int n) {
  const int l = blockIdx.y, i = blockIdx.x;
  for (int j = threadIdx.x; j <= i; j += 256) dst[(int64_t)l * sd + (int64_t)i * ldd + j] = src[(int64_t)l * ss + (int64_t)i * lds_ + j];
}

int potrf_f64(int n, int L, const double* A, int64_t lda, int64_t sa, double* Lo, int64_t ldo, int64_t so,
              double* logdet, int32_t* info, hipStream_t st) {
  if (n <= 0) return -1;
  if (L <= 0) return -2;
  if (!A) return -3;
  if (lda < n) return -4;
  if (!Lo) return -6;
  if (ldo < n) return -7;
  if (!logdet) return -9;
  if (!info) return -10;
  if (Lo != A) {
    p64_copy_lower_kernel<double><<<dim3(n, L), 256, 0, st>>>(A, lda, sa, Lo, ldo, so, n);
  } else if (lda != ldo || sa != so) {
    return -7;
  }
  (void)zero_async(logdet, sizeof(double) * L, st);
  (void)zero_async(info, sizeof(int32_t) * L, st);
  const int nt = cdiv(n, kPB);
  for (int k = 0; k < nt; ++k) {
    p64_diag_kernel<<<L, 256, 0, st>>>(Lo, ldo, so, n, k, logdet, info);
    const int m = nt - k - 1;
    if (m > 0) {
      p64_panel_kernel<<<dim3(m, L), 256, 0, st>>>(Lo, ldo, so, n, k);
      p64_update_kernel<<<dim3(m * (m + 1) / 2, L), 256, 0, st>>>(Lo, ldo, so, n, k);
    }
  }
  LVAE_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------------------------
// triangular solves
// ---------------------------------------------------------------------------------------------------------
// Dinv[l][k] = L_kk^-1 (64 x 64, lower; padding rows = identity), one 64-thread workgroup per (k, l): lane c
// solves L y = e_c by forward substitution (y kept in LDS column c)
template <typename T>
__global__ __launch_bounds__(64) void trsm_dinv_kernel(const T* __restrict__ Lf, int64_t ldl, int64_t sl, int n,
                                                       double* __restrict__ Dinv) {
  __shared__ double S[kPB * kPBL];
  __shared__ double Y[kPB * kPBL];
  const int k = blockIdx.x, l = blockIdx.y, c = threadIdx.x, nt = gridDim.x;
  const T* Ll = Lf + (int64_t)l * sl;
  const int k0 = k * kPB, nb = min(kPB, n - k0);
  for (int r = 0; r < kPB; ++r)
    S[r * kPBL + c] = (r < nb && c < nb) ? (c <= r ? (double)Ll[(int64_t)(k0 + r) * ldl + k0 + c] : 0.0) : (r == c ? 1.0 : 0.0);
  __syncthreads();
  for (int r = 0; r < kPB; ++r) {
    double acc = (r == c) ? 1.0 : 0.0;
    for (int q = c; q < r; ++q) acc -= S[r * kPBL + q] * Y[q * kPBL + c];
    Y[r * kPBL + c] = r >= c ? acc / S[r * kPBL + r] : 0.0;
  }
  double* D = Dinv + ((int64_t)l * nt + k) * kPB * kPB;
  for (int r = 0; r < kPB; ++r) D[r * kPB + c] = Y[r * kPBL + c];
}

// B <- op(L)^-1 B (op = L, or L^T when trans), 64-column chunk cblk of B, matrix l: block rows in dependency
// order (forward for L, backward for L^T); R = B_k - sum_j op(L)_kj X_j, X_k = op(Dinv_k) R.  The solved
// blocks are stored into B and read back by the same workgroup (workgroup-scope ordering: the barriers).
template <typename T>
__global__ __launch_bounds__(256) void trsm_sweep_kernel(int trans, int n, int nrhs, const T* __restrict__ Lf,
                                                         int64_t ldl, int64_t sl, T* __restrict__ B, int64_t ldb,
                                                         int64_t sb, const double* __restrict__ Dinv) {
  __shared__ double As[kPB * kPBL];  // [row][kk]
  __shared__ double Bs[kPB * kPBL];  // [kk][col]
  const int cblk = blockIdx.x, l = blockIdx.y, tid = threadIdx.x, nt = (n + kPB - 1) / kPB;
  const int lane = tid & 63, w = tid >> 6, li = lane & 15, lk = lane >> 4;
  const T* Ll = Lf + (int64_t)l * sl;
  T* Bl = B + (int64_t)l * sb;
  const int c0 = cblk * kPB;
  for (int s = 0; s < nt; ++s) {
    const int k = trans ? nt - 1 - s : s, k0 = k * kPB;
    bi_f64x4 acc[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) acc[cb] = bi_f64x4{0.0, 0.0, 0.0, 0.0};
    for (int q = 0; q < s; ++q) {  // the solved blocks j
      const int j = trans ? nt - 1 - q : q, j0 = j * kPB;
      for (int e = tid; e < kPB * kPB; e += 256) {
        const int r = e >> 6, c = e & 63;
        // op(L)_kj [r][c]: L[k0 + r][j0 + c] (forward) or L[j0 + c][k0 + r] (backward)
        const int gi = trans ? j0 + c : k0 + r, gj = trans ? k0 + r : j0 + c;
        As[r * kPBL + c] = (gi < n && gj < n) ? (double)Ll[(int64_t)gi * ldl + gj] : 0.0;
        Bs[r * kPBL + c] = (j0 + r < n && c0 + c < nrhs) ? (double)Bl[(int64_t)(j0 + r) * ldb + c0 + c] : 0.0;
      }
      __syncthreads();
      p64_mma(As, Bs, acc);
      __syncthreads();
    }
    // R = B_k - acc -> Bs; op(Dinv_k) -> As
    const double* D = Dinv + ((int64_t)l * nt + k) * kPB * kPB;
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * w + lk + 4 * r, col = 16 * cb + li;
        const double bv = (k0 + row < n && c0 + col < nrhs) ? (double)Bl[(int64_t)(k0 + row) * ldb + c0 + col] : 0.0;
        Bs[row * kPBL + col] = bv - acc[cb][r];
      }
    for (int e = tid; e < kPB * kPB; e += 256) {
      const int r = e >> 6, c = e & 63;
      As[r * kPBL + c] = trans ? D[c * kPB + r] : D[r * kPB + c];
    }
    __syncthreads();
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) acc[cb] = bi_f64x4{0.0, 0.0, 0.0, 0.0};
    p64_mma(As, Bs, acc);
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * w + lk + 4 * r, col = 16 * cb + li;
        if (k0 + row < n && c0 + col < nrhs) Bl[(int64_t)(k0 + row) * ldb + c0 + col] = (T)acc[cb][r];
      }
    __syncthreads();  // X_k stored before the next block row reads it; As / Bs free
  }
}

size_t trsm_ws_bytes(int n, int L) { return align256((size_t)L * cdiv(n, kPB) * kPB * kPB * sizeof(double)); }

template <typename T>
int trsm_t(int nsweep, const int* trans, int n, int nrhs, int L, const T* Lf, int64_t ldl, int64_t sl, T* B,
           int64_t ldb, int64_t sb, void* ws, hipStream_t st) {
  if (n <= 0) return -2;
  if (nrhs < 0) return -3;
  if (L <= 0) return -4;
  if (!Lf) return -5;
  if (ldl < n) return -6;
  if (!B) return -8;
  if (ldb < nrhs) return -9;
  if (!ws || ((uintptr_t)ws & 255)) return -11;
  if (nrhs == 0) return 0;
  const int nt = cdiv(n, kPB);
  double* Dinv = (double*)ws;
  trsm_dinv_kernel<T><<<dim3(nt, L), 64, 0, st>>>(Lf, ldl, sl, n, Dinv);
  for (int s = 0; s < nsweep; ++s)
    trsm_sweep_kernel<T><<<dim3(cdiv(nrhs, kPB), L), 256, 0, st>>>(trans[s], n, nrhs, Lf, ldl, sl, B, ldb, sb, Dinv);
  LVAE_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------------------------
// potrf_f32: chol_inv.hip's factorisation alone, L exported in fp32
// ---------------------------------------------------------------------------------------------------------
// the padded working matrix: Ap[l] = A[l] (lower triangle) with the identity on the padding
__global__ __launch_bounds__(256) void pf32_pad_kernel(const float* __restrict__ A, int64_t lda, int64_t sa, int n,
                                                       int np_, float* __restrict__ Ap) {
  const int l = blockIdx.y, i = blockIdx.x;
  float* o = Ap + ((int64_t)l * np_ + i) * np_;
  const float* a = A + (int64_t)l * sa + (int64_t)i * lda;
  for (int j = threadIdx.x; j <= i; j += 256) o[j] = (i < n) ? a[j] : (i == j ? 1.0f : 0.0f);
}
// Lout[l] = the lower triangle of the padded factor (zero strict upper part), cropped to n
__global__ __launch_bounds__(256) void pf32_out_kernel(const float* __restrict__ Ap, int np_, int n, float* __restrict__ Lo,
                                                       int64_t ldo, int64_t so) {
  const int l = blockIdx.y, i = blockIdx.x;
  const float* a = Ap + ((int64_t)l * np_ + i) * np_;
  float* o = Lo + (int64_t)l * so + (int64_t)i * ldo;
  for (int j = threadIdx.x; j < n; j += 256) o[j] = j <= i ? a[j] : 0.0f;
}

size_t potrf_f32_ws_bytes(int n, int L) {
  const int np_ = (n + kSwB - 1) / kSwB * kSwB;
  return align256((size_t)L * np_ * np_ * sizeof(float)) + ci_scratch_bytes(np_, L);
}

int potrf_f32(int n, int L, const float* A, int64_t lda, int64_t sa, float* Lo, int64_t ldo, int64_t so,
              double* logdet, int32_t* info, void* ws, hipStream_t st) {
  if (n <= 0) return -1;
  if (L <= 0) return -2;
  if (!A) return -3;
  if (lda < n) return -4;
  if (!Lo) return -6;
  if (ldo < n) return -7;
  if (!logdet) return -9;
  if (!info) return -10;
  if (!ws || ((uintptr_t)ws & 255)) return -11;
  const int np_ = (n + kSwB - 1) / kSwB * kSwB;
  if (np_ / kSwB > 64) return -1;
  float* Ap = (float*)ws;
  char* scratch = (char*)ws + align256((size_t)L * np_ * np_ * sizeof(float));
  pf32_pad_kernel<<<dim3(np_, L), 256, 0, st>>>(A, lda, sa, n, np_, Ap);
  LVAE_TRY(ci_potrf_f32(np_, L, Ap, scratch, logdet, info, st));
  pf32_out_kernel<<<dim3(n, L), 256, 0, st>>>(Ap, np_, n, Lo, ldo, so);
  LVAE_CHECK_LAUNCH();
  return 0;
}

}  // namespace lvae

extern "C" {
int lvae_potrf_f64(int n, int L, const double* A, int64_t lda, int64_t stride_a, double* Lout, int64_t ldo,
                   int64_t stride_o, double* logdet, int32_t* info, void* stream) {
  return lvae::potrf_f64(n, L, A, lda, stride_a, Lout, ldo, stride_o, logdet, info, (hipStream_t)stream);
}
size_t lvae_potrf_f32_workspace_size(int n, int L) { return lvae::potrf_f32_ws_bytes(n, L); }
int lvae_potrf_f32(int n, int L, const float* A, int64_t lda, int64_t stride_a, float* Lout, int64_t ldo,
                   int64_t stride_o, double* logdet, int32_t* info, void* workspace, void* stream) {
  return lvae::potrf_f32(n, L, A, lda, stride_a, Lout, ldo, stride_o, logdet, info, workspace, (hipStream_t)stream);
}
size_t lvae_trsm_workspace_size(int n, int L) { return lvae::trsm_ws_bytes(n, L); }
int lvae_trsm_f64(int trans, int n, int nrhs, int L, const double* Lf, int64_t ldl, int64_t stride_l, double* B,
                  int64_t ldb, int64_t stride_b, void* workspace, void* stream) {
  if (trans != 0 && trans != 1) return -1;
  return lvae::trsm_t<double>(1, &trans, n, nrhs, L, Lf, ldl, stride_l, B, ldb, stride_b, workspace, (hipStream_t)stream);
}
int lvae_trsm_f32(int trans, int n, int nrhs, int L, const float* Lf, int64_t ldl, int64_t stride_l, float* B,
                  int64_t ldb, int64_t stride_b, void* workspace, void* stream) {
  if (trans != 0 && trans != 1) return -1;
  return lvae::trsm_t<float>(1, &trans, n, nrhs, L, Lf, ldl, stride_l, B, ldb, stride_b, workspace, (hipStream_t)stream);
}
int lvae_potrs_f64(int n, int nrhs, int L, const double* Lf, int64_t ldl, int64_t stride_l, double* B, int64_t ldb,
                   int64_t stride_b, void* workspace, void* stream) {
  static const int tr[2] = {0, 1};
  const int rc = lvae::trsm_t<double>(2, tr, n, nrhs, L, Lf, ldl, stride_l, B, ldb, stride_b, workspace, (hipStream_t)stream);
  return rc < 0 && rc != LVAE_ERR_LAUNCH ? rc + 1 : rc;  // (argument indices of this signature: no leading trans)
}
int lvae_potrs_f32(int n, int nrhs, int L, const float* Lf, int64_t ldl, int64_t stride_l, float* B, int64_t ldb,
                   int64_t stride_b, void* workspace, void* stream) {
  static const int tr[2] = {0, 1};
  const int rc = lvae::trsm_t<float>(2, tr, n, nrhs, L, Lf, ldl, stride_l, B, ldb, stride_b, workspace, (hipStream_t)stream);
  return rc < 0 && rc != LVAE_ERR_LAUNCH ? rc + 1 : rc;
}
}
