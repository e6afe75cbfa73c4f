// potrf.hip -- blocked Cholesky, triangular inverse and SPD inverse of L batched N x N fp32
// matrices on CDNA4 (replaces torch.cholesky / cholesky_solve(I) in elbo_functions.py:26-28).
//
// Right-looking, panel width 128 (= the MFMA tile edge):
//   per panel k:  diag   : one workgroup per matrix factors the 128x128 diagonal block in LDS
//                          (4 sub-panels of 32: one-wave register factorisation + LDS trsm/syrk)
//                          and also inverts it (the diagonal block of L^-1, reused by trtri);
//                 panel  : L_ik = A_ik W_kk^T                 (MFMA, one tile per workgroup)
//                 update : A_ij -= L_ik L_jk^T, k < j <= i    (MFMA, lower tiles only)
//   trtri, block row i: W_ic = -W_ii (sum_{c<=j<i} L_ij W_jc)  (two MFMA launches per row)
//   lauum            : A^-1_IJ = sum_{K>=I} W_KI^T W_KJ, written to both triangles
// Matrices are [L][np][np] row-major, np % 128 == 0; grids are (tiles, L) so all latent dims of
// a step share every launch.
#include "mfma_tile.hpp"

namespace lvae {

constexpr int kNB = 128;
constexpr int kLs = kNB + 1;  // padded LDS row of the diagonal block

// ------------------------------------------------------------------------------------------
// diagonal block: factor + invert in LDS
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void potrf_diag_kernel(float* __restrict__ Aall, float* __restrict__ Wall, int np_,
                                                         int kb, double* __restrict__ logdet,
                                                         int32_t* __restrict__ info) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Ls = smem;                 // [128][129] factor
  float* Xs = smem + kNB * kLs;     // [128][129] inverse
  float* Ts = Xs + kNB * kLs;       // [32][97]   trtri temp (3 sub-blocks of 32)
  const int l = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  float* A = Aall + (int64_t)l * np_ * np_ + (int64_t)kb * kNB * np_ + kb * kNB;
  float* W = Wall + (int64_t)l * np_ * np_ + (int64_t)kb * kNB * np_ + kb * kNB;

  for (int e = tid; e < kNB * kNB; e += 256) {
    const int i = e >> 7, j = e & 127;
    Ls[i * kLs + j] = (j <= i) ? A[(int64_t)i * np_ + j] : 0.f;
    Xs[i * kLs + j] = 0.f;
  }
  __syncthreads();

  double ld_acc = 0.0;  // wave 0 lanes: sum of log pivots
  int fail = 0;         // wave 0 lane 0: first failing local column + 1
  for (int s = 0; s < 4; ++s) {
    const int c0 = 32 * s;
    // (a) wave 0: factor the 32x32 diagonal sub-block in registers (lane i < 32 owns row i)
    if (w == 0) {
      float row[32];
      const int i = lane & 31;
#pragma unroll
      for (int c = 0; c < 32; ++c) row[c] = Ls[(c0 + i) * kLs + c0 + c];
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        const float d = __shfl(row[j], j, 64);
        const bool bad = !(d > 0.f) || !isfinite(d);
        if (bad && fail == 0) fail = c0 + j + 1;
        const float piv = sqrtf(d);
        if (lane == j) ld_acc += log((double)piv);
        if (i > j) row[j] /= piv;
        else if (i == j) row[j] = piv;
#pragma unroll
        for (int c = j + 1; c < 32; ++c) {
          const float lcj = __shfl(row[j], c, 64);
          if (i >= c) row[c] -= row[j] * lcj;
        }
      }
      if (lane < 32) {
#pragma unroll
        for (int c = 0; c < 32; ++c) Ls[(c0 + i) * kLs + c0 + c] = (c <= i) ? row[c] : 0.f;
      }
      // inverse of the 32x32 lower block: lane c computes column c (forward substitution)
      float xc[32];
      const int c = lane & 31;
#pragma unroll
      for (int r = 0; r < 32; ++r) {
        float acc = (r == c) ? 1.f : 0.f;
#pragma unroll
        for (int k = 0; k < r; ++k) acc -= Ls[(c0 + r) * kLs + c0 + k] * xc[k];
        xc[r] = acc / Ls[(c0 + r) * kLs + c0 + r];
      }
      if (lane < 32) {
#pragma unroll
        for (int r = 0; r < 32; ++r) Xs[(c0 + r) * kLs + c0 + c] = xc[r];
      }
    }
    __syncthreads();
    const int R = kNB - c0 - 32;  // rows below the sub-panel
    if (R > 0) {
      // (b) sub-panel below: L[i][c0+c] = sum_{k<=c} A[i][c0+k] X[c0+c][c0+k]
      float outv[12];
      const int c = tid & 31, rbase = tid >> 5;
#pragma unroll
      for (int q = 0; q < 12; ++q) {
        const int i = c0 + 32 + rbase + 8 * q;
        float acc = 0.f;
        if (i < kNB) {
#pragma unroll 8
          for (int k = 0; k < 32; ++k) acc += Ls[i * kLs + c0 + k] * Xs[(c0 + c) * kLs + c0 + k];
        }
        outv[q] = acc;
      }
      __syncthreads();
#pragma unroll
      for (int q = 0; q < 12; ++q) {
        const int i = c0 + 32 + rbase + 8 * q;
        if (i < kNB) Ls[i * kLs + c0 + c] = outv[q];
      }
      __syncthreads();
      // (c) rank-32 update of the remaining lower triangle
      for (int e = tid; e < R * R; e += 256) {
        const int ii = e / R, jj = e - ii * R;
        if (jj > ii) continue;
        const int i = c0 + 32 + ii, j = c0 + 32 + jj;
        float acc = 0.f;
#pragma unroll 8
        for (int k = 0; k < 32; ++k) acc += Ls[i * kLs + c0 + k] * Ls[j * kLs + c0 + k];
        Ls[i * kLs + j] -= acc;
      }
      __syncthreads();
    }
  }
  // off-diagonal 32x32 blocks of the inverse: X_IJ = -X_II sum_{J<=K<I} L_IK X_KJ
  for (int I = 1; I < 4; ++I) {
    const int n_el = I * 32 * 32;  // all J < I
    for (int e = tid; e < n_el; e += 256) {
      const int J = e >> 10, r = (e >> 5) & 31, c = e & 31;
      float acc = 0.f;
      for (int k = 32 * J; k < 32 * I; ++k) acc += Ls[(32 * I + r) * kLs + k] * Xs[k * kLs + 32 * J + c];
      Ts[r * 97 + 32 * J + c] = acc;
    }
    __syncthreads();
    for (int e = tid; e < n_el; e += 256) {
      const int J = e >> 10, r = (e >> 5) & 31, c = e & 31;
      float acc = 0.f;
      for (int k = 0; k <= r; ++k) acc += Xs[(32 * I + r) * kLs + 32 * I + k] * Ts[k * 97 + 32 * J + c];
      Xs[(32 * I + r) * kLs + 32 * J + c] = -acc;
    }
    __syncthreads();
  }
  // write back: L (lower) into A, L^-1 (lower, zero upper) into W
  for (int e = tid; e < kNB * kNB; e += 256) {
    const int i = e >> 7, j = e & 127;
    if (j <= i) A[(int64_t)i * np_ + j] = Ls[i * kLs + j];
    W[(int64_t)i * np_ + j] = (j <= i) ? Xs[i * kLs + j] : 0.f;
  }
  if (w == 0) {
    const double sld = wave_sum(ld_acc);
    if (lane == 0) {
      logdet[l] += 2.0 * sld;
      if (fail && info[l] == 0) info[l] = kb * kNB + fail;
    }
  }
}

constexpr size_t kDiagLds = (2 * kNB * kLs + 32 * 97) * sizeof(float);

// ------------------------------------------------------------------------------------------
// panel: L_ik = A_ik W_kk^T for tile rows i > kb
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void potrf_panel_kernel(float* __restrict__ Aall, const float* __restrict__ Wall,
                                                          int np_, int kb) {
  __shared__ __attribute__((aligned(16))) float lds[tile_lds_floats<true, true>()];
  const int l = blockIdx.y, i = kb + 1 + blockIdx.x;
  float* A = Aall + (int64_t)l * np_ * np_;
  const float* W = Wall + (int64_t)l * np_ * np_;
  float* Aik = A + (int64_t)i * kNB * np_ + kb * kNB;
  const float* Wkk = W + (int64_t)kb * kNB * np_ + kb * kNB;
  Frag f;
  f.zero();
  tile_gemm<true, true>(Aik, np_, Wkk, np_, 0, kNB, f, lds);
  __syncthreads();
  frag_foreach(f, [&](int r, int c, float v) { Aik[(int64_t)r * np_ + c] = v; });
}

// trailing update: A_ij -= L_i,kb L_j,kb^T, kb < j <= i
__device__ inline void tri_index2(int t, int& I, int& J) {
  int r = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
  while ((r + 1) * (r + 2) / 2 <= t) ++r;
  while (r * (r + 1) / 2 > t) --r;
  I = r;
  J = t - r * (r + 1) / 2;
}

__global__ __launch_bounds__(256) void potrf_update_kernel(float* __restrict__ Aall, int np_, int kb) {
  __shared__ __attribute__((aligned(16))) float lds[tile_lds_floats<true, true>()];
  int I, J;
  tri_index2(blockIdx.x, I, J);
  const int l = blockIdx.y, i = kb + 1 + I, j = kb + 1 + J;
  float* A = Aall + (int64_t)l * np_ * np_;
  const float* Li = A + (int64_t)i * kNB * np_ + kb * kNB;
  const float* Lj = A + (int64_t)j * kNB * np_ + kb * kNB;
  Frag f;
  f.zero();
  tile_gemm<true, true>(Li, np_, Lj, np_, 0, kNB, f, lds);
  float* C = A + (int64_t)i * kNB * np_ + j * kNB;
  frag_foreach(f, [&](int r, int c, float v) { C[(int64_t)r * np_ + c] -= v; });
}

// ------------------------------------------------------------------------------------------
// trtri: block row i (i >= 1).  step 1: W_ic <- sum_{c<=j<i} L_ij W_jc ; step 2: W_ic <- -W_ii W_ic
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void trtri_step1_kernel(const float* __restrict__ Aall, float* __restrict__ Wall,
                                                          int np_, int ib) {
  __shared__ __attribute__((aligned(16))) float lds[tile_lds_floats<true, false>()];
  const int l = blockIdx.y, c = blockIdx.x;
  const float* A = Aall + (int64_t)l * np_ * np_;
  float* W = Wall + (int64_t)l * np_ * np_;
  Frag f;
  f.zero();
  // op(A)(m,k) = L[ib*128 + m][k], op(B)(k,n) = W[k][c*128 + n], k in [c*128, ib*128)
  tile_gemm<true, false>(A + (int64_t)ib * kNB * np_, np_, W + c * kNB, np_, c * kNB, ib * kNB, f, lds);
  float* C = W + (int64_t)ib * kNB * np_ + c * kNB;
  frag_foreach(f, [&](int r, int cc, float v) { C[(int64_t)r * np_ + cc] = v; });
}

__global__ __launch_bounds__(256) void trtri_step2_kernel(float* __restrict__ Wall, int np_, int ib) {
  __shared__ __attribute__((aligned(16))) float lds[tile_lds_floats<true, false>()];
  const int l = blockIdx.y, c = blockIdx.x;
  float* W = Wall + (int64_t)l * np_ * np_;
  const float* Wii = W + (int64_t)ib * kNB * np_ + ib * kNB;
  float* C = W + (int64_t)ib * kNB * np_ + c * kNB;
  Frag f;
  f.zero();
  tile_gemm<true, false>(Wii, np_, C, np_, 0, kNB, f, lds);
  __syncthreads();
  frag_foreach(f, [&](int r, int cc, float v) { C[(int64_t)r * np_ + cc] = -v; });
}

// ------------------------------------------------------------------------------------------
// lauum: Ainv_IJ = sum_{K >= I} W_KI^T W_KJ (I >= J), mirrored into the upper triangle
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void lauum_kernel(const float* __restrict__ Wall, float* __restrict__ Ball,
                                                    int np_) {
  __shared__ __attribute__((aligned(16))) float lds[tile_lds_floats<false, false>()];
  int I, J;
  tri_index2(blockIdx.x, I, J);
  const int l = blockIdx.y;
  const float* W = Wall + (int64_t)l * np_ * np_;
  float* B = Ball + (int64_t)l * np_ * np_;
  Frag f;
  f.zero();
  tile_gemm<false, false>(W + I * kNB, np_, W + J * kNB, np_, I * kNB, np_, f, lds);
  float* C = B + (int64_t)I * kNB * np_ + J * kNB;
  float* Ct = B + (int64_t)J * kNB * np_ + I * kNB;
  const bool mirror = I != J;
  frag_foreach(f, [&](int r, int c, float v) {
    C[(int64_t)r * np_ + c] = v;
    if (mirror) Ct[(int64_t)c * np_ + r] = v;
  });
}

// ------------------------------------------------------------------------------------------
// S = B diag(v) B (lower tiles), B symmetric: S_IJ = sum_k B[I m][k] v_k B[J n][k]
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void syrk_scaled_kernel(const float* __restrict__ Ball, const float* __restrict__ vall,
                                                          float* __restrict__ Sall, int np_) {
  __shared__ __attribute__((aligned(16))) float lds[tile_lds_floats<true, true>()];
  int I, J;
  tri_index2(blockIdx.x, I, J);
  const int l = blockIdx.y;
  const float* B = Ball + (int64_t)l * np_ * np_;
  const float* v = vall + (int64_t)l * np_;
  Frag f;
  f.zero();
  tile_gemm<true, true>(B + (int64_t)I * kNB * np_, np_, B + (int64_t)J * kNB * np_, np_, 0, np_, f, lds, v);
  float* C = Sall + (int64_t)l * np_ * np_ + (int64_t)I * kNB * np_ + J * kNB;
  frag_foreach(f, [&](int r, int c, float val) { C[(int64_t)r * np_ + c] = val; });
}

// ------------------------------------------------------------------------------------------
// host sequencing
// ------------------------------------------------------------------------------------------
int potrf_f32(int np_, int L, float* A, float* W, double* logdet, int32_t* info, hipStream_t st) {
  if (np_ <= 0 || np_ % kNB) return -1;
  if (L <= 0) return -2;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)potrf_diag_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kDiagLds);
    attr_set = true;
  }
  (void)hipMemsetAsync(logdet, 0, sizeof(double) * L, st);
  (void)hipMemsetAsync(info, 0, sizeof(int32_t) * L, st);
  const int nt = np_ / kNB;
  for (int kb = 0; kb < nt; ++kb) {
    potrf_diag_kernel<<<L, 256, kDiagLds, st>>>(A, W, np_, kb, logdet, info);
    const int T = nt - kb - 1;
    if (T > 0) {
      potrf_panel_kernel<<<dim3(T, L), 256, 0, st>>>(A, W, np_, kb);
      potrf_update_kernel<<<dim3(T * (T + 1) / 2, L), 256, 0, st>>>(A, np_, kb);
    }
  }
  LVAE_CHECK_LAUNCH();
  return 0;
}

int potri_f32(int np_, int L, const float* A, float* W, float* Ainv, hipStream_t st) {
  if (np_ <= 0 || np_ % kNB) return -1;
  const int nt = np_ / kNB;
  for (int ib = 1; ib < nt; ++ib) {
    trtri_step1_kernel<<<dim3(ib, L), 256, 0, st>>>(A, W, np_, ib);
    trtri_step2_kernel<<<dim3(ib, L), 256, 0, st>>>(W, np_, ib);
  }
  lauum_kernel<<<dim3(nt * (nt + 1) / 2, L), 256, 0, st>>>(W, Ainv, np_);
  LVAE_CHECK_LAUNCH();
  return 0;
}

int syrk_scaled_f32(int np_, int L, const float* B, const float* v, float* S, hipStream_t st) {
  const int nt = np_ / kNB;
  syrk_scaled_kernel<<<dim3(nt * (nt + 1) / 2, L), 256, 0, st>>>(B, v, S, np_);
  LVAE_CHECK_LAUNCH();
  return 0;
}

}  // namespace lvae

extern "C" {
int lvae_potrf_f32(int np_, int L, float* A, float* W, double* logdet, int32_t* info, void* stream) {
  return lvae::potrf_f32(np_, L, A, W, logdet, info, (hipStream_t)stream);
}
int lvae_potri_f32(int np_, int L, const float* A, float* W, float* Ainv, void* stream) {
  return lvae::potri_f32(np_, L, A, W, Ainv, (hipStream_t)stream);
}
}
