// sweep.hpp -- SPD inverse + log-determinant of a small (<= 128) matrix held entirely in the MFMA
// accumulators of one workgroup (chol_inverse below): blocked Cholesky and two blocked triangular
// solves, 4 columns per step, each step one rank-4 update = one 16x16x4 MFMA per 16x16 tile
// (v_mfma_f32_16x16x4_f32 / v_mfma_f64_16x16x4_f64); one LDS panel + one barrier per step.
#pragma once
#include "common.hpp"

namespace lvae {

typedef float sw_f32x4 __attribute__((ext_vector_type(4)));
typedef double sw_f64x4 __attribute__((ext_vector_type(4)));

template <typename T>
struct SweepTraits;
template <>
struct SweepTraits<float> {
  typedef sw_f32x4 acc_t;
  // C/D layout of v_mfma_f32_16x16x4_f32: row = (lane>>4)*4 + r, col = lane & 15
  __device__ static inline int row(int lane, int r) { return ((lane >> 4) << 2) + r; }
  __device__ static inline acc_t mfma(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
};
template <>
struct SweepTraits<double> {
  typedef sw_f64x4 acc_t;
  // C/D layout of v_mfma_f64_16x16x4_f64: row = (lane>>4) + 4 r, col = lane & 15
  __device__ static inline int row(int lane, int r) { return (lane >> 4) + (r << 2); }
  __device__ static inline acc_t mfma(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
};

// 4x4 Cholesky of the pivot block (lower, in registers) and the inverse of its factor (only 4
// divisions).  first_bad: first non-positive pivot (0..3) or -1.
template <typename T>
__device__ inline void chol4(const T (&P)[4][4], T (&Lp)[4][4], T (&Li)[4][4], int& first_bad) {
  first_bad = -1;
  T ik[4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) Lp[a][b] = T(0), Li[a][b] = T(0);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    T d = P[k][k];
#pragma unroll
    for (int m = 0; m < k; ++m) d -= Lp[k][m] * Lp[k][m];
    if (first_bad < 0 && (!(d > T(0)) || !isfinite(d))) first_bad = k;
    const T lkk = sqrt(d);
    Lp[k][k] = lkk;
    ik[k] = T(1) / lkk;
#pragma unroll
    for (int i = k + 1; i < 4; ++i) {
      T v = P[i][k];
#pragma unroll
      for (int m = 0; m < k; ++m) v -= Lp[i][m] * Lp[k][m];
      Lp[i][k] = v * ik[k];
    }
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    Li[c][c] = ik[c];
#pragma unroll
    for (int r = c + 1; r < 4; ++r) {
      T v = T(0);
#pragma unroll
      for (int m = c; m < r; ++m) v += Lp[r][m] * Li[m][c];
      Li[r][c] = -v * ik[r];
    }
  }
}

// v[idx] for a runtime idx in [0,4) by selects (runtime-indexed register arrays go to scratch)
template <typename T>
__device__ inline T pick4(T v0, T v1, T v2, T v3, int idx) {
  return idx == 0 ? v0 : (idx == 1 ? v1 : (idx == 2 ? v2 : v3));
}

// Shared memory of chol_inverse (the factor L is kept in LDS for the two solve passes).
template <typename T, int TS>
struct CholInvLds {
  static constexpr int NP = 16 * TS, LDL = NP + 1;
  T Ls[NP * LDL];
  T cpanel[2][NP][4];   // column block K (pass 1)
  T rpanel[2][4][NP];   // row block K (passes 2, 3)
  T Lpi[NP / 4][4][4];  // inverse of each 4x4 diagonal factor block
  T pdiag[NP];          // diagonal of L (log-determinant at the end)
  double red[16];
};

// One workgroup (64 * TS * TS / TPW threads) inverts one SPD matrix, fully in MFMA accumulators:
//   pass 1  blocked Cholesky, 4 columns per step: A_ij -= L_iK L_jK^T (one 16x16x4 MFMA per tile)
//   pass 2  Y = L^-1 : Y_K <- Lp^-1 Y_K ; Y_i -= L_iK Y_K      (i > K)
//   pass 3  X = L^-T Y: X_K <- Lp^-T X_K ; X_i -= L_Ki^T X_K   (i < K, K descending)
// Cholesky + triangular solves are backward stable.  Matrix padded to NP = 16 TS with identity;
// a wave owns TPW consecutive 16x16 tiles of one tile row.  Per-lane coefficient rows are picked
// once per step (lane group lg = lane >> 4 is the MFMA k index), keeping the step short.
//   in : element (i, j) at in[i * ldi + j], i, j < n; only the lower triangle is read
//   out: A^-1 element (i, j) at out[i * ldo + j]
//   logdet: log|A| (accumulate = 1: +=);  info: first bad pivot column + col_offset
template <typename T, int TS, int TPW>
__device__ inline void chol_inverse(int n, const T* __restrict__ in, int64_t ldi, T* __restrict__ out, int64_t ldo,
                                    double* __restrict__ logdet, int accumulate, int32_t* __restrict__ info,
                                    int col_offset) {
  typedef SweepTraits<T> Tr;
  typedef typename Tr::acc_t acc_t;
  constexpr int NP = 16 * TS, WPR = TS / TPW, NSTEP = NP / 4, LDL = NP + 1;
  __shared__ CholInvLds<T, TS> sm;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const int tr = w / WPR, tc0 = (w % WPR) * TPW;
  const int lc = lane & 15, lg = lane >> 4;
  acc_t acc[TPW];
#pragma unroll
  for (int u = 0; u < TPW; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = tr * 16 + Tr::row(lane, r), j = (tc0 + u) * 16 + lc;
      const int64_t off = (j <= i) ? (int64_t)i * ldi + j : (int64_t)j * ldi + i;
      acc[u][r] = (i < n && j < n) ? in[off] : (i == j ? T(1) : T(0));
    }
  // ---------------- pass 1: Cholesky ----------------
// (macros, not lambdas: a lambda capturing the accumulator array by reference made hipcc keep it
//  in scratch)
#define LVAE_PUBLISH_COL(PP)                                                                              \
  do {                                                                                                    \
    const int tcK_ = (PP) >> 2, c0_ = ((PP)&3) << 2;                                                      \
    if (tcK_ >= tc0 && tcK_ < tc0 + TPW && lc >= c0_ && lc < c0_ + 4) {                                   \
      _Pragma("unroll") for (int uu = 0; uu < TPW; ++uu) if (uu == tcK_ - tc0) {                          \
        _Pragma("unroll") for (int r = 0; r < 4; ++r) sm.cpanel[(PP)&1][tr * 16 + Tr::row(lane, r)][lc - c0_] = \
            acc[uu][r];                                                                                   \
      }                                                                                                   \
    }                                                                                                     \
  } while (0)
#define LVAE_PUBLISH_ROW(PP)                                                                              \
  do {                                                                                                    \
    const int K0_ = 4 * (PP);                                                                             \
    if (tr == (K0_ >> 4)) {                                                                               \
      _Pragma("unroll") for (int u = 0; u < TPW; ++u) {                                                   \
        _Pragma("unroll") for (int r = 0; r < 4; ++r) {                                                   \
          const int i_ = tr * 16 + Tr::row(lane, r);                                                      \
          if (i_ >= K0_ && i_ < K0_ + 4) sm.rpanel[(PP)&1][i_ - K0_][(tc0 + u) * 16 + lc] = acc[u][r];    \
        }                                                                                                 \
      }                                                                                                   \
    }                                                                                                     \
  } while (0)
  LVAE_PUBLISH_COL(0);
  __syncthreads();
  int fail = 0;
  for (int p = 0; p < NSTEP; ++p) {
    const T(*pn)[4] = sm.cpanel[p & 1];
    const int K0 = 4 * p;
    T P[4][4], Lp[4][4], Li[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) P[a][b] = pn[K0 + a][b];
    int fb;
    chol4<T>(P, Lp, Li, fb);
    if (t == 0) {
      if (!fail && fb >= 0) fail = K0 + fb + 1;
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        sm.pdiag[K0 + a] = Lp[a][a];
#pragma unroll
        for (int b = 0; b < 4; ++b) sm.Lpi[p][a][b] = Li[a][b];
      }
    }
    // L_iK[m] = sum_k A_iK[k] Li[m][k]; this lane's m = lg
    T cA[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) cA[k] = pick4(Li[0][k], Li[1][k], Li[2][k], Li[3][k], lg);
    const int ia = tr * 16 + lc;
    T aop = T(0);
    if (ia >= K0 + 4) {
#pragma unroll
      for (int k = 0; k < 4; ++k) aop += pn[ia][k] * cA[k];
    }
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
      const int jb = (tc0 + u) * 16 + lc;
      T bop = T(0);
#pragma unroll
      for (int k = 0; k < 4; ++k) bop += pn[jb][k] * cA[k];
      bop = (jb >= K0 + 4) ? bop : T(0);
      acc[u] = Tr::mfma(-aop, bop, acc[u]);
    }
    // column block K becomes L_iK (rows >= K0); this lane's column in the block: b = lc - c0
    const int tcK = K0 >> 4, c0 = K0 & 15;
    if (tcK >= tc0 && tcK < tc0 + TPW) {
      const int b = lc - c0;
      const bool inb = (b >= 0 && b < 4);
      const int bb = inb ? b : 0;
      T cB[4], lpb[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        cB[k] = pick4(Li[0][k], Li[1][k], Li[2][k], Li[3][k], bb);
        lpb[k] = pick4(Lp[k][0], Lp[k][1], Lp[k][2], Lp[k][3], bb);
      }
#pragma unroll
      for (int uu = 0; uu < TPW; ++uu)
        if (uu == tcK - tc0) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = tr * 16 + Tr::row(lane, r);
            T v = T(0);
#pragma unroll
            for (int k = 0; k < 4; ++k) v += pn[i][k] * cB[k];
            const int ii = i - K0;
            const T vin = pick4(lpb[0], lpb[1], lpb[2], lpb[3], (ii >= 0 && ii < 4) ? ii : 0);
            if (inb && i >= K0) acc[uu][r] = (ii < 4) ? vin : v;
          }
        }
    }
    if (p + 1 < NSTEP) LVAE_PUBLISH_COL(p + 1);
    __syncthreads();
  }
  // L (lower, zero upper) into LDS
#pragma unroll
  for (int u = 0; u < TPW; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = tr * 16 + Tr::row(lane, r), j = (tc0 + u) * 16 + lc;
      sm.Ls[i * LDL + j] = (j <= i) ? acc[u][r] : T(0);
    }
  // ---------------- pass 2: Y = L^-1 (acc <- I) ----------------
#pragma unroll
  for (int u = 0; u < TPW; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = tr * 16 + Tr::row(lane, r), j = (tc0 + u) * 16 + lc;
      acc[u][r] = (i == j) ? T(1) : T(0);
    }
  // one solve pass: acc_i -= coef(i) * z_K, rows K <- z_K, z_K[m][j] = sum_k C[m][k] rp[k][j]
  //   pass 2: C = Lpi[p],   coef(i) = L[i][K0+m] (i > K)
  //   pass 3: C = Lpi[p]^T, coef(i) = L[K0+m][i] (i < K)
  LVAE_PUBLISH_ROW(0);
  __syncthreads();
  for (int p = 0; p < NSTEP; ++p) {
    constexpr bool fwd = true;
    const int K0 = 4 * p;
    const T(*rp)[NP] = sm.rpanel[p & 1];
    T cm[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) cm[k] = fwd ? sm.Lpi[p][lg][k] : sm.Lpi[p][k][lg];
    const int ia = tr * 16 + lc;
    const bool act = fwd ? (ia >= K0 + 4) : (ia < K0);
    const T aop = act ? (fwd ? sm.Ls[ia * LDL + K0 + lg] : sm.Ls[(K0 + lg) * LDL + ia]) : T(0);
    T zb[TPW];
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
      const int jb = (tc0 + u) * 16 + lc;
      T z = T(0);
#pragma unroll
      for (int k = 0; k < 4; ++k) z += cm[k] * rp[k][jb];
      zb[u] = z;
      acc[u] = Tr::mfma(-aop, z, acc[u]);
    }
    if (tr == (K0 >> 4)) {
#pragma unroll
      for (int u = 0; u < TPW; ++u) {
        const int jb = (tc0 + u) * 16 + lc;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = tr * 16 + Tr::row(lane, r);
          const int m = i - K0;
          if (m >= 0 && m < 4) {
            if (m == lg) {
              acc[u][r] = zb[u];
            } else {
              T z = T(0);
#pragma unroll
              for (int k = 0; k < 4; ++k) z += (fwd ? sm.Lpi[p][m][k] : sm.Lpi[p][k][m]) * rp[k][jb];
              acc[u][r] = z;
            }
          }
        }
      }
    }
    if (p + 1 < NSTEP) LVAE_PUBLISH_ROW(p + 1);
    __syncthreads();
  }
  // ---------------- pass 3: X = L^-T Y, pivot blocks descending ----------------
  LVAE_PUBLISH_ROW(NSTEP - 1);
  __syncthreads();
  for (int p = NSTEP - 1; p >= 0; --p) {
    constexpr bool fwd = false;
    const int K0 = 4 * p;
    const T(*rp)[NP] = sm.rpanel[p & 1];
    T cm[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) cm[k] = fwd ? sm.Lpi[p][lg][k] : sm.Lpi[p][k][lg];
    const int ia = tr * 16 + lc;
    const bool act = fwd ? (ia >= K0 + 4) : (ia < K0);
    const T aop = act ? (fwd ? sm.Ls[ia * LDL + K0 + lg] : sm.Ls[(K0 + lg) * LDL + ia]) : T(0);
    T zb[TPW];
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
      const int jb = (tc0 + u) * 16 + lc;
      T z = T(0);
#pragma unroll
      for (int k = 0; k < 4; ++k) z += cm[k] * rp[k][jb];
      zb[u] = z;
      acc[u] = Tr::mfma(-aop, z, acc[u]);
    }
    if (tr == (K0 >> 4)) {
#pragma unroll
      for (int u = 0; u < TPW; ++u) {
        const int jb = (tc0 + u) * 16 + lc;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = tr * 16 + Tr::row(lane, r);
          const int m = i - K0;
          if (m >= 0 && m < 4) {
            if (m == lg) {
              acc[u][r] = zb[u];
            } else {
              T z = T(0);
#pragma unroll
              for (int k = 0; k < 4; ++k) z += (fwd ? sm.Lpi[p][m][k] : sm.Lpi[p][k][m]) * rp[k][jb];
              acc[u][r] = z;
            }
          }
        }
      }
    }
    if (p > 0) LVAE_PUBLISH_ROW(p - 1);
    __syncthreads();
  }
#undef LVAE_PUBLISH_COL
#undef LVAE_PUBLISH_ROW
#pragma unroll
  for (int u = 0; u < TPW; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = tr * 16 + Tr::row(lane, r), j = (tc0 + u) * 16 + lc;
      if (i < n && j < n) out[(int64_t)i * ldo + j] = acc[u][r];
    }
  // log|A| = 2 sum log L_ii  (off the step critical path)
  double lgd = 0.0;
  for (int i = t; i < NP; i += 64 * TS * TS / TPW) lgd += log((double)sm.pdiag[i]);
  lgd = wave_sum(lgd);
  if (lane == 0) sm.red[w] = lgd;
  __syncthreads();
  if (t == 0) {
    double ld = 0.0;
    for (int q = 0; q < TS * TS / TPW; ++q) ld += sm.red[q];
    ld *= 2.0;
    if (accumulate) *logdet += ld;
    else *logdet = ld;
    if (info) {
      if (accumulate) {
        if (fail && *info == 0) *info = col_offset + fail;
      } else {
        *info = fail ? col_offset + fail : 0;
      }
    }
  }
}

}  // namespace lvae
