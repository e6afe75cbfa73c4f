// blkinv.hpp -- SPD inverse + log-determinant of a small (n <= 128) matrix by ONE workgroup, the
// whole matrix held in MFMA accumulators (16x16 tiles, v_mfma_{f32,f64}_16x16x4), 16-wide blocks:
//
//   pass 1  block Cholesky:  L_kk = chol(A_kk), L_ik = A_ik L_kk^-T (substitution), A_ij -= L_ik L_jk^T
//   pass 2  Y = L^-1         (block forward substitution on I: Y_k <- X_k Y_k, Y_i -= L_ik Y_k)
//   pass 3  A^-1 = L^-T Y    (block backward substitution: R_k <- X_k^T R_k, R_i -= L_ki^T R_k)
//
// Each 16x16 pivot block is factored by one wave entirely in registers (chol16_trinv): a
// right-looking Cholesky with the factor inverse X = L^-1 built alongside by forward substitution.
// Column broadcasts inside a 16-lane row use DPP row_newbcast, the two cross-row transfers per pivot
// (row J's values to every lane group) v_permlane32_swap + v_permlane16_swap: no LDS round trip.  In fp64 the panel L_ik is formed by
// substitution, as LAPACK's potrf (trsm) does; only the diagonal-block solves of passes 2/3 use the
// explicit X_k (as LAPACK's blocked trtri).  Explicit-inverse panels (X_k or D_k^-1 = X_k^T X_k) or a
// Gauss-Jordan sweep lose 1.5 to 5 digits at cond ~1e8 (K0zz with its 1e-6 jitter; scripts/micro).
//
// Barriers: 2 per block step in pass 1, 1 in passes 2 and 3 (32 at n = 128, vs 96 steps of the
// four-column element-wise formulation); the pivot-block factorisation is the only serial part.
//
// MFMA operand convention (both dtypes): chunk c of a 16x16x16 product uses, in lane l, the
// k-index kap(l, c) = row(l, c) of the accumulator layout, so the accumulator of a transposed
// product IS the A operand of the next product, and any accumulator tile is directly a B operand.
#pragma once
#include "common.hpp"

namespace lvae {

typedef float bi_f32x4 __attribute__((ext_vector_type(4)));
typedef double bi_f64x4 __attribute__((ext_vector_type(4)));

template <int J>
__device__ inline int bi_dpp_bcast(int v) {  // lane J of each 16-lane row -> the whole row
  return __builtin_amdgcn_update_dpp(0, v, 0x150 + J, 0xF, 0xF, false);
}

template <typename T>
struct BiTraits;
template <>
struct BiTraits<float> {
  typedef bi_f32x4 acc_t;
  // v_mfma_f32_16x16x4_f32: C[4 (lane >> 4) + r][lane & 15]
  __device__ static inline int row(int lane, int r) { return ((lane >> 4) << 2) + r; }
  static constexpr int grp(int i) { return i >> 2; }  // lane group holding row i
  static constexpr int reg(int i) { return i & 3; }   // accumulator register holding row i
  __device__ static inline acc_t mfma(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  template <int J>
  __device__ static inline float bcast16(float v) {
    return __int_as_float(bi_dpp_bcast<J>(__float_as_int(v)));
  }
  __device__ static inline float rdlane(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
  }
};
template <>
struct BiTraits<double> {
  typedef bi_f64x4 acc_t;
  // v_mfma_f64_16x16x4_f64: C[(lane >> 4) + 4 r][lane & 15]
  __device__ static inline int row(int lane, int r) { return (lane >> 4) + (r << 2); }
  static constexpr int grp(int i) { return i & 3; }
  static constexpr int reg(int i) { return i >> 2; }
  __device__ static inline acc_t mfma(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  template <int J>
  __device__ static inline double bcast16(double v) {
    const long long u = __double_as_longlong(v);
    const int lo = bi_dpp_bcast<J>((int)u), hi = bi_dpp_bcast<J>((int)(u >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
  }
  __device__ static inline double rdlane(double v, int l) {
    const long long u = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)u, l), hi = __builtin_amdgcn_readlane((int)(u >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
  }
};

// lane (G, c) -> every lane (., c): the 16-lane group G's values in all four groups, by two half
// exchanges (v_permlane32_swap of v with itself duplicates a half, v_permlane16_swap then a row of it)
// instead of a ds_bpermute round trip through the LDS crossbar
template <int G>
__device__ inline unsigned bi_group_bcast32(unsigned v) {
  const auto a = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  const unsigned h = (G >> 1) ? a[1] : a[0];
  const auto b = __builtin_amdgcn_permlane16_swap(h, h, false, false);
  return (G & 1) ? b[1] : b[0];
}
template <int G>
__device__ inline float bi_group_bcast(float v) {
  return __uint_as_float(bi_group_bcast32<G>(__float_as_uint(v)));
}
template <int G>
__device__ inline double bi_group_bcast(double v) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = bi_group_bcast32<G>((unsigned)u), hi = bi_group_bcast32<G>((unsigned)(u >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

template <typename T>
__device__ inline T bi_pick4(T v0, T v1, T v2, T v3, int idx) {
  return idx == 0 ? v0 : (idx == 1 ? v1 : (idx == 2 ? v2 : v3));
}

// Pivot J of the in-register 16x16 Cholesky: s = trailing Schur complement (full symmetric tile),
// x = rows of L^-1 built so far.  pd[J] = L_JJ; bad = first non-positive pivot.
template <typename T, int J>
struct Chol16Step {
  typedef BiTraits<T> Tr;
  typedef typename Tr::acc_t acc_t;
  __device__ __attribute__((always_inline)) static inline void run(acc_t& s, acc_t& x, int lane, const int (&irow)[4],
                                                                   T* __restrict__ pd, T* __restrict__ lk,
                                                                   T* __restrict__ ipv, int& bad) {
    constexpr int gj = Tr::grp(J), rj = Tr::reg(J);
    const int lc = lane & 15;
    const T d = Tr::rdlane(s[rj], gj * 16 + J);
    if (bad < 0 && !(d > T(0) && isfinite(d))) bad = J;
    const T p = sqrt(d), ip = T(1) / p;
    T cI[4];  // L[i][J] for this lane's rows i
#pragma unroll
    for (int r = 0; r < 4; ++r) cI[r] = Tr::template bcast16<J>(s[r]) * ip;
    // L[c][J] (c = lc) = s[J][c] / L_JJ by the symmetry of the Schur complement (both triangles are
    // updated with the same products): row J's value in column c, held by group gj, broadcast to the
    // other groups; likewise X[J][c] (final)
    const T cC = bi_group_bcast<gj>(s[rj]) * ip;
    const T xj = bi_group_bcast<gj>(x[rj] * ip);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = irow[r];
      s[r] = (i > J && lc > J) ? s[r] - cI[r] * cC : s[r];
      x[r] = (i > J) ? x[r] - cI[r] * xj : (i == J ? xj : x[r]);
    }
    if (lc == J) {  // column J of L_kk (rows >= J) for the panel substitution of pass 1
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (irow[r] >= J) lk[irow[r] * 17 + J] = cI[r];
    }
    if (lane == 0) {
      pd[J] = p;
      ipv[J] = ip;
    }
    Chol16Step<T, J + 1>::run(s, x, lane, irow, pd, lk, ipv, bad);
  }
};
template <typename T>
struct Chol16Step<T, 16> {
  __device__ static inline void run(typename BiTraits<T>::acc_t&, typename BiTraits<T>::acc_t&, int, const int (&)[4],
                                    T*, T*, T*, int&) {}
};

// One wave: Cholesky of the SPD 16x16 tile s (accumulator layout); writes X = L^-1 (lower) to
// xout[m * 17 + c], L (lower) to lk[m * 17 + c], 1 / L_jj to ipv[0..16) and the pivots L_jj to
// pd[0..16).  Returns the first bad pivot (0..15) or -1.
template <typename T>
__device__ __attribute__((always_inline)) inline int chol16_trinv(typename BiTraits<T>::acc_t s, T* __restrict__ xout,
                                                                  T* __restrict__ lk, T* __restrict__ ipv,
                                                                  T* __restrict__ pd) {
  typedef BiTraits<T> Tr;
  typedef typename Tr::acc_t acc_t;
  const int lane = threadIdx.x & 63, lc = lane & 15;
  int irow[4];
  acc_t x;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    irow[r] = Tr::row(lane, r);
    x[r] = (irow[r] == lc) ? T(1) : T(0);
  }
  int bad = -1;
  Chol16Step<T, 0>::run(s, x, lane, irow, pd, lk, ipv, bad);
#pragma unroll
  for (int r = 0; r < 4; ++r) xout[irow[r] * 17 + lc] = x[r];
  return bad;
}

// a (accumulator layout, rows of one tile row) <- a L^-T for the lower 16x16 L given by its
// columns lk[m * 17 + j] and 1 / L_jj in ipv: column j is final once the columns < j are
// eliminated; it is broadcast along each 16-lane row and subtracted from the columns > j.
template <typename T, int J>
__device__ __attribute__((always_inline)) inline void bi_panel_solve(typename BiTraits<T>::acc_t& a, int lc,
                                                                   const T* __restrict__ lk,
                                                                   const T* __restrict__ ipv) {
  if constexpr (J < 16) {
    typedef BiTraits<T> Tr;
    const T iv = ipv[J];
    const T l = lc > J ? lk[lc * 17 + J] : T(0);  // L_kk[c][J]
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const T cj = Tr::template bcast16<J>(a[r]) * iv;  // L_Ik[i][J]
      a[r] = (lc == J) ? cj : (lc > J ? a[r] - cj * l : a[r]);
    }
    bi_panel_solve<T, J + 1>(a, lc, lk, ipv);
  }
}

// Pass-1 panel: substitution against L_kk (fp64: the Hensman K0zz / H are ill conditioned) or
// the explicit X_k in four MFMAs (fp32 Regime B pivot blocks, conditioned >= noise I).
template <typename T>
constexpr bool kPanelSubst = sizeof(T) == 8;

template <typename T, int TS>
struct BlkInvLds {
  static constexpr int NP = 16 * TS, BLD = 17, RLD = NP + 1, NLB = TS * (TS - 1) / 2;
  T W[NLB > 0 ? NLB : 1][16 * BLD];  // L_Ik (I > k): block I(I-1)/2 + k, element [m][kk]
  T Xinv[TS][16 * BLD];              // X_k = L_kk^-1 (lower), element [m][kk]
  T Lkk[TS][16 * BLD];               // L_kk (lower), element [m][kk]
  T ipiv[TS][16];                    // 1 / (L_kk)_jj
  union {
    T cpan[2][NP * BLD];   // pass 1: column block k of A, element [row i][kk]
    T rpan[2][16 * RLD];   // passes 2/3: row block k of Y / X, element [kk][col j]
  } pan;
  T pdiag[NP];
  double red[16];
  int fail;
};

// One workgroup of 64 * TS * TS / TPW threads inverts one SPD matrix.  Wave w owns the TPW
// consecutive 16x16 tiles (tr, tc0 .. tc0+TPW-1) of one tile row.  Matrix padded to 16 TS with
// the identity.
//   in : element (i, j) at in[i * ldi + j], i, j < n; only the lower triangle is read
//   out: A^-1 element (i, j) at out[i * ldo + j]
//   logdet: log|A| (accumulate = 1: +=);  info: first bad pivot column + col_offset
//   MODE 1 (the N x N potrf's diagonal blocks, potrf.hip): stop after pass 2 -- L into lout (lower, i >= j),
//   Y = L^-1's strict lower part TRANSPOSED into out's strict upper triangle (out[j * ldo + i], i > j; out may be
//   null).  in / out / lout may alias: every read of in precedes the first write.
template <typename T, int TS, int TPW, int MODE = 0>
__device__ inline void blk_inverse(int n, const T* in, int64_t ldi, T* out, int64_t ldo,
                                   double* __restrict__ logdet, int accumulate, int32_t* __restrict__ info,
                                   int col_offset, T* lout = nullptr, int64_t ldl = 0) {
  typedef BiTraits<T> Tr;
  typedef typename Tr::acc_t acc_t;
  typedef BlkInvLds<T, TS> Lds;
  constexpr int WPR = TS / TPW, BLD = Lds::BLD, RLD = Lds::RLD, NT = 64 * TS * TS / TPW;
  __shared__ Lds sm;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63, lc = lane & 15;
  const int tr = w / WPR, tc0 = (w % WPR) * TPW;
  int rw[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) rw[r] = Tr::row(lane, r);
  acc_t acc[TPW];
#pragma unroll
  for (int u = 0; u < TPW; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = tr * 16 + rw[r], j = (tc0 + u) * 16 + lc;
      const int64_t off = (j <= i) ? (int64_t)i * ldi + j : (int64_t)j * ldi + i;
      acc[u][r] = (i < n && j < n) ? in[off] : (i == j ? T(1) : T(0));
    }
  if (t == 0) sm.fail = 0;

  // ---------------- pass 1: block Cholesky ----------------
  // publish column block 0; factor pivot block 0
  if (tc0 == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) sm.pan.cpan[0][(tr * 16 + rw[r]) * BLD + lc] = acc[0][r];
    if (tr == 0) {
      const int bad = chol16_trinv<T>(acc[0], sm.Xinv[0], sm.Lkk[0], sm.ipiv[0], sm.pdiag);
      if (bad >= 0 && lane == 0) sm.fail = bad + 1;
    }
  }
  __syncthreads();
  for (int k = 0; k < TS; ++k) {
    const T* __restrict__ cp = sm.pan.cpan[k & 1];
    if constexpr (kPanelSubst<T>) {
      if (tr > k && tc0 == 0) {
        // L_Ik = A_Ik L_kk^-T by column substitution in registers (one wave per tile row): column
        // j is broadcast along each 16-lane row (DPP) and eliminated from the columns > j
        const T* __restrict__ lk = sm.Lkk[k];
        const T* __restrict__ ipv = sm.ipiv[k];
        acc_t a;
#pragma unroll
        for (int r = 0; r < 4; ++r) a[r] = cp[(tr * 16 + rw[r]) * BLD + lc];
        bi_panel_solve<T, 0>(a, lc, lk, ipv);
        T* __restrict__ Lb = sm.W[tr * (tr - 1) / 2 + k];
#pragma unroll
        for (int r = 0; r < 4; ++r) Lb[rw[r] * BLD + lc] = a[r];
      }
    } else {
      if (tr > k && tc0 == 0) {
        // L_Ik^T = X_k A_kI: four MFMAs with the explicit X_k = L_kk^-1 (fp32: the Schur
        // complements of K = Gram + noise I are >= noise I, so X_k is well conditioned)
        const T* __restrict__ Xk = sm.Xinv[k];
        acc_t lt;
#pragma unroll
        for (int r = 0; r < 4; ++r) lt[r] = T(0);
#pragma unroll
        for (int c = 0; c < 4; ++c) lt = Tr::mfma(Xk[lc * BLD + rw[c]], cp[(tr * 16 + lc) * BLD + rw[c]], lt);
        T* __restrict__ Lb = sm.W[tr * (tr - 1) / 2 + k];
#pragma unroll
        for (int r = 0; r < 4; ++r) Lb[lc * BLD + rw[r]] = lt[r];
      }
    }
    __syncthreads();  // L_Jk of the whole block column visible
    if (tr > k) {
      // trailing update of the own lower tiles k < J <= tr:  A_IJ -= L_Ik L_Jk^T
      const T* __restrict__ Li = sm.W[tr * (tr - 1) / 2 + k];
      T a[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) a[c] = -Li[lc * BLD + rw[c]];
#pragma unroll
      for (int u = 0; u < TPW; ++u) {
        const int J = tc0 + u;
        if (J > k && J <= tr) {
          const T* __restrict__ Lj = sm.W[J * (J - 1) / 2 + k];
#pragma unroll
          for (int c = 0; c < 4; ++c) acc[u] = Tr::mfma(a[c], Lj[lc * BLD + rw[c]], acc[u]);
        }
      }
    }
    if (k + 1 < TS) {
      const int J = k + 1;
      if (J >= tc0 && J < tc0 + TPW && tr >= J) {
        T* __restrict__ cn = sm.pan.cpan[J & 1];
        acc_t tile;
#pragma unroll
        for (int u = 0; u < TPW; ++u)
          if (u == J - tc0) tile = acc[u];
#pragma unroll
        for (int r = 0; r < 4; ++r) cn[(tr * 16 + rw[r]) * BLD + lc] = tile[r];
        if (tr == J) {
          const int bad = chol16_trinv<T>(tile, sm.Xinv[J], sm.Lkk[J], sm.ipiv[J], sm.pdiag + 16 * J);
          if (bad >= 0 && lane == 0 && sm.fail == 0) sm.fail = 16 * J + bad + 1;
        }
      }
    }
    __syncthreads();
  }

  // ---------------- pass 2: Y = L^-1 (acc <- I) ----------------
#pragma unroll
  for (int u = 0; u < TPW; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[u][r] = (tr * 16 + rw[r] == (tc0 + u) * 16 + lc) ? T(1) : T(0);
  // row block KK <- op(X_KK) row block KK (tiles J <= JMAX), published to rpan[KK & 1] if PUB
#define LVAE_BI_ROW_SOLVE(KK, JMAX, TRANS, PUB)                                                   \
  do {                                                                                            \
    if (tr == (KK)) {                                                                             \
      const T* __restrict__ xk_ = sm.Xinv[(KK)];                                                  \
      T a_[4];                                                                                    \
      _Pragma("unroll") for (int c = 0; c < 4; ++c) a_[c] = (TRANS) ? xk_[rw[c] * BLD + lc] : xk_[lc * BLD + rw[c]]; \
      T* __restrict__ rn_ = sm.pan.rpan[(KK)&1];                                                  \
      _Pragma("unroll") for (int u = 0; u < TPW; ++u) {                                           \
        const int J_ = tc0 + u;                                                                   \
        if (J_ <= (JMAX)) {                                                                       \
          acc_t z_;                                                                               \
          _Pragma("unroll") for (int r = 0; r < 4; ++r) z_[r] = T(0);                             \
          _Pragma("unroll") for (int c = 0; c < 4; ++c) z_ = Tr::mfma(a_[c], acc[u][c], z_);      \
          acc[u] = z_;                                                                            \
          if (PUB) {                                                                              \
            _Pragma("unroll") for (int r = 0; r < 4; ++r) rn_[rw[r] * RLD + J_ * 16 + lc] = z_[r]; \
          }                                                                                       \
        }                                                                                         \
      }                                                                                           \
    }                                                                                             \
  } while (0)
  for (int k = 0; k < TS; ++k) {
    LVAE_BI_ROW_SOLVE(k, k, false, k + 1 < TS);  // Y_k <- X_k Y_k
    if (k + 1 == TS) break;
    __syncthreads();
    const T* __restrict__ rp = sm.pan.rpan[k & 1];
    if (tr > k) {  // Y_I -= L_Ik Y_k
      const T* __restrict__ Lb = sm.W[tr * (tr - 1) / 2 + k];
      T a[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) a[c] = -Lb[lc * BLD + rw[c]];
#pragma unroll
      for (int u = 0; u < TPW; ++u) {
        const int J = tc0 + u;
        if (J <= k) {
#pragma unroll
          for (int c = 0; c < 4; ++c) acc[u] = Tr::mfma(a[c], rp[rw[c] * RLD + J * 16 + lc], acc[u]);
        }
      }
    }
  }

  if constexpr (MODE == 1) {
    if (out) {
#pragma unroll
      for (int u = 0; u < TPW; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = tr * 16 + rw[r], j = (tc0 + u) * 16 + lc;
          if (j < i && i < n) out[(int64_t)j * ldo + i] = acc[u][r];
        }
    }
    for (int e = t; e < 256 * TS * TS; e += NT) {
      const int i = e / (16 * TS), j = e % (16 * TS);
      if (j <= i && i < n) {
        const int I = i >> 4, J = j >> 4;
        lout[(int64_t)i * ldl + j] = I == J ? sm.Lkk[I][(i & 15) * BLD + (j & 15)]
                                            : sm.W[I * (I - 1) / 2 + J][(i & 15) * BLD + (j & 15)];
      }
    }
  } else {
  // ---------------- pass 3: A^-1 = L^-T Y ----------------
  for (int k = TS - 1; k >= 0; --k) {
    LVAE_BI_ROW_SOLVE(k, TS, true, k > 0);  // R_k <- X_k^T R_k
    if (k == 0) break;
    __syncthreads();
    const T* __restrict__ rp = sm.pan.rpan[k & 1];
    if (tr < k) {  // R_I -= L_kI^T R_k
      const T* __restrict__ Lb = sm.W[k * (k - 1) / 2 + tr];
      T a[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) a[c] = -Lb[rw[c] * BLD + lc];
#pragma unroll
      for (int u = 0; u < TPW; ++u) {
        const int J = tc0 + u;
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[u] = Tr::mfma(a[c], rp[rw[c] * RLD + J * 16 + lc], acc[u]);
      }
    }
  }
#undef LVAE_BI_ROW_SOLVE
#pragma unroll
  for (int u = 0; u < TPW; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = tr * 16 + rw[r], j = (tc0 + u) * 16 + lc;
      if (i < n && j < n) out[(int64_t)i * ldo + j] = acc[u][r];
    }
  }
  // log|A| = 2 sum log L_jj over the pivot blocks (off the step critical path)
  double lgd = 0.0;
  for (int i = t; i < 16 * TS; i += NT) lgd += log((double)sm.pdiag[i]);
  lgd = wave_sum(lgd);
  if (lane == 0) sm.red[w] = lgd;
  __syncthreads();
  if (t == 0) {
    double ld = 0.0;
    for (int q = 0; q < NT / 64; ++q) ld += sm.red[q];
    ld *= 2.0;
    if (accumulate) *logdet += ld;
    else *logdet = ld;
    const int fail = sm.fail;
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
