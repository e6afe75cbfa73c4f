// potrf.hip -- blocked factorisation and SPD inverse of L batched N x N fp32 covariances on CDNA4
// (replaces torch.cholesky / cholesky_solve(I) / log-det in elbo_functions.py:26-29).
//
// Right-looking block LDL^T with 128-wide pivot blocks (K = Lt Dt Lt^T, Lt unit block-lower,
// Dt = diag(D_k) the Schur-complement pivot blocks; the Cholesky factor is Lt chol(Dt)):
//   per pivot block k:
//     diag   : D_k^-1 and log|D_k| by the in-accumulator 16-block MFMA Cholesky inverse (blkinv.hpp), one WG per matrix
//     panel  : Lt_ik = A_ik D_k^-1                      (the trsm, as an MFMA GEMM)
//     update : A_ij -= Lt_ik A_jk^T, k < j <= i          (MFMA, lower tiles only)
//   log|K| = sum_k log|D_k|
// Inverse K^-1 = X^T Dt^-1 X with X = Lt^-1:
//   trtri  : Y = -X (strictly lower) in place over Lt: Y_rc = Lt_rc - sum_{c<j<r} Lt_rj Y_jc
//   Z      : Z_KJ = -D_K^-1 Y_KJ (K > J)
//   lauum  : K^-1_IJ = Z_IJ - sum_{K>I} Y_KI^T Z_KJ  (Z_II = D_I^-1), mirrored to both triangles
// Buffers [L][np][np] row-major, np % 128 == 0: A (covariance, later Z), W (D_k^-1 on the diagonal
// tiles, Lt -> Y below), Ainv.  Grids are (tiles, L): all latent dims share every launch.
#include "mfma_tile.hpp"
#include "blkinv.hpp"
#include "mfma_x3.hpp"

#include <cstdlib>

namespace lvae {

constexpr int kNB = 128;

// GEMM engine per kernel: fp32-input MFMA (exact fp32 products) or the 3-product f16 split
// (mfma_x3.hpp, ~2^-22 per product, 3/16 of the cost).  Bit i of the mask selects X3 for
// kernel class i (GemmClass); LVAE_X3 in the environment overrides the default.
enum GemmClass { GC_PANEL = 0, GC_UPDATE = 1, GC_TRTRI = 2, GC_Z = 3, GC_LAUUM = 4, GC_SYRK = 5, GC_REC = 6 };
constexpr int kX3DefaultMask = 0x7f;  // all classes: KL/grad parity within 1e-4 (tests), 1.36x step
inline int x3_mask() {
  static const int m = [] {
    const char* e = getenv("LVAE_X3");
    return e ? (int)strtol(e, nullptr, 0) : kX3DefaultMask;
  }();
  return m;
}
inline bool use_x3(GemmClass c) { return (x3_mask() >> c) & 1; }

constexpr int cmax(int a, int b) { return a > b ? a : b; }
template <bool AK, bool BK_>
constexpr int gemm_lds_bytes() {
  return cmax(tile_lds_floats<AK, BK_>() * (int)sizeof(float), x3_lds_bytes());
}

template <bool X3, bool AK, bool BKc, bool NEG = false>
__device__ inline void tile_gemm_any(const float* __restrict__ A, int64_t lda, const float* __restrict__ B, int64_t ldb,
                                     int kbeg, int kend, Frag& f, void* lds, const float* __restrict__ ascale = nullptr) {
  if constexpr (X3)
    tile_gemm_x3<AK, BKc, NEG>(A, lda, B, ldb, kbeg, kend, f, (_Float16*)lds, ascale);
  else
    tile_gemm<AK, BKc, NEG>(A, lda, B, ldb, kbeg, kend, f, (float*)lds, ascale);
}

__device__ inline void tri_index2(int t, int& I, int& J) {
  int r = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
  while ((r + 1) * (r + 2) / 2 <= t) ++r;
  while (r * (r + 1) / 2 > t) --r;
  I = r;
  J = t - r * (r + 1) / 2;
}

// diag: W_kk = D_k^-1, logdet += log|D_k|
__global__ __launch_bounds__(1024) void ldl_diag_kernel(const float* __restrict__ Aall, float* __restrict__ Wall,
                                                        int np_, int kb, double* __restrict__ logdet,
                                                        int32_t* __restrict__ info) {
  const int l = blockIdx.x;
  const int64_t off = (int64_t)l * np_ * np_ + (int64_t)kb * kNB * np_ + kb * kNB;
  blk_inverse<float, 8, 4>(kNB, Aall + off, np_, Wall + off, np_, logdet + l, 1, info + l, kb * kNB);
}

// panel: W_ik = A_ik D_k^-1 for tile rows i > kb
template <bool X3>
__global__ __launch_bounds__(256) void ldl_panel_kernel(const float* __restrict__ Aall, float* __restrict__ Wall,
                                                        int np_, int kb) {
  __shared__ __attribute__((aligned(16))) char lds[gemm_lds_bytes<true, true>()];
  const int l = blockIdx.y, i = kb + 1 + blockIdx.x;
  const float* A = Aall + (int64_t)l * np_ * np_;
  float* W = Wall + (int64_t)l * np_ * np_;
  Frag f;
  f.zero();
  // op(B)(k, n) = Dinv[k][n] = Dinv[n][k]: k-contiguous rows of the symmetric W_kk
  tile_gemm_any<X3, true, true>(A + (int64_t)i * kNB * np_ + kb * kNB, np_, W + (int64_t)kb * kNB * np_ + kb * kNB, np_, 0,
                        kNB, f, lds);
  float* C = W + (int64_t)i * kNB * np_ + kb * kNB;
  frag_foreach(f, [&](int r, int c, float v) { C[(int64_t)r * np_ + c] = v; });
}

// update: A_ij -= W_ik A_jk^T, kb < j <= i
template <bool X3>
__global__ __launch_bounds__(256) void ldl_update_kernel(float* __restrict__ Aall, const float* __restrict__ Wall,
                                                         int np_, int kb) {
  __shared__ __attribute__((aligned(16))) char lds[gemm_lds_bytes<true, true>()];
  int I, J;
  tri_index2(blockIdx.x, I, J);
  const int l = blockIdx.y, i = kb + 1 + I, j = kb + 1 + J;
  float* A = Aall + (int64_t)l * np_ * np_;
  const float* W = Wall + (int64_t)l * np_ * np_;
  float* C = A + (int64_t)i * kNB * np_ + j * kNB;
  Frag f;
  frag_load(f, C, np_);
  tile_gemm_any<X3, true, true, true>(W + (int64_t)i * kNB * np_ + kb * kNB, np_, A + (int64_t)j * kNB * np_ + kb * kNB, np_,
                              0, kNB, f, lds);
  frag_foreach(f, [&](int r, int c, float v) { C[(int64_t)r * np_ + c] = v; });
}

// trtri step jb: W_rc -= W_r,jb W_jb,c   (r > jb > c)
template <bool X3>
__global__ __launch_bounds__(256) void ldl_trtri_kernel(float* __restrict__ Wall, int np_, int jb) {
  __shared__ __attribute__((aligned(16))) char lds[gemm_lds_bytes<true, false>()];
  const int l = blockIdx.y, r = jb + 1 + blockIdx.x / jb, c = blockIdx.x % jb;
  float* W = Wall + (int64_t)l * np_ * np_;
  float* C = W + (int64_t)r * kNB * np_ + c * kNB;
  Frag f;
  frag_load(f, C, np_);
  tile_gemm_any<X3, true, false, true>(W + (int64_t)r * kNB * np_ + jb * kNB, np_, W + (int64_t)jb * kNB * np_ + c * kNB, np_,
                               0, kNB, f, lds);
  frag_foreach(f, [&](int rr, int cc, float v) { C[(int64_t)rr * np_ + cc] = v; });
}

// Z_KJ = -D_K^-1 Y_KJ (K > J), into A's tile (K, J)
template <bool X3>
__global__ __launch_bounds__(256) void ldl_z_kernel(float* __restrict__ Aall, const float* __restrict__ Wall,
                                                    int np_) {
  __shared__ __attribute__((aligned(16))) char lds[gemm_lds_bytes<true, false>()];
  int I, J;
  tri_index2(blockIdx.x, I, J);  // strictly lower: (I + 1, J)
  const int K = I + 1, l = blockIdx.y;
  float* A = Aall + (int64_t)l * np_ * np_;
  const float* W = Wall + (int64_t)l * np_ * np_;
  Frag f;
  f.zero();
  tile_gemm_any<X3, true, false, true>(W + (int64_t)K * kNB * np_ + K * kNB, np_, W + (int64_t)K * kNB * np_ + J * kNB, np_,
                               0, kNB, f, lds);
  float* C = A + (int64_t)K * kNB * np_ + J * kNB;
  frag_foreach(f, [&](int r, int c, float v) { C[(int64_t)r * np_ + c] = v; });
}

// lauum: Ainv_IJ = Z_IJ - sum_{K > I} Y_KI^T Z_KJ  (I >= J), mirrored into the upper triangle
template <bool X3>
__global__ __launch_bounds__(256) void ldl_lauum_kernel(const float* __restrict__ Zall, const float* __restrict__ Wall,
                                                        float* __restrict__ Ball, int np_) {
  __shared__ __attribute__((aligned(16))) char lds[gemm_lds_bytes<false, false>()];
  int I, J;
  tri_index2(blockIdx.x, I, J);
  const int l = blockIdx.y;
  const float* Z = Zall + (int64_t)l * np_ * np_;
  const float* W = Wall + (int64_t)l * np_ * np_;
  float* B = Ball + (int64_t)l * np_ * np_;
  Frag f;
  if (I == J) frag_load(f, W + (int64_t)I * kNB * np_ + I * kNB, np_);
  else frag_load(f, Z + (int64_t)I * kNB * np_ + J * kNB, np_);
  tile_gemm_any<X3, false, false, true>(W + I * kNB, np_, Z + J * kNB, np_, (I + 1) * kNB, np_, f, lds);
  float* C = B + (int64_t)I * kNB * np_ + J * kNB;
  float* Ct = B + (int64_t)J * kNB * np_ + I * kNB;
  const bool mirror = I != J;
  frag_foreach(f, [&](int r, int c, float v) {
    C[(int64_t)r * np_ + c] = v;
    if (mirror) Ct[(int64_t)c * np_ + r] = v;
  });
}

// S = B diag(v) B (lower tiles), B symmetric: S_IJ = sum_k B[I m][k] v_k B[J n][k]
template <bool X3>
__global__ __launch_bounds__(256) void syrk_scaled_kernel(const float* __restrict__ Ball, const float* __restrict__ vall,
                                                          float* __restrict__ Sall, int np_) {
  __shared__ __attribute__((aligned(16))) char lds[gemm_lds_bytes<true, true>()];
  int I, J;
  tri_index2(blockIdx.x, I, J);
  const int l = blockIdx.y;
  const float* B = Ball + (int64_t)l * np_ * np_;
  const float* v = vall + (int64_t)l * np_;
  Frag f;
  f.zero();
  tile_gemm_any<X3, true, true>(B + (int64_t)I * kNB * np_, np_, B + (int64_t)J * kNB * np_, np_, 0, np_, f, lds, v);
  float* C = Sall + (int64_t)l * np_ * np_ + (int64_t)I * kNB * np_ + J * kNB;
  frag_foreach(f, [&](int r, int c, float val) { C[(int64_t)r * np_ + c] = val; });
}

// ------------------------------------------------------------------------------------------
// Recursive Schur-complement inverse (the Regime B path): for K = [[A, B^T], [B, C]],
//   A^-1 (recursion), X = B A^-1, S = C - X B^T, S^-1 (recursion), Y = S^-1 X,
//   K^-1 = [[A^-1 + X^T Y, -Y^T], [-Y, S^-1]],   log|K| = log|A| + log|S|.
// Same n^3 flops as Cholesky + inverse, but the GEMMs of the top levels have K = n/2, n/4, ...
// (compute-bound) where the right-looking block LDL^T spends its time in rank-128 updates
// (memory-bound, one launch per block column).  Leaves are the 128x128 in-register inverse.
// ------------------------------------------------------------------------------------------
struct RecGemm {
  const float* A;
  int64_t lda, sA;
  const float* B;
  int64_t ldb, sB;
  float* C;
  int64_t ldc, sC;
  float* Ct;  // mirror base (nullable): element (r, c) of tile (I, J) also to Ct[(J*128 + c) * ldc + I*128 + r]
  int K, tm, tn;
};

template <bool X3, bool AK, bool BKc, bool NEG, bool LOWER, bool CIN>
__global__ __launch_bounds__(256) void rec_gemm_kernel(RecGemm g) {
  __shared__ __attribute__((aligned(16))) char lds[gemm_lds_bytes<AK, BKc>()];
  int I, J;
  if constexpr (LOWER) {
    tri_index2(blockIdx.x, I, J);
  } else {
    I = blockIdx.x / g.tn;
    J = blockIdx.x % g.tn;
  }
  const int64_t l = blockIdx.y;
  const float* A = g.A + l * g.sA + (AK ? (int64_t)I * kNB * g.lda : (int64_t)I * kNB);
  const float* B = g.B + l * g.sB + (BKc ? (int64_t)J * kNB * g.ldb : (int64_t)J * kNB);
  float* C = g.C + l * g.sC + (int64_t)I * kNB * g.ldc + J * kNB;
  Frag f;
  if constexpr (CIN) frag_load(f, C, g.ldc);
  else f.zero();
  tile_gemm_any<X3, AK, BKc, NEG>(A, g.lda, B, g.ldb, 0, g.K, f, lds);
  float* Ct = g.Ct ? g.Ct + l * g.sC + (int64_t)J * kNB * g.ldc + I * kNB : nullptr;
  const bool mir = Ct != nullptr && !(LOWER && I == J);
  const int64_t ldc = g.ldc;
  frag_foreach(f, [&](int r, int c, float v) {
    C[(int64_t)r * ldc + c] = v;
    if (mir) Ct[(int64_t)c * ldc + r] = v;
  });
}

__global__ __launch_bounds__(1024) void rec_leaf_kernel(const float* __restrict__ Kall, float* __restrict__ Kinv,
                                                        int np_, int off, double* __restrict__ logdet,
                                                        int32_t* __restrict__ info) {
  const int l = blockIdx.x;
  const int64_t o = (int64_t)l * np_ * np_ + (int64_t)off * np_ + off;
  blk_inverse<float, 8, 4>(kNB, Kall + o, np_, Kinv + o, np_, logdet + l, 1, info + l, off);
}

template <bool AK, bool BKc, bool NEG, bool LOWER, bool CIN>
static void rec_launch(const RecGemm& g, int L, hipStream_t st) {
  const int nt = LOWER ? g.tm * (g.tm + 1) / 2 : g.tm * g.tn;
  if (nt <= 0 || g.K <= 0) return;
  if (use_x3(GC_REC))
    rec_gemm_kernel<true, AK, BKc, NEG, LOWER, CIN><<<dim3(nt, L), 256, 0, st>>>(g);
  else
    rec_gemm_kernel<false, AK, BKc, NEG, LOWER, CIN><<<dim3(nt, L), 256, 0, st>>>(g);
}

// Kinv[off:off+n, off:off+n] <- K[off:off+n, off:off+n]^-1 (K: lower 128-tiles valid; the C block's
// lower tiles are overwritten by the Schur complement); W: scratch of K's shape.
static void rec_inv(float* K, float* Kinv, float* W, int np_, int L, int off, int n, double* logdet, int32_t* info,
                    hipStream_t st) {
  if (n == kNB) {
    rec_leaf_kernel<<<L, 1024, 0, st>>>(K, Kinv, np_, off, logdet, info);
    return;
  }
  const int64_t np2 = (int64_t)np_ * np_;
  const int t = n / kNB, h1 = (t / 2) * kNB, h2 = n - h1, o2 = off + h1;
  auto at = [&](float* base, int r, int c) { return base + (int64_t)r * np_ + c; };
  rec_inv(K, Kinv, W, np_, L, off, h1, logdet, info, st);  // A^-1
  // X = B A^-1   [h2 x h1] -> W
  rec_launch<true, false, false, false, false>(
      RecGemm{at(K, o2, off), np_, np2, at(Kinv, off, off), np_, np2, at(W, o2, off), np_, np2, nullptr, h1, h2 / kNB,
              h1 / kNB}, L, st);
  // S = C - X B^T   (lower tiles, in place)
  rec_launch<true, true, true, true, true>(
      RecGemm{at(W, o2, off), np_, np2, at(K, o2, off), np_, np2, at(K, o2, o2), np_, np2, nullptr, h1, h2 / kNB,
              h2 / kNB}, L, st);
  rec_inv(K, Kinv, W, np_, L, o2, h2, logdet, info, st);  // S^-1
  // -Y = -S^-1 X  -> Kinv lower-left, mirrored to upper-right
  rec_launch<true, false, true, false, false>(
      RecGemm{at(Kinv, o2, o2), np_, np2, at(W, o2, off), np_, np2, at(Kinv, o2, off), np_, np2, at(Kinv, off, o2), h2,
              h2 / kNB, h1 / kNB}, L, st);
  // A^-1 += X^T Y = A^-1 - X^T (-Y)   (lower tiles, mirrored)
  rec_launch<false, false, true, true, true>(
      RecGemm{at(W, o2, off), np_, np2, at(Kinv, o2, off), np_, np2, at(Kinv, off, off), np_, np2, at(Kinv, off, off),
              h2, h1 / kNB, h1 / kNB}, L, st);
}

int spd_inverse_f32(int np_, int L, float* A, float* W, float* Ainv, double* logdet, int32_t* info, hipStream_t st) {
  if (np_ <= 0 || np_ % kNB) return -1;
  if (L <= 0) return -2;
  (void)hipMemsetAsync(logdet, 0, sizeof(double) * L, st);
  (void)hipMemsetAsync(info, 0, sizeof(int32_t) * L, st);
  rec_inv(A, Ainv, W, np_, L, 0, np_, logdet, info, st);
  LVAE_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------------------------------
// host sequencing
// ------------------------------------------------------------------------------------------
int potrf_f32(int np_, int L, float* A, float* W, double* logdet, int32_t* info, hipStream_t st) {
  if (np_ <= 0 || np_ % kNB) return -1;
  if (L <= 0) return -2;
  (void)hipMemsetAsync(logdet, 0, sizeof(double) * L, st);
  (void)hipMemsetAsync(info, 0, sizeof(int32_t) * L, st);
  const int nt = np_ / kNB;
  for (int kb = 0; kb < nt; ++kb) {
    ldl_diag_kernel<<<L, 1024, 0, st>>>(A, W, np_, kb, logdet, info);
    const int T = nt - kb - 1;
    if (T > 0) {
      (use_x3(GC_PANEL) ? ldl_panel_kernel<true> : ldl_panel_kernel<false>)<<<dim3(T, L), 256, 0, st>>>(A, W, np_, kb);
      (use_x3(GC_UPDATE) ? ldl_update_kernel<true> : ldl_update_kernel<false>)<<<dim3(T * (T + 1) / 2, L), 256, 0, st>>>(A, W, np_, kb);
    }
  }
  LVAE_CHECK_LAUNCH();
  return 0;
}

int potri_f32(int np_, int L, float* A, float* W, float* Ainv, hipStream_t st) {
  if (np_ <= 0 || np_ % kNB) return -1;
  const int nt = np_ / kNB;
  for (int jb = 1; jb + 1 < nt; ++jb) (use_x3(GC_TRTRI) ? ldl_trtri_kernel<true> : ldl_trtri_kernel<false>)<<<dim3((nt - jb - 1) * jb, L), 256, 0, st>>>(W, np_, jb);
  if (nt > 1) (use_x3(GC_Z) ? ldl_z_kernel<true> : ldl_z_kernel<false>)<<<dim3(nt * (nt - 1) / 2, L), 256, 0, st>>>(A, W, np_);
  (use_x3(GC_LAUUM) ? ldl_lauum_kernel<true> : ldl_lauum_kernel<false>)<<<dim3(nt * (nt + 1) / 2, L), 256, 0, st>>>(A, W, Ainv, np_);
  LVAE_CHECK_LAUNCH();
  return 0;
}

int syrk_scaled_f32(int np_, int L, const float* B, const float* v, float* S, hipStream_t st) {
  const int nt = np_ / kNB;
  (use_x3(GC_SYRK) ? syrk_scaled_kernel<true> : syrk_scaled_kernel<false>)<<<dim3(nt * (nt + 1) / 2, L), 256, 0, st>>>(B, v, S, np_);
  LVAE_CHECK_LAUNCH();
  return 0;
}

}  // namespace lvae

extern "C" {
int lvae_gemm_engine_mask(void) { return lvae::x3_mask(); }
int lvae_spd_inverse_f32(int np_, int L, float* A, float* W, float* Ainv, double* logdet, int32_t* info,
                         void* stream) {
  return lvae::spd_inverse_f32(np_, L, A, W, Ainv, logdet, info, (hipStream_t)stream);
}
int lvae_potrf_f32(int np_, int L, float* A, float* W, double* logdet, int32_t* info, void* stream) {
  return lvae::potrf_f32(np_, L, A, W, logdet, info, (hipStream_t)stream);
}
int lvae_potri_f32(int np_, int L, float* A, float* W, float* Ainv, void* stream) {
  return lvae::potri_f32(np_, L, A, W, Ainv, (hipStream_t)stream);
}
}
