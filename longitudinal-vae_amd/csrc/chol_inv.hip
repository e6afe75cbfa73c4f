// chol_inv.hip -- K^-1 and log|K| of L batched SPD np x np fp32 covariances by a blocked Cholesky
// factorisation, a blocked triangular inverse and their product (LAPACK potrf + trtri + lauum), the
// Regime B inverse of the exact KL: torch.cholesky(K1), cholesky_solve(I, LK1) and the log-det of
// elbo_functions.py:26-29.  256-wide blocks, every GEMM on the f16 matrix cores with the fp32-accurate
// 3-product split (mfma_x3.hpp / x3_dma.hpp: x s = hi + lo per operand block, a power-of-two split
// scale s = x3_scale(max |block|) per 256 x 256 block from the block's exact max, taken by the kernel
// that writes the block).
//
// Why Cholesky and not the block sweep (spd_sweep.hip): the sweep (Gauss-Jordan on SPD) updates the
// already inverted part in every pass, and its K^-1 error grows ~100x faster with cond(K) (emulated
// in fp32 at N = 1024, cond 1.3e5: |I - K X|_2 = 2.7 against 0.03 here).  Same n^3 flops.
//
//   1. potrf, right-looking, one pass per block column k (all L dims in every launch):
//        pivot(k)  A_kk -> L_kk (blocked Cholesky in LDS on fp32 MFMA, pv_lds.hpp), log|A_kk|, info,
//                  and Y_kk = L_kk^-1 (recursive doubling) as fp16 planes: row-major into D (the panel's
//                  operand) and transposed into tile (k, k) of the Y^T planes
//        panel(k)  L_ik = A_ik Y_kk^T for i > k, from the planes of the updated column (C) -> the
//                  planes of L (tile (i, k)), one 256 x 256 x3 tile GEMM per block
//        U1(k)     column k+1: A_I,k+1 -= L_Ik L_k+1,k^T, written straight as the planes of pass k+1's
//                  C operand (+ the next pivot block in fp32 when the pivot does not update it itself)
//        U2(k)     the trailing tiles I >= J >= k+2: A_IJ -= L_Ik L_Jk^T, in place (HBM-streaming rank-256
//                  update, A read and written under the MFMAs as in the sweep)
//      with lookahead: the next pivot (+ panel) runs on the side stream beside U2 (schedules below).
//   2. trtri, Y = L^-1 by recursive doubling over levels of h = 1, 2, 4, ... blocks: for every aligned
//      pair of inverted diagonal groups [A 0; B C] (A = rows [o, o+h), C = [o+h, o+2h)), B <- -C^-1 B A^-1:
//        X_ij = sum_{k=j}^{o+h-1} L_ik Y_kj,   Y_ij = -sum_{k=o+h}^{i} Y_ik X_kj    (ci_gemm_kernel)
//      two launches per level, every GEMM K-deep over whole blocks (MFMA-bound, not HBM-bound)
//   3. lauum, K^-1 = Y^T Y: (K^-1)_IJ = sum_{k >= I} Y_kI^T Y_kJ for I >= J, written with its mirror.
//
// GEMM operands are pre-split fp16 planes [row][k] (x3_dma.hpp's NT form: both operands k-contiguous),
// so Y is kept in both orientations: Y planes (row-major, the A operand of the Y step) and Y^T planes
// (the B operand of the X step and both operands of lauum); X is written transposed.  A K range that
// crosses blocks changes the operand scales: the accumulators are rescaled by the (power-of-two) ratio
// at each block boundary (exact).
//
// Buffers (ci_inverse): A [L, np, np] fp32 (lower tiles read; dead after potrf, then reused as the Y
// planes), YT [L, np, np] x 2 halves (Y^T planes; caller-provided), Kinv [L, np, np] fp32 out (reused as
// the X^T planes during trtri), scratch (CiScratch): C planes 2 x [L, np, 256] by pass parity, the
// pivot's X block, D [L, nt, 256, 256], the L planes [L, np, np] and the per-tile scales.
#include "prof.hpp"
#include "pv_lds.hpp"
#include "side_stream.hpp"
#include "x3_c16.hpp"

#ifndef LVAE_CI_C16
#define LVAE_CI_C16 1
#endif
// the pivot's pending update (dev A/B switches): skip the zero half of Y_kk in X = C Y_kk^T, and load X's
// planes once for X X^T
#ifndef LVAE_PV_BTRI
#define LVAE_PV_BTRI 1
#endif
#ifndef LVAE_PV_SAMEAB
#define LVAE_PV_SAMEAB 1
#endif
#ifndef LVAE_CI_KREV
#define LVAE_CI_KREV 1
#endif

namespace lvae {

// the trtri / lauum planes (Y, Y^T, X^T) in the chunk-major layout and their GEMMs on the c16 core
// (x3_c16.hpp: a 4-stage ring, 128 KB of LDS beside the epilogues' own); 0: row-major planes on x3_dma.hpp
constexpr bool kCiC16 = LVAE_CI_C16 != 0;

// Few latent dims per call (a sharded rank: L <= kCiPipeMaxL): trtri runs PIPELINED with potrf, by block
// rows, on the caller's stream between the passes (the GPU is mostly idle beside the pivot chain there):
// once pivot(m) has Y_mm and panel(m) column m of L,
//   rowY(m)   Y_mj = -Y_mm X_mj for j < m (+ the diagonal Y^T tile from D)   X_mj = sum_{k=j}^{m-1} L_mk Y_kj
//   Xupd(m)   X_ij += L_im Y_mj for i > m, j <= m (fp32 in the Kinv buffer; row m+1, complete now, as the
//             split X^T planes rowY(m+1) reads)
// so that after the last pivot only rowY(nt-1) is left of trtri (recursive doubling: 2 log2(nt) launches
// of under-filled tiles after potrf).  Same flops; the Y planes (row-major Y, read only by the doubling's
// Y step) are not produced.
#ifndef LVAE_CI_PIPE_MAX_L
#define LVAE_CI_PIPE_MAX_L 2  // (scripts/inv_ab.py: L = 2 2.18 vs 2.60 ms for the inverse; L = 4 2.84 either way)
#endif
// the latent-dim bound of the pipelined schedule: LVAE_CI_PIPE_L overrides it for A/B runs (read once per
// process, so the workspace size query and the calls agree)
inline int ci_pipe_max_l() {
  static const int v = getenv("LVAE_CI_PIPE_L") ? atoi(getenv("LVAE_CI_PIPE_L")) : LVAE_CI_PIPE_MAX_L;
  return v;
}
inline bool ci_pipe_alloc(int np_, int L) { return L <= ci_pipe_max_l() && L <= 16 && np_ >= 512; }  // (16: kCiFuseMaxL)
// 0: recursive-doubling trtri after potrf; 1: pipelined trtri; 2: pipelined trtri + lauum (K^-1 accumulated
// as the rows of Y arrive: Lupd(m), K^-1_IJ += Y_mI^T Y_mJ for J <= I <= m, fp32 in the Kinv buffer, whose
// tiles of rows <= m the pipelined X no longer uses; the reduce's lauum is then its epilogue alone).
// LVAE_CI_PIPE=0 / LVAE_CI_PIPE_LAUUM=0 switch the stages off (A/B runs; read once per process).
inline int ci_pipe_mode(int np_, int L) {
  static const bool on = !getenv("LVAE_CI_PIPE") || atoi(getenv("LVAE_CI_PIPE")) != 0;
  static const bool lau = !getenv("LVAE_CI_PIPE_LAUUM") || atoi(getenv("LVAE_CI_PIPE_LAUUM")) != 0;
  if (!on || !ci_pipe_alloc(np_, L)) return 0;
  return lau ? 2 : 1;
}

struct CiScratch {
  _Float16 *Ch[2], *Cl[2];  // [L][np][256] planes of the updated column (pass k's C operand), by parity
  _Float16 *Xh, *Xl;        // [L][256][256] the pivot's own L_{k,k-1} block (schedule (a))
  _Float16 *Dh, *Dl;        // [L][nt][256][256] planes of Y_kk = L_kk^-1 (row-major)
  _Float16 *Lh, *Ll;        // [L][np][np] planes of L (off-diagonal lower tiles)
  float* csc;               // [L][nt][nt] (l, k, i): block i of pass k's C operand
  float* lsc;               // [L][nt][nt] (l, i, k): tile (i, k) of L
  float* ysc;               // [L][nt][nt] (l, i, j): tile (i, j) of Y (both plane orientations; D for i == j)
  float* xsc;               // [L][nt][nt] (l, i, j): tile (i, j) of the trtri intermediate X
  _Float16 *XRh[2], *XRl[2];  // pipelined trtri: the X^T tiles (j, m) of row block m, [L][nt][256 x 256] (one
                              // chunk-major tile each), by row parity; nullptr unless ci_pipe_alloc
  float* lout = nullptr;      // potrf-only export (ci_potrf_f32): the pivots write L_kk, the panels L_ik, in fp32
                              // into the lower tiles of this [L][np][np] matrix (not part of `bytes`)
  int* cnt;                   // [L][nt] split pivots: arrival tickets per (dim, pass), zeroed per call (own block)
  float* xs;                  // [L][kCiPvG] split pivots: the split scale of each helper's X slab
  int nt;
  size_t bytes;
  CiScratch(char* base, int np_, int L) {
    size_t off = 0;
    auto take = [&](size_t b) {
      char* p = base ? base + off : nullptr;
      off += align256(b);
      return p;
    };
    nt = np_ / kSwB;
    const size_t col = (size_t)L * np_ * kSwB;
    for (int b = 0; b < 2; ++b) {
      Ch[b] = (_Float16*)take(col * 2);
      Cl[b] = (_Float16*)take(col * 2);
    }
    Xh = (_Float16*)take((size_t)L * kSwBB * 2);
    Xl = (_Float16*)take((size_t)L * kSwBB * 2);
    Dh = (_Float16*)take(col * 2);
    Dl = (_Float16*)take(col * 2);
    const size_t full = (size_t)L * np_ * np_;
    Lh = (_Float16*)take(full * 2);
    Ll = (_Float16*)take(full * 2);
    csc = (float*)take((size_t)L * nt * nt * 4);
    lsc = (float*)take((size_t)L * nt * nt * 4);
    ysc = (float*)take((size_t)L * nt * nt * 4);
    xsc = (float*)take((size_t)L * nt * nt * 4);
    for (int b = 0; b < 2; ++b) {
      XRh[b] = ci_pipe_alloc(np_, L) ? (_Float16*)take(col * 2) : nullptr;
      XRl[b] = ci_pipe_alloc(np_, L) ? (_Float16*)take(col * 2) : nullptr;
    }
    cnt = (int*)take(cnt_bytes(L, nt));
    xs = (float*)take((size_t)L * 8 * 4);
    bytes = off;
  }
  static size_t cnt_bytes(int L, int nt) { return ((size_t)L * nt * 4 + 15) & ~size_t(15); }
  __device__ float& c_scale(int l, int k, int i) const { return csc[((int64_t)l * nt + k) * nt + i]; }
  __device__ float& t_scale(float* s, int l, int i, int j) const { return s[((int64_t)l * nt + i) * nt + j]; }
};

// ------------------------------------------------------------------------------------------
// pivot(kb): A_kk (lower triangle) -> L_kk in LDS -> Y_kk = L_kk^-1; out: Y_kk planes (D, row-major)
// with the split scale of max |Y_kk|, log|A_kk|, info.  One 1024-thread
// workgroup per dim.  With `pending` (schedule (a), kb > 0) the block still lacks pass kb-1's update,
// applied here: X = L_{kb,kb-1} = C_kb Y_{kb-1}^T (C planes of pass kb-1, block kb; D of kb-1), split
// at its exact max into Xh / Xl, then A_kk - X X^T.
// ------------------------------------------------------------------------------------------
__device__ inline void ci_pending_update(const float* __restrict__ T, int64_t np_, const CiScratch& S, int l, int kb,
                                         float* __restrict__ lf, uint32_t* red) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, rl = lane & 31, hh = lane >> 5;
  const int kp = kb - 1;
  const int64_t oc = (int64_t)l * np_ * kSwB + (int64_t)kb * kSwBB, od = ((int64_t)l * S.nt + kp) * kSwBB;
  const int64_t ox = (int64_t)l * kSwBB;
  float sxo;
  {
    const _Float16* src[4] = {S.Ch[kp & 1] + oc, S.Cl[kp & 1] + oc, S.Dh + od, S.Dl + od};
    int bi[4], bj[4];
#pragma unroll
    for (int h = 0; h < 4; ++h) bi[h] = (4 * w + h) >> 3, bj[h] = (4 * w + h) & 7;
    pv_f32x16 x[4];
#pragma unroll
    for (int h = 0; h < 4; ++h) x[h] = pv_f32x16{};
    pv_x3_gemm<4, false, false, LVAE_PV_BTRI != 0>(src, lf, bi, bj, x);  // (D = Y_kk: lower triangular)
    const float inv = 1.0f / (S.c_scale(l, kp, kb) * S.ysc[((int64_t)l * S.nt + kp) * S.nt + kp]);
    float m = 0.f;
#pragma unroll
    for (int h = 0; h < 4; ++h)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        x[h][e] *= inv;
        m = fmaxf(m, fabsf(x[h][e]));
      }
    const float sx = x3_scale(sw_block_max(m, red));
    _Float16* xh = S.Xh + ox;
    _Float16* xl = S.Xl + ox;
#pragma unroll
    for (int h = 0; h < 4; ++h)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int r = 32 * bi[h] + pv_row(e, hh), c = 32 * bj[h] + rl;
        const float y = x[h][e] * sx;
        const _Float16 yh = (_Float16)y;
        xh[r * kSwB + c] = yh;
        xl[r * kSwB + c] = (_Float16)(y - (float)yh);
      }
    sxo = sx;
    __syncthreads();  // the X planes are visible to the workgroup
  }
  const float sx = sxo;
  const _Float16* src[4] = {S.Xh + ox, S.Xl + ox, S.Xh + ox, S.Xl + ox};
  int bi[3], bj[3];
#pragma unroll
  for (int h = 0; h < 3; ++h) {
    const int n = kLauum[w][h];
    if (n < 0) {
      bi[h] = bj[h] = -1;
    } else {
      pv_ij(n, bi[h], bj[h]);
    }
  }
  pv_f32x16 acc[3];
#pragma unroll
  for (int h = 0; h < 3; ++h) acc[h] = pv_f32x16{};
  pv_x3_gemm<3, true, LVAE_PV_SAMEAB != 0>(src, lf, bi, bj, acc);  // (X X^T: X's planes loaded once)
  const float inv = 1.0f / (sx * sx);
  float old[3][16];
#pragma unroll
  for (int h = 0; h < 3; ++h) {
    if (bi[h] < 0) continue;
#pragma unroll
    for (int e = 0; e < 16; ++e) old[h][e] = T[(int64_t)(32 * bi[h] + pv_row(e, hh)) * np_ + 32 * bj[h] + rl];
  }
  __syncthreads();  // every wave's last staging read
#pragma unroll
  for (int h = 0; h < 3; ++h) {
    const int n = kLauum[w][h];
    if (n < 0) continue;
#pragma unroll
    for (int e = 0; e < 16; ++e) lf[n * kPvBlk + pv_row(e, hh) * kPvL + rl] = old[h][e] - acc[h][e] * inv;
  }
}

// ------------------------------------------------------------------------------------------
// Split pivot (kCiPvG workgroups per dim, schedule (a)): the pending update's X = C_kb Y_kp^T is computed
// by the dim's kCiPvG workgroups in row slabs of 256 / kCiPvG rows, each split at its own exact max into
// the X planes (scale xs[l][h]); a ticket per (dim, pass) elects the LAST arriving workgroup (in-launch
// hand-off, cdna_hip_programming.md's split-K recipe: plain stores, vmcnt drain, barrier, agent release,
// relaxed agent ticket; the last: agent acquire, then plain loads), which goes on alone with A_kk - X X^T
// (per-slab-pair scales), the Cholesky and the rest.  The others exit.  Placement is for speed only (a
// dim's workgroups share blockIdx % 8: one XCD under round-robin dispatch, the slabs read from its L2).
// ------------------------------------------------------------------------------------------
constexpr int kCiPvG = 4;                 // workgroups per split pivot
constexpr int kCiPvR = kSwB / kCiPvG;     // X rows per helper (64: 2 x 8 blocks of 32 x 32, one per wave)
__device__ inline void ci_pending_slab(const CiScratch& S, int64_t np_, int l, int kb, int h, float* __restrict__ lf,
                                       uint32_t* red) {
  static_assert(kCiPvR / 32 * 8 == 16, "one 32 x 32 block of the slab per wave");
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, rl = lane & 31, hh = lane >> 5;
  const int kp = kb - 1;
  const int64_t oc = (int64_t)l * np_ * kSwB + (int64_t)kb * kSwBB + (int64_t)h * kCiPvR * kSwB;
  const int64_t od = ((int64_t)l * S.nt + kp) * kSwBB;
  const _Float16* src[4] = {S.Ch[kp & 1] + oc, S.Cl[kp & 1] + oc, S.Dh + od, S.Dl + od};
  _Float16* st = reinterpret_cast<_Float16*>(lf);
  // staging per 64-deep chunk: A parts [2][64 rows][kPvKP], B parts [2][256 rows][kPvKP]; thread t loads A
  // piece t (part t >> 9, row (t >> 3) & 63, 16-B chunk t & 7) and B pieces t + 1024 u (u < 4: part u >> 1,
  // row ((t >> 3) & 127) + 128 (u & 1)); B rows < kc are zero (Y_kp lower triangular): not loaded
  const int arow = (tid >> 3) & 63, ap = tid >> 9, c8 = tid & 7, brow0 = (tid >> 3) & 127;
  auto aoff = [&](int p, int row) { return (p * kCiPvR + row) * kPvKP; };
  auto boff = [&](int p, int row) { return (2 * kCiPvR + p * kSwB + row) * kPvKP; };
  x3_half8 va, vb[4];
  auto load = [&](int kc) {
    va = *reinterpret_cast<const x3_half8*>(src[ap] + arow * kSwB + kc + 8 * c8);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int row = brow0 + 128 * (u & 1);
      if (row >= kc) vb[u] = *reinterpret_cast<const x3_half8*>(src[2 + (u >> 1)] + row * kSwB + kc + 8 * c8);
    }
  };
  const int bi = w >> 3, bj = w & 7;
  pv_f32x16 acc = {};
  load(0);
  for (int kc = 0; kc < kSwB; kc += kPvKC) {
    __syncthreads();  // the previous chunk's readers are done
    *reinterpret_cast<x3_half8*>(st + aoff(ap, arow) + 8 * c8) = va;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int row = brow0 + 128 * (u & 1);
      if (row >= kc) *reinterpret_cast<x3_half8*>(st + boff(u >> 1, row) + 8 * c8) = vb[u];
    }
    __syncthreads();
    if (kc + kPvKC < kSwB) load(kc + kPvKC);
    if (32 * bj + 31 >= kc) {  // (wave-uniform) a non-zero chunk of Y_kp's row block bj
      const _Float16* ar = st + aoff(0, 32 * bi + rl);
      const _Float16* br = st + boff(0, 32 * bj + rl);
#pragma unroll
      for (int ks = 0; ks < kPvKC / 16; ++ks) {
        const int ko = 16 * ks + 8 * hh;
        const x3_half8 aH = *reinterpret_cast<const x3_half8*>(ar + ko);
        const x3_half8 aL = *reinterpret_cast<const x3_half8*>(ar + kCiPvR * kPvKP + ko);
        const x3_half8 bH = *reinterpret_cast<const x3_half8*>(br + ko);
        const x3_half8 bL = *reinterpret_cast<const x3_half8*>(br + kSwB * kPvKP + ko);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(aL, bH, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(aH, bL, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(aH, bH, acc, 0, 0, 0);
      }
    }
  }
  const float inv = 1.0f / (S.c_scale(l, kp, kb) * S.ysc[((int64_t)l * S.nt + kp) * S.nt + kp]);
  float m = 0.f;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    acc[e] *= inv;
    m = fmaxf(m, fabsf(acc[e]));
  }
  const float sx = x3_scale(sw_block_max(m, red));
  const int64_t ox = (int64_t)l * kSwBB + (int64_t)h * kCiPvR * kSwB;
  _Float16* xh = S.Xh + ox;
  _Float16* xl = S.Xl + ox;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int r = 32 * bi + pv_row(e, hh), c = 32 * bj + rl;
    const float y = acc[e] * sx;
    const _Float16 yh = (_Float16)y;
    xh[r * kSwB + c] = yh;
    xl[r * kSwB + c] = (_Float16)(y - (float)yh);
  }
  if (tid == 0) S.xs[l * 8 + h] = sx;
}

// the last workgroup's A_kk - X X^T (X planes of kCiPvG slabs, slab h at scale xs[l][h]) into lf
__device__ inline void ci_pending_reduce(const float* __restrict__ T, int64_t np_, const CiScratch& S, int l,
                                         float* __restrict__ lf) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, rl = lane & 31, hh = lane >> 5;
  const int64_t ox = (int64_t)l * kSwBB;
  float xsl[kCiPvG];
#pragma unroll
  for (int h = 0; h < kCiPvG; ++h) xsl[h] = S.xs[l * 8 + h];
  const _Float16* src[4] = {S.Xh + ox, S.Xl + ox, S.Xh + ox, S.Xl + ox};
  int bi[3], bj[3];
#pragma unroll
  for (int h = 0; h < 3; ++h) {
    const int n = kLauum[w][h];
    if (n < 0) {
      bi[h] = bj[h] = -1;
    } else {
      pv_ij(n, bi[h], bj[h]);
    }
  }
  pv_f32x16 acc[3];
#pragma unroll
  for (int h = 0; h < 3; ++h) acc[h] = pv_f32x16{};
  pv_x3_gemm<3, true, LVAE_PV_SAMEAB != 0>(src, lf, bi, bj, acc);
  float old[3][16];
#pragma unroll
  for (int h = 0; h < 3; ++h) {
    if (bi[h] < 0) continue;
#pragma unroll
    for (int e = 0; e < 16; ++e) old[h][e] = T[(int64_t)(32 * bi[h] + pv_row(e, hh)) * np_ + 32 * bj[h] + rl];
  }
  __syncthreads();  // every wave's last staging read
#pragma unroll
  for (int h = 0; h < 3; ++h) {
    const int n = kLauum[w][h];
    if (n < 0) continue;
    const float inv = 1.0f / (xsl[(32 * bi[h]) / kCiPvR] * xsl[(32 * bj[h]) / kCiPvR]);
#pragma unroll
    for (int e = 0; e < 16; ++e) lf[n * kPvBlk + pv_row(e, hh) * kPvL + rl] = old[h][e] - acc[h][e] * inv;
  }
}

// dev: phase timestamps of the pivots (s_memrealtime, 100 MHz) into prof[(kb * L + l) * 8 + phase] when
// lvae_dev_pivot_prof set a buffer (scripts/pivot_prof.py); nullptr in the product
static unsigned long long* g_pivot_prof = nullptr;
#define CI_STAMP(q)                                                                     \
  do {                                                                                  \
    if (prof && threadIdx.x == 0) prof[((int64_t)kb * L + l) * 8 + (q)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

// (dev builds, LVAE_PV_STAMP_CHOL: stamp i < 24 of pivot kb == 1 only, slots of kb = 1 + i / 8)
#define CI_STAMPX(i)                                                                                \
  do {                                                                                              \
    if (prof && kb == 1 && threadIdx.x == 0)                                                        \
      prof[((int64_t)(1 + (i) / 8) * L + l) * 8 + (i) % 8] = __builtin_amdgcn_s_memrealtime();        \
  } while (0)

// G == 1: one workgroup per dim (blockIdx = dim); G == kCiPvG (pending only): the split pivot, workgroup b
// of dim b % Lr, slab b / Lr (Lr = gridDim.x / G, a multiple of 8; dims >= L exit)
template <int G>
__global__ __launch_bounds__(1024) void ci_pivot_kernel(const float* __restrict__ Aall, int np_, int kb, CiScratch S,
                                                        double* __restrict__ logdet, int32_t* __restrict__ info,
                                                        int pending, int L, unsigned long long* __restrict__ prof) {
  __shared__ float lf[kPvBlocks * kPvBlk];
  __shared__ uint32_t ymax_s, xmax_s, dmax_s;
  __shared__ float bsc[kPvBlocks];
  __shared__ int bad_s, last_s;
  const int Lr = gridDim.x / G, l = G == 1 ? blockIdx.x : blockIdx.x % Lr, hs = G == 1 ? 0 : blockIdx.x / Lr;
  if (l >= L) return;  // (uniform; padding dims of the split grid)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, rl = lane & 31, hh = lane >> 5;
  const float* T = Aall + (int64_t)l * np_ * np_ + (int64_t)kb * kSwB * np_ + kb * kSwB;
#ifdef LVAE_PV_STAMP_CHOL
  if (hs == 0) CI_STAMPX(0);
#else
  if (hs == 0) CI_STAMP(0);
#endif
  if (tid == 0) {
    bad_s = INT_MAX;
    ymax_s = 0u;
    xmax_s = 0u;
  }
  if (G > 1) {  // (pending) the slab, the hand-off, then only the last arriving workgroup goes on
    __syncthreads();  // xmax_s
    ci_pending_slab(S, np_, l, kb, hs, lf, &xmax_s);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's slab stores done
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int t = __hip_atomic_fetch_add(S.cnt + (int64_t)l * S.nt + kb, 1, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
      last_s = t == G - 1;
    }
    __syncthreads();
    if (!last_s) return;  // (uniform)
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    ci_pending_reduce(T, np_, S, l, lf);
  } else if (pending) {
    __syncthreads();  // xmax_s
    ci_pending_update(T, np_, S, l, kb, lf, &xmax_s);
  } else {
    const int r = tid >> 5, c = tid & 31;
    float v[kPvBlocks];
#pragma unroll
    for (int R = 0, b = 0; R < 8; ++R)
#pragma unroll
      for (int C = 0; C <= R; ++C, ++b) v[b] = T[(int64_t)(32 * R + r) * np_ + 32 * C + c];
#pragma unroll
    for (int b = 0; b < kPvBlocks; ++b) lf[b * kPvBlk + r * kPvL + c] = v[b];
  }
  __syncthreads();
#ifdef LVAE_PV_STAMP_CHOL
  CI_STAMPX(1);
#else
  CI_STAMP(1);
#endif
  double ld = 0.0;
  int bad = INT_MAX;

  // 1. Cholesky A_kk = L L^T, panel by panel (two elimination steps per MFMA, pv_panel2), then the
  //    trailing update A_ij -= L_iq L_jq^T on the f16 cores with the x3 split (pv_mma3): every entry of
  //    L obeys |L_ij| <= sqrt(A_ii), so one split scale from the block's largest diagonal entry serves
  //    every panel block
  {
    float m = 0.f;
    if (tid < kSwB) m = fabsf(pv_blk(lf, tid >> 5, tid >> 5)[(tid & 31) * kPvL + (tid & 31)]);
    dmax_s = 0u;  // (after the loads' barrier: nobody reads it before the one below)
    __syncthreads();
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if (lane == 0) atomicMax(&dmax_s, __float_as_uint(m));
    __syncthreads();
  }
  const float sL = x3_scale(sqrtf(__uint_as_float(dmax_s)));
  for (int q = 0; q < 8; ++q) {
    if (w <= 7 - q) {
      pv_panel2(lf, q, w, lane, ld, bad);
    } else {
      __syncthreads();  // pv_panel2's barrier
    }
    __syncthreads();
#ifdef LVAE_PV_STAMP_CHOL  // (dev builds: pivot 1's panel q end at stamp 2 + 2 q, its update's at 3 + 2 q)
    CI_STAMPX(2 + 2 * q);
#endif
    const int m = 7 - q, nb = m * (m + 1) / 2;
    for (int t = w; t < nb; t += 16) {
      int jj = 0, u = t;
      while (u >= m - jj) {
        u -= m - jj;
        ++jj;
      }
      const int j = q + 1 + jj, i = j + u;
      pv_f32x16 acc;
      float* Bij = pv_blk(lf, i, j);
      pv_load(acc, Bij, rl, hh);
      pv_mma3<false, false>(acc, pv_blk(lf, i, q), pv_blk(lf, j, q), sL, sL, rl, hh, -1.f);
      pv_store(acc, Bij, rl, hh);
    }
    __syncthreads();
#ifdef LVAE_PV_STAMP_CHOL
    CI_STAMPX(3 + 2 * q);
#endif
  }
#ifndef LVAE_PV_STAMP_CHOL
  CI_STAMP(2);
#endif
  if (S.lout) {  // (potrf-only) L_kk, zero strict upper part, into tile (kb, kb) of lout
    float* O = S.lout + (int64_t)l * np_ * np_ + (int64_t)kb * kSwB * np_ + kb * kSwB;
    for (int e = tid; e < kSwBB; e += 1024) {
      const int r = e >> 8, c = e & 255;
      O[(int64_t)r * np_ + c] = c <= r ? pv_blk(lf, r >> 5, c >> 5)[(r & 31) * kPvL + (c & 31)] : 0.f;
    }
  }
  if (w < 8) pv_trinv(pv_blk(lf, w, w), lane);
  __syncthreads();
#ifndef LVAE_PV_STAMP_CHOL
  CI_STAMP(3);
#endif

  // 2. L^-1 in place by recursive doubling (levels of 64, 128, 256 rows; see spd_sweep.hip's pivot)
  if (w < 4) {
    const int a = 2 * w;
    pv_f32x16 X = {}, Y = {};
    pv_mma<false, true>(X, pv_blk(lf, a + 1, a), pv_blk(lf, a, a), rl, hh);
    const float* Ci = pv_blk(lf, a + 1, a + 1);
#pragma unroll
    for (int s = 0; s < 16; ++s)
      Y = __builtin_amdgcn_mfma_f32_32x32x2f32(Ci[rl * kPvL + pv_row(s, hh)], X[s], Y, 0, 0, 0);
    pv_store(Y, pv_blk(lf, a + 1, a), rl, hh, -1.f);
  }
  __syncthreads();
#pragma unroll 1
  for (int lv = 1; lv <= 2; ++lv) {
    pv_block_scales(lf, bsc, w, lane, rl, hh);
    const int h = 1 << lv;
    const int per = h * h;
    const int inst = w / per, t = w % per;
    const bool act = inst < 4 / h;
    const int o = 2 * h * inst;
    const int i = o + h + t / h, j = o + t % h;
    const int nij = i * (i + 1) / 2 + j;
    pv_f32x16 acc = {};
    if (act)
      for (int k = j; k < o + h; ++k) {
        const int a = i * (i + 1) / 2 + k, b = k * (k + 1) / 2 + j;
        pv_mma3<false, true>(acc, lf + a * kPvBlk, lf + b * kPvBlk, bsc[a], bsc[b], rl, hh);
      }
    __syncthreads();
    if (act) {
      pv_store(acc, pv_blk(lf, i, j), rl, hh);
      float m = 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e) m = fmaxf(m, fabsf(acc[e]));
#pragma unroll
      for (int q = 32; q > 0; q >>= 1) m = fmaxf(m, __shfl_xor(m, q, 64));
      if (lane == 0) bsc[nij] = x3_scale(m);
    }
    __syncthreads();
    acc = pv_f32x16{};
    if (act)
      for (int k = o + h; k <= i; ++k) {
        const int a = i * (i + 1) / 2 + k, b = k * (k + 1) / 2 + j;
        pv_mma3<false, true>(acc, lf + a * kPvBlk, lf + b * kPvBlk, bsc[a], bsc[b], rl, hh);
      }
    __syncthreads();
    if (act) pv_store(acc, pv_blk(lf, i, j), rl, hh, -1.f);
    __syncthreads();
  }

#ifndef LVAE_PV_STAMP_CHOL
  CI_STAMP(4);
#endif
  // 3. max |Y_kk| -> its split scale; out: D (row-major planes; the diagonal copy puts them into the
  //    Y and Y^T planes after potrf).  Thread (r0 = tid >> 6, c = 4 (tid & 63)) covers rows r0, r0 + 16,
  //    ... (a wave writes one whole row: half4 runs).
  {
    float m = 0.f;
    for (int e = tid; e < kPvBlocks * 1024; e += 1024) {
      const int n = e >> 10, r = (e >> 5) & 31, c = e & 31;
      m = fmaxf(m, fabsf(lf[n * kPvBlk + r * kPvL + c]));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if (lane == 0) atomicMax(&ymax_s, __float_as_uint(m));
  }
  __syncthreads();
  const float sY = x3_scale(__uint_as_float(ymax_s));
  const int c = 4 * (tid & 63);
  const int64_t od = ((int64_t)l * S.nt + kb) * kSwBB;
  _Float16* dh = S.Dh + od;
  _Float16* dl = S.Dl + od;
  for (int r = tid >> 6; r < kSwB; r += 16) {
    x3_half4 h4, l4;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int cq = c + q;
      const float v = r >= cq ? pv_blk(lf, r >> 5, cq >> 5)[(r & 31) * kPvL + (cq & 31)] : 0.f;  // Y(r, cq)
      const float y = v * sY;
      const _Float16 yh = (_Float16)y;
      h4[q] = yh;
      l4[q] = (_Float16)(y - (float)yh);
    }
    *reinterpret_cast<x3_half4*>(dh + r * kSwB + c) = h4;
    *reinterpret_cast<x3_half4*>(dl + r * kSwB + c) = l4;
  }
  if (w == 0 && lane == 0) bad_s = bad;
  __syncthreads();
#ifdef LVAE_PV_STAMP_CHOL
  CI_STAMPX(18);
#else
  CI_STAMP(5);
#endif
  if (tid == 0) {
    S.ysc[((int64_t)l * S.nt + kb) * S.nt + kb] = sY;
    logdet[l] += ld;
    if (bad_s != INT_MAX && info[l] == 0) info[l] = kb * kSwB + bad_s + 1;
  }
}

__device__ inline void ci_split4(f32x4 v, float s, _Float16* __restrict__ hi, _Float16* __restrict__ lo) {
  x3_half4 h, l;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float y = v[e] * s;
    const _Float16 hh = (_Float16)y;
    h[e] = hh;
    l[e] = (_Float16)(y - (float)hh);
  }
  *reinterpret_cast<x3_half4*>(hi) = h;
  *reinterpret_cast<x3_half4*>(lo) = l;
}

// 256 x 256 accumulator tile (value = acc * mul) out TRANSPOSED through the 128 KB LDS stage:
// fn(c, r0, v), v = (value(r0 + q, c))_{q < 4}; every (c, r0) once.  Starts with a barrier.
template <typename Fn>
__device__ inline void ci_transposed_out(const sx_f32x16 (&acc)[4][2], float mul, _Float16* lds, Fn fn) {
  float* U = reinterpret_cast<float*>(lds);
  const int tid = threadIdx.x, w = tid >> 6;
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    __syncthreads();
    if ((w >> 2) == hh) {
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int e = 0; e < 16; ++e)
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            const int rl = sx_row(a, e) - 128 * hh, c = sx_col(b);
            U[c * 128 + (rl ^ ((c & 31) << 2))] = acc[a][b][e] * mul;
          }
    }
    __syncthreads();
    const int t4 = tid & 31;
#pragma unroll 4
    for (int cc = 0; cc < kSwB; cc += 16) {
      const int c = cc + (tid >> 5), rl = 4 * t4;
      fn(c, 128 * hh + rl, *reinterpret_cast<const f32x4*>(&U[c * 128 + (rl ^ ((c & 31) << 2))]));
    }
  }
}

// accumulator tile (value = acc * mul) -> fp16 planes hi / lo (row stride ld halves) scaled by s
__device__ inline void ci_planes_out(const sx_f32x16 (&acc)[4][2], float mul, float s, _Float16* __restrict__ hi,
                                     _Float16* __restrict__ lo, int64_t ld) {
  const float m = mul * s;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int r = sx_row(a, e), c = sx_col(b);
        const float y = acc[a][b][e] * m;
        const _Float16 yh = (_Float16)y;
        hi[r * ld + c] = yh;
        lo[r * ld + c] = (_Float16)(y - (float)yh);
      }
}

// as ci_planes_out through buffer stores (offsets from compile-time parts: fewer address registers beside the
// c16 core's fragment sets)
__device__ inline void ci_planes_out_buf(const sx_f32x16 (&acc)[4][2], float mul, float s, _Float16* __restrict__ hi,
                                         _Float16* __restrict__ lo, int ld) {
  const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc(hi, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(lo, (short)0, 0x7fffffff, 0x00020000);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int vb = (((w >> 2) * 128 + 4 * (lane >> 5)) * ld + (w & 3) * 64 + (lane & 31)) * 2;
  const float m = mul * s;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const float y = acc[a][b][e] * m;
        const _Float16 yh = (_Float16)y;
        const _Float16 yl = (_Float16)(y - (float)yh);
        const int so = ((32 * a + (e & 3) + 8 * (e >> 2)) * ld + 32 * b) * 2;
        __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, yh), rh, vb, so, 0);
        __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, yl), rl, vb, so, 0);
      }
}

__device__ inline float ci_acc_absmax(const sx_f32x16 (&acc)[4][2]) {
  float m = 0.f;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) m = fmaxf(m, fabsf(acc[a][b][e]));
  return m;
}

// ------------------------------------------------------------------------------------------
// pass-0 C operand: blocks i >= 1 of column 0 of A, each with the split scale of its exact max.
// grid (nt - 1, L), 256 threads.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void ci_prep0_kernel(const float* __restrict__ Aall, int np_, CiScratch S,
                                                       int col = 0) {
  __shared__ uint32_t red;
  const int l = blockIdx.y, i = col + 1 + blockIdx.x, t = threadIdx.x;
  const float* T = Aall + (int64_t)l * np_ * np_ + (int64_t)i * kSwB * np_ + (int64_t)col * kSwB;
  if (t == 0) red = 0u;
  float m = 0.f;
  for (int e = t; e < kSwBB / 4; e += 256) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(T + (int64_t)(e >> 6) * np_ + (e & 63) * 4);
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
  }
  __syncthreads();
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((t & 63) == 0) atomicMax(&red, __float_as_uint(m));
  __syncthreads();
  const float sc = x3_scale(__uint_as_float(red));
  const int64_t o = (int64_t)l * np_ * kSwB + (int64_t)i * kSwBB;
  for (int e = t; e < kSwBB / 4; e += 256) {
    const int r = e >> 6, c = (e & 63) * 4;
    const f32x4 v = *reinterpret_cast<const f32x4*>(T + (int64_t)r * np_ + c);
    ci_split4(v, sc, S.Ch[col & 1] + o + r * kSwB + c, S.Cl[col & 1] + o + r * kSwB + c);
  }
  if (t == 0) S.c_scale(l, col, i) = sc;
}

// ------------------------------------------------------------------------------------------
// panel(k): L_ik = C_i Y_kk^T for i > k (C_i: block i of pass k's C planes; Y_kk rows from D), one
// 512-thread workgroup per block, grid (nt - k - 1, L) -> the planes of L, tile (i, k), with the split
// scale of the block's exact max.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(512) void ci_panel_kernel(CiScratch S, int np_, int k) {
  __shared__ __attribute__((aligned(16))) _Float16 lds[2 * 4 * kSxPart];
  __shared__ uint32_t red;
  const int l = blockIdx.y, i = k + 1 + blockIdx.x;
  const int64_t oc = (int64_t)l * np_ * kSwB + (int64_t)i * kSwBB, od = ((int64_t)l * S.nt + k) * kSwBB;
  if (threadIdx.x == 0) red = 0u;
  sx_f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = sx_f32x16{};
  sx_gemm(S.Ch[k & 1] + oc, S.Cl[k & 1] + oc, S.Dh + od, S.Dl + od, kSwB, kSwB, lds, acc);
  const float inv = 1.0f / (S.c_scale(l, k, i) * S.ysc[((int64_t)l * S.nt + k) * S.nt + k]);
  const float sl = x3_scale(sw_block_max(ci_acc_absmax(acc) * inv, &red));
  const int64_t ot = (int64_t)l * np_ * np_ + (int64_t)i * kSwB * np_ + k * kSwB;
  ci_planes_out(acc, inv, sl, S.Lh + ot, S.Ll + ot, np_);
  if (threadIdx.x == 0) S.lsc[((int64_t)l * S.nt + i) * S.nt + k] = sl;
  if (S.lout) {  // (potrf-only) L_ik in fp32 into tile (i, k) of lout
    float* O = S.lout + ot;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int e = 0; e < 16; ++e) O[(int64_t)sx_row(a, e) * np_ + sx_col(b)] = acc[a][b][e] * inv;
  }
}

// ------------------------------------------------------------------------------------------
// update(k): A_IJ -= L_Ik L_Jk^T on lower 256-tiles, K = 256, one 512-thread workgroup per tile on the
// pre-split planes of L (DMA-staged, double-buffered chunks of 32); A enters in 8 chunks of 16
// accumulator elements INSIDE the K loop (non-temporal: the A stream does not evict the planes), as in
// the sweep's update (spd_sweep.hip).  MODE:
//   kCiU1  column k+1 (tiles (I, k+1), I >= k+1 with the next pivot block, I >= k+2 without it):
//          written as the planes of pass k+1's C operand (the diagonal tile in fp32, for the pivot)
//   kCiU2  the trailing tiles I >= J >= k+2, in place
// ------------------------------------------------------------------------------------------
constexpr int kCiU2 = 0, kCiU1 = 1, kCiU12 = 2;  // kCiU12: U1 (without the pivot block) + U2, one launch
constexpr int kCiFuseMaxL = 16; // latent dims per call up to which the pivot updates its own block
template <int MODE>
__global__ __launch_bounds__(512) void ci_update_kernel(float* __restrict__ Aall, CiScratch S, int np_, int k,
                                                        int ntl, int nwg, int n1 = 0, int t0 = 0) {
  __shared__ __attribute__((aligned(16))) _Float16 lds[2 * 4 * kSxPart];
  __shared__ uint32_t red;
  if (MODE != kCiU2 && threadIdx.x == 0) red = 0u;
  const int nt = np_ / kSwB;
  // kCiU12: workgroups [0, n1 L) are column k+1's tiles (dispatched first: the next pass's C operand),
  // the rest the trailing tiles; ntl / nwg describe the trailing part
  const bool u1 = MODE == kCiU1 || (MODE == kCiU12 && (int)blockIdx.x < n1 * (nwg / max(ntl, 1)));
  int l, I, J;
  if (MODE == kCiU12 && u1) {
    l = blockIdx.x / n1;
    I = k + 2 + blockIdx.x % n1;
    J = k + 1;
  } else {
    const int orig = MODE == kCiU12 ? blockIdx.x - n1 * (nwg / ntl) : blockIdx.x;
    const int xcd = orig % 8, q8 = nwg / 8, r8 = nwg % 8;
    const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
    l = wgid / ntl;
    const int t = t0 + wgid % ntl;  // (t0: the launch's first trailing tile, lookahead split)
    if constexpr (MODE == kCiU1) {
      I = (ntl == nt - k - 1) ? k + 1 + t : k + 2 + t;  // with / without the pivot block
      J = k + 1;
    } else {
      sx_tri_blocked(t, nt - k - 2, I, J);
      I += k + 2;
      J += k + 2;
    }
  }
  const int64_t np2 = (int64_t)np_ * np_;
  float* C = Aall + l * np2 + (int64_t)I * kSwB * np_ + J * kSwB;
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(C, (short)0, 0x7fffffff, 0x00020000);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int vo = (((w >> 2) * 128 + 4 * (lane >> 5)) * np_ + (w & 3) * 64 + (lane & 31)) * 4;
  const int64_t oa = l * np2 + (int64_t)I * kSwB * np_ + k * kSwB, ob = l * np2 + (int64_t)J * kSwB * np_ + k * kSwB;
  const float cs = S.lsc[((int64_t)l * S.nt + I) * S.nt + k] * S.lsc[((int64_t)l * S.nt + J) * S.nt + k];
  const float ncs = -cs, ninv = -1.0f / cs;  // acc = L_I L_J^T - A (units of cs); the result is -acc / cs
  const _Float16* ah = S.Lh + oa;
  const _Float16* al = S.Ll + oa;
  const _Float16* bh = S.Lh + ob;
  const _Float16* bl = S.Ll + ob;
  sx_f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = sx_f32x16{};
  constexpr int CAUX = 2;
  float cv[2][16];
  constexpr int nk = kSwB / kSxBK;
  sx_issue(ah, al, bh, bl, np_, 0, lds);
#pragma unroll
  for (int s = 0; s < nk; ++s) {
    if (s == 0) SX_WAIT_VM(0);
    else __builtin_amdgcn_s_waitcnt(0x4F70);  // vmcnt(16): DMA s and A chunk s - 2 landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + 1 < nk) sx_issue(ah, al, bh, bl, np_, (s + 1) * kSxBK, lds + ((s + 1) & 1) * 4 * kSxPart);
    if (s >= 2) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int i = 16 * (s - 2) + q, a = i >> 5, e = (i >> 1) & 15, b = i & 1;
        acc[a][b][e] += cv[s & 1][q] * ncs;
      }
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int i = 16 * s + q, a = i >> 5, e = (i >> 1) & 15, b = i & 1;
      cv[s & 1][q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
          rc, vo, ((32 * a + (e & 3) + 8 * (e >> 2)) * np_ + 32 * b) * 4, CAUX));
    }
    __builtin_amdgcn_s_setprio(1);
    sx_mma_stage(lds + (s & 1) * 4 * kSxPart, acc);
    __builtin_amdgcn_s_setprio(0);
  }
#pragma unroll
  for (int j = nk - 2; j < nk; ++j)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int i = 16 * j + q, a = i >> 5, e = (i >> 1) & 15, b = i & 1;
      acc[a][b][e] += cv[j & 1][q] * ncs;
    }
  if (u1 && I != J) {
    // a block of column k+1 = block I of the next pass's C operand: straight to its planes
    const float sc = x3_scale(sw_block_max(ci_acc_absmax(acc) * fabsf(ninv), &red));
    const int64_t on = (int64_t)l * np_ * kSwB + (int64_t)I * kSwBB;
    ci_planes_out(acc, ninv, sc, S.Ch[(k + 1) & 1] + on, S.Cl[(k + 1) & 1] + on, kSwB);
    if (threadIdx.x == 0) S.c_scale(l, k + 1, I) = sc;
  } else {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int e = 0; e < 16; ++e)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[a][b][e] * ninv), rc, vo,
                                                ((32 * a + (e & 3) + 8 * (e >> 2)) * np_ + 32 * b) * 4, CAUX);
  }
}

// ------------------------------------------------------------------------------------------
// The trailing update (U1 + U2 as ci_update_kernel<kCiU12>) with a deeper DMA pipeline (r6, opt-in LVAE_CI_URING=1:
// measured slower, 211 vs 166 us per launch -- twice the barriers per tile and 32-B row pieces): 16-deep
// K stages in a ring of 4 (4 x 32 KB of LDS, the same 128 KB as the 2 x 32-deep double buffer), each stage's DMA
// issued THREE stages ahead, so that ~3 stages of MFMAs (~2.2 us) cover an HBM round trip instead of one (the
// double-buffered form waits on most chunks' DMA: 0.26 MFMA-busy, 0.29 of HBM).  The A tile streams in 16 pieces
// of 8 accumulator elements, each consumed three stages after its loads were issued; one counted vmcnt per stage
// covers both (every stage issues a DMA -- past the last chunk a re-read into a dead buffer -- so the count is
// uniform).  LDS rows of 16 halves (32 B): the two 8-half groups swapped on bit 3 of the row (the c16 planes'
// swizzle), so a ds_read_b128 phase of 16 consecutive rows covers all 64 banks.
// ------------------------------------------------------------------------------------------
constexpr int kU16K = 16, kU16Part = kSwB * kU16K, kU16Ring = 4;

// one stage's DMA: 4 parts x 256 rows x 32 B, one 1 KB instruction per part and wave (4 per thread)
__device__ inline void u16_issue(const _Float16* __restrict__ ah, const _Float16* __restrict__ al,
                                 const _Float16* __restrict__ bh, const _Float16* __restrict__ bl, int64_t ld, int k0,
                                 _Float16* __restrict__ stage) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const _Float16* src[4] = {ah, al, bh, bl};
  // wave w, instruction p: part p, rows 32 w .. 32 w + 31 (2 lanes per row); LDS image [row][16] linear per wave,
  // the global source's 8-half group chosen so that physical group (lane & 1) holds logical group (lane & 1) ^ bit 3
  const int row = 32 * w + (lane >> 1), g = (lane & 1) ^ ((row >> 3) & 1);
  const int64_t go = (int64_t)row * ld + k0 + 8 * g;
#pragma unroll
  for (int p = 0; p < 4; ++p)
    __builtin_amdgcn_global_load_lds((const void*)(src[p] + go), (void*)(stage + p * kU16Part + w * 512), 16, 0, 0);
}

__device__ inline sx_half8 u16_frag(const _Float16* __restrict__ part, int row, int h) {
  return *reinterpret_cast<const sx_half8*>(part + row * kU16K + ((h ^ ((row >> 3) & 1)) << 3));
}

// one 16-deep stage: acc[a][b] += A rows x B rows (x3 products), the wave's 128 x 64 (sx_mma_stage's layout)
__device__ inline void u16_mma_stage(const _Float16* __restrict__ cur, sx_f32x16 (&acc)[4][2]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w >> 2) * 128, wn = (w & 3) * 64, r32 = lane & 31, kh = lane >> 5;
  sx_half8 bH[2], bL[2];
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    bH[b] = u16_frag(cur + 2 * kU16Part, wn + 32 * b + r32, kh);
    bL[b] = u16_frag(cur + 3 * kU16Part, wn + 32 * b + r32, kh);
  }
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const sx_half8 aH = u16_frag(cur, wm + 32 * a + r32, kh);
    const sx_half8 aL = u16_frag(cur + kU16Part, wm + 32 * a + r32, kh);
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(aL, bH[b], acc[a][b], 0, 0, 0);
      acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(aH, bL[b], acc[a][b], 0, 0, 0);
      acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(aH, bH[b], acc[a][b], 0, 0, 0);
    }
  }
}

// MODE and arguments as ci_update_kernel (kCiU12 / kCiU2 / kCiU1)
template <int MODE>
__global__ __launch_bounds__(512) void ci_update_ring_kernel(float* __restrict__ Aall, CiScratch S, int np_, int k,
                                                             int ntl, int nwg, int n1 = 0) {
  __shared__ __attribute__((aligned(16))) _Float16 lds[kU16Ring * 4 * kU16Part];
  __shared__ uint32_t red;
  if (MODE != kCiU2 && threadIdx.x == 0) red = 0u;
  const int nt = np_ / kSwB;
  const bool u1 = MODE == kCiU1 || (MODE == kCiU12 && (int)blockIdx.x < n1 * (nwg / max(ntl, 1)));
  int l, I, J;
  if (MODE == kCiU12 && u1) {
    l = blockIdx.x / n1;
    I = k + 2 + blockIdx.x % n1;
    J = k + 1;
  } else {
    const int orig = MODE == kCiU12 ? blockIdx.x - n1 * (nwg / ntl) : blockIdx.x;
    const int xcd = orig % 8, q8 = nwg / 8, r8 = nwg % 8;
    const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
    l = wgid / ntl;
    const int t = wgid % ntl;
    if constexpr (MODE == kCiU1) {
      I = (ntl == nt - k - 1) ? k + 1 + t : k + 2 + t;
      J = k + 1;
    } else {
      sx_tri_blocked(t, nt - k - 2, I, J);
      I += k + 2;
      J += k + 2;
    }
  }
  const int64_t np2 = (int64_t)np_ * np_;
  float* C = Aall + l * np2 + (int64_t)I * kSwB * np_ + J * kSwB;
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(C, (short)0, 0x7fffffff, 0x00020000);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int vo = (((w >> 2) * 128 + 4 * (lane >> 5)) * np_ + (w & 3) * 64 + (lane & 31)) * 4;
  const int64_t oa = l * np2 + (int64_t)I * kSwB * np_ + k * kSwB, ob = l * np2 + (int64_t)J * kSwB * np_ + k * kSwB;
  const float cs = S.lsc[((int64_t)l * S.nt + I) * S.nt + k] * S.lsc[((int64_t)l * S.nt + J) * S.nt + k];
  const float ncs = -cs, ninv = -1.0f / cs;  // acc = L_I L_J^T - A (units of cs); the result is -acc / cs
  const _Float16* ah = S.Lh + oa;
  const _Float16* al = S.Ll + oa;
  const _Float16* bh = S.Lh + ob;
  const _Float16* bl = S.Ll + ob;
  sx_f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = sx_f32x16{};
  constexpr int CAUX = 2;
  constexpr int nk = kSwB / kU16K;  // 16 stages; 128 A elements per thread, 8 per stage
  float cv[4][8];
  auto a_load = [&](int s, float (&dst)[8]) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int i = 8 * s + q, a = i >> 5, e = (i >> 1) & 15, b = i & 1;
      dst[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
          rc, vo, ((32 * a + (e & 3) + 8 * (e >> 2)) * np_ + 32 * b) * 4, CAUX));
    }
  };
  auto a_add = [&](int s, const float (&src)[8]) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int i = 8 * s + q, a = i >> 5, e = (i >> 1) & 15, b = i & 1;
      acc[a][b][e] += src[q] * ncs;
    }
  };
#pragma unroll
  for (int s = 0; s < kU16Ring - 1; ++s) u16_issue(ah, al, bh, bl, np_, s * kU16K, lds + s * 4 * kU16Part);
#pragma unroll
  for (int s = 0; s < nk; ++s) {
    // issued after DMA s: DMA s+1, s+2 (4 each) and the A pieces s-3 .. s-1 (8 each) -- DMA s and A piece s-3 landed
    if (s == 0) SX_WAIT_VM(8);
    else if (s == 1) __builtin_amdgcn_s_waitcnt(0x4F70);  // vmcnt(16)
    else __builtin_amdgcn_s_waitcnt(0x4F78);              // vmcnt(24)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // stage s in LDS for every wave; every wave's reads of stage s-1 retired
    const int sn = s + kU16Ring - 1 < nk ? s + kU16Ring - 1 : nk - 1;  // (past the end: a re-read into a dead buffer)
    u16_issue(ah, al, bh, bl, np_, sn * kU16K, lds + ((s + kU16Ring - 1) % kU16Ring) * 4 * kU16Part);
    a_load(s, cv[s & 3]);
    if (s >= 3) a_add(s - 3, cv[(s - 3) & 3]);
    __builtin_amdgcn_s_setprio(1);
    u16_mma_stage(lds + (s % kU16Ring) * 4 * kU16Part, acc);
    __builtin_amdgcn_s_setprio(0);
  }
  SX_WAIT_VM(0);
#pragma unroll
  for (int j = nk - 3; j < nk; ++j) a_add(j, cv[j & 3]);
  if (u1 && I != J) {
    // a block of column k+1 = block I of the next pass's C operand: straight to its planes
    const float sc = x3_scale(sw_block_max(ci_acc_absmax(acc) * fabsf(ninv), &red));
    const int64_t on = (int64_t)l * np_ * kSwB + (int64_t)I * kSwBB;
    ci_planes_out(acc, ninv, sc, S.Ch[(k + 1) & 1] + on, S.Cl[(k + 1) & 1] + on, kSwB);
    if (threadIdx.x == 0) S.c_scale(l, k + 1, I) = sc;
  } else {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int e = 0; e < 16; ++e)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[a][b][e] * ninv), rc, vo,
                                                ((32 * a + (e & 3) + 8 * (e >> 2)) * np_ + 32 * b) * 4, CAUX);
  }
}

// ------------------------------------------------------------------------------------------
// U2 on 128 x 128 sub-tiles (r6, opt-in LVAE_CI_U128=1; measured slower in the step, see ci_factor_f32): A_IJ -=
// L_Ik L_Jk^T for the lower tiles I >= J >= k+2,
// each 256-tile as four 256-thread workgroups of 128 x 128 (the upper-right quarter of a diagonal tile skipped: no
// reader needs A's strict upper part), K = 256 in 8 DMA-staged chunks of 32, double-buffered: 64 KB of LDS and
// ~128 VGPRs per workgroup, so TWO workgroups share a CU and each one's HBM round trips and barriers hide under
// the other's MFMAs (the 256-tile form holds a CU alone: 128 KB of LDS, 2 waves per SIMD, and stalls on every
// chunk's DMA).  The A tile streams in 8 pieces of 8 accumulator elements inside the K loop, as in
// ci_update_kernel.  Waves 2 x 2, 64 x 64 each = 2 x 2 blocks of v_mfma_f32_32x32x16_f16 x 3 products.
// ------------------------------------------------------------------------------------------
constexpr int kU8Rows = 128, kU8Part = kU8Rows * kSxBK;  // rows per operand part; halves per part and stage

// one stage: 4 parts (A hi, A lo, B hi, B lo) x 8 blocks of 16 rows (1 KB each); wave w issues blocks 2w, 2w+1
__device__ inline void u8_issue(const _Float16* __restrict__ ah, const _Float16* __restrict__ al,
                                const _Float16* __restrict__ bh, const _Float16* __restrict__ bl, int64_t ld, int k0,
                                _Float16* __restrict__ stage) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const _Float16* src[4] = {ah, al, bh, bl};
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int blk = 2 * w + q;
    const int row = 16 * blk + (lane >> 2);
    const int c = (lane & 3) ^ ((row >> 2) & 3);  // logical chunk stored at physical chunk lane & 3 (sx_frag's)
    const int64_t go = (int64_t)row * ld + k0 + 8 * c;
#pragma unroll
    for (int p = 0; p < 4; ++p)
      __builtin_amdgcn_global_load_lds((const void*)(src[p] + go), (void*)(stage + p * kU8Part + blk * 512), 16, 0, 0);
  }
}

// one 32-deep stage of the wave's 64 x 64: acc[a][b] (a, b < 2) += A rows x B rows (three products each)
__device__ inline void u8_mma_stage(const _Float16* __restrict__ cur, sx_f32x16 (&acc)[2][2]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w >> 1) * 64, wn = (w & 1) * 64, r32 = lane & 31, kh = lane >> 5;
#pragma unroll
  for (int ks = 0; ks < kSxBK / 16; ++ks) {
    const int c = 2 * ks + kh;
    sx_half8 bH[2], bL[2];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      bH[b] = sx_frag(cur + 2 * kU8Part, wn + 32 * b + r32, c);
      bL[b] = sx_frag(cur + 3 * kU8Part, wn + 32 * b + r32, c);
    }
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const sx_half8 aH = sx_frag(cur, wm + 32 * a + r32, c);
      const sx_half8 aL = sx_frag(cur + kU8Part, wm + 32 * a + r32, c);
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(aL, bH[b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(aH, bL[b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(aH, bH[b], acc[a][b], 0, 0, 0);
      }
    }
  }
}

// grid: 4 ntl L workgroups (ntl trailing 256-tiles per dim, pass k), XCD-contiguous like ci_update_kernel
__global__ __launch_bounds__(256, 2) void ci_update128_kernel(float* __restrict__ Aall, CiScratch S, int np_, int k,
                                                              int ntl, int nwg, int n1 = 0) {
  __shared__ __attribute__((aligned(16))) _Float16 lds[2 * 4 * kU8Part];
  const int nt = np_ / kSwB;
  const int orig = blockIdx.x, xcd = orig % 8, q8 = nwg / 8, r8 = nwg % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int per = 4 * (n1 + ntl), l = wgid / per, t = (wgid % per) >> 2, si = (wgid & 3) >> 1, sj = wgid & 1;
  int I, J;
  if (t < n1) {  // column k+1's tiles (without the pivot block): fp32 into A, split by ci_prep0_kernel(col k+1)
    I = k + 2 + t;
    J = k + 1;
  } else {
    sx_tri_blocked(t - n1, nt - k - 2, I, J);
    I += k + 2;
    J += k + 2;
  }
  if (I == J && si < sj) return;  // (uniform) the diagonal tile's upper-right quarter
  const int64_t np2 = (int64_t)np_ * np_;
  const int r0 = I * kSwB + si * kU8Rows, c0 = J * kSwB + sj * kU8Rows;
  float* C = Aall + l * np2 + (int64_t)r0 * np_ + c0;
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(C, (short)0, 0x7fffffff, 0x00020000);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // accumulator element (a, e, b) of this lane: row (w >> 1) 64 + 32 a + (e & 3) + 8 (e >> 2) + 4 (lane >> 5),
  // column (w & 1) 64 + 32 b + (lane & 31)
  const int vo = (((w >> 1) * 64 + 4 * (lane >> 5)) * np_ + (w & 1) * 64 + (lane & 31)) * 4;
  const int64_t oa = l * np2 + (int64_t)r0 * np_ + k * kSwB, ob = l * np2 + (int64_t)c0 * np_ + k * kSwB;
  const float cs = S.lsc[((int64_t)l * S.nt + I) * S.nt + k] * S.lsc[((int64_t)l * S.nt + J) * S.nt + k];
  const float ncs = -cs, ninv = -1.0f / cs;  // acc = L_I L_J^T - A (units of cs); the result is -acc / cs
  const _Float16* ah = S.Lh + oa;
  const _Float16* al = S.Ll + oa;
  const _Float16* bh = S.Lh + ob;
  const _Float16* bl = S.Ll + ob;
  sx_f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = sx_f32x16{};
  constexpr int CAUX = 2;
  constexpr int nk = kSwB / kSxBK;  // 8 chunks; 64 A elements per thread, 8 per chunk
  float cv[2][8];
  u8_issue(ah, al, bh, bl, np_, 0, lds);
#pragma unroll
  for (int s = 0; s < nk; ++s) {
    if (s == 0) SX_WAIT_VM(0);
    else __builtin_amdgcn_s_waitcnt(0x0F78);  // vmcnt(8): DMA s and A piece s - 2 landed (A piece s - 1 may fly)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + 1 < nk) u8_issue(ah, al, bh, bl, np_, (s + 1) * kSxBK, lds + ((s + 1) & 1) * 4 * kU8Part);
    if (s >= 2) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int i = 8 * (s - 2) + q, a = i >> 5, e = (i >> 1) & 15, b = i & 1;
        acc[a][b][e] += cv[s & 1][q] * ncs;
      }
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int i = 8 * s + q, a = i >> 5, e = (i >> 1) & 15, b = i & 1;
      cv[s & 1][q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
          rc, vo, ((32 * a + (e & 3) + 8 * (e >> 2)) * np_ + 32 * b) * 4, CAUX));
    }
    __builtin_amdgcn_s_setprio(1);
    u8_mma_stage(lds + (s & 1) * 4 * kU8Part, acc);
    __builtin_amdgcn_s_setprio(0);
  }
#pragma unroll
  for (int j = nk - 2; j < nk; ++j)
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int i = 8 * j + q, a = i >> 5, e = (i >> 1) & 15, b = i & 1;
      acc[a][b][e] += cv[j & 1][q] * ncs;
    }
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int e = 0; e < 16; ++e)
#pragma unroll
      for (int b = 0; b < 2; ++b)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[a][b][e] * ninv), rc, vo,
                                              ((32 * a + (e & 3) + 8 * (e >> 2)) * np_ + 32 * b) * 4, CAUX);
}

// D (the pivots' Y_kk planes) -> the diagonal tiles of the row-major Y planes (after potrf: the Y
// planes alias A) and, transposed through LDS, of the Y^T planes.  grid (16 nt, L): one 256-thread
// workgroup per 64 x 64 piece (a, b) of a diagonal tile, Y (a, b) = D (a, b) and Y^T (b, a) = D (a, b)^T.
__global__ __launch_bounds__(256) void ci_diag_copy_kernel(CiScratch S, int np_, _Float16* __restrict__ Yh,
                                                           _Float16* __restrict__ Yl, _Float16* __restrict__ YTh,
                                                           _Float16* __restrict__ YTl) {
  __shared__ _Float16 tp[2][64][66];
  const int k = blockIdx.x >> 4, pa = (blockIdx.x >> 2) & 3, pb = blockIdx.x & 3, l = blockIdx.y, t = threadIdx.x;
  const int64_t od = ((int64_t)l * S.nt + k) * kSwBB + (int64_t)(64 * pa) * kSwB + 64 * pb;
  const int64_t ot = (int64_t)l * np_ * np_ + (int64_t)k * kSwB * np_ + k * kSwB;
  const int64_t oy = ot + (int64_t)(64 * pa) * np_ + 64 * pb, oyt = ot + (int64_t)(64 * pb) * np_ + 64 * pa;
  for (int e = t; e < 64 * 8; e += 256) {  // rows of 8-half vectors: direct copy + LDS image
    const int r = e >> 3, c = (e & 7) * 8;
    const x3_half8 h = *reinterpret_cast<const x3_half8*>(S.Dh + od + r * kSwB + c);
    const x3_half8 lo = *reinterpret_cast<const x3_half8*>(S.Dl + od + r * kSwB + c);
    // (chunk-major: an aligned 8-half run stays one 16-B run under the swizzle)
    const int64_t oyc = kCiC16 ? c16_off(l, np_, k * kSwB + 64 * pa + r, k * kSwB + 64 * pb + c) : oy + (int64_t)r * np_ + c;
    *reinterpret_cast<x3_half8*>(Yh + oyc) = h;
    *reinterpret_cast<x3_half8*>(Yl + oyc) = lo;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      tp[0][r][c + q] = h[q];
      tp[1][r][c + q] = lo[q];
    }
  }
  __syncthreads();
  for (int e = t; e < 64 * 8; e += 256) {  // Y^T (b, a) row c, columns r0 .. r0 + 7 = D (a, b) (r, c): 16-B stores
    const int c = e >> 3, r0 = (e & 7) * 8;
    x3_half8 h, lo;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      h[q] = tp[0][r0 + q][c];
      lo[q] = tp[1][r0 + q][c];
    }
    const int64_t o = kCiC16 ? c16_off(l, np_, k * kSwB + 64 * pb + c, k * kSwB + 64 * pa + r0) : oyt + (int64_t)c * np_ + r0;
    *reinterpret_cast<x3_half8*>(YTh + o) = h;
    *reinterpret_cast<x3_half8*>(YTl + o) = lo;
  }
}

// ------------------------------------------------------------------------------------------
// ci_gemm_kernel<MODE>: out tile (i, j) = sum_{kb in [kb0, kb1)} A(i, kb) B(kb, j) over whole 256-blocks
// on the x3 DMA tile machinery (x3_dma.hpp), operands from full [L, np, np] plane arrays (row stride np:
// the K range of a row is contiguous), the accumulators rescaled at every block boundary to the new
// block pair's split scales (powers of two: exact).
//   kCiX  (trtri, step 1): X_ij = sum_{k=j}^{o+h-1} L_ik Y_kj      A = L planes (i, k),  B = Y^T planes (j, k)
//                          -> X^T planes, tile (j, i) (transposed out), scale xsc(i, j)
//   kCiY  (trtri, step 2): Y_ij = -sum_{k=o+h}^{i} Y_ik X_kj      A = Y planes (i, k),  B = X^T planes (j, k)
//                          -> Y planes (i, j) and Y^T planes (j, i), scale ysc(i, j)
//   kCiLauum:  (K^-1)_IJ = sum_{k>=I} Y_kI^T Y_kJ                  A = Y^T planes (I, k), B = Y^T planes (J, k)
//                          -> Kinv (I, J) and its mirror (J, I), fp32
// trtri launches cover every (instance m, ii, jj) of level h: i = o + h + ii, j = o + jj, o = 2 h m
// (workgroups with i >= nt exit at once); lauum the L nt (nt + 1) / 2 lower tiles.
// ------------------------------------------------------------------------------------------
constexpr int kCiX = 0, kCiY = 1, kCiLauum = 2, kCiLauumKL = 3;
// pipelined trtri (ci_pipe_alloc; h = the pass m):
//   kCiTrY  rowY(m): tile j < m: Y_mj = -Y_mm X_mj   A = D_m (row-major planes), B = the X^T row planes (j)
//                    of parity m & 1 -> Y^T planes tile (j, m) (transposed out), scale ysc(m, j); workgroups
//                    t >= m: the 16 64 x 64 pieces of Y^T (m, m) = D_m^T
//   kCiTrX  Xupd(m): tile (i, j), i > m, j <= m: X_ij (+)= L_im Y_mj   A = L planes (i, m), B = Y^T planes
//                    (j, m) -> fp32 X in g.Kinv (written at j == m, accumulated after), or for i == m + 1 (its
//                    last term) the X^T row planes of parity (m + 1) & 1, scale xsc(m + 1, j); workgroups
//                    t >= g.inst0 (mode 2): Lupd(m), tile (I, J), J <= I <= m: K^-1_IJ (+)= Y_mI^T Y_mJ
//                    (A, B = Y^T planes (I, m), (J, m); written at m == I) into g.Kinv
constexpr int kCiTrY = 4, kCiTrX = 5;
// potrf's panel and trailing update on the same core, for ci_pair_kernel launches of the pipelined schedule
// (h = the pass m, dims interleaved: workgroup b of dim b % L):
//   kCiPanel  tile i = m + 1 + t: L_im = C_i Y_mm^T   A = pass m's C planes (block i, row-major), B = D_m
//             -> the L planes (i, m), scale lsc(i, m) (as ci_panel_kernel)
//   kCiU12c   t < g.inst0: column m + 1's tile I = m + 2 + t, else a trailing tile I >= J >= m + 2:
//             A_IJ - L_Im L_Jm^T (A = g.Kinv, the fp32 matrix), column tiles -> pass m + 1's C planes, scale
//             csc(m + 1, I), trailing ones in place (as ci_update_kernel<kCiU12>, the A tile read after the K loop)
constexpr int kCiPanel = 6, kCiU12c = 7;
#ifndef LVAE_KL_MIRROR
#define LVAE_KL_MIRROR 0  // 1: the KL lauum also writes the upper tiles of K^-1 (no reader needs them)
#endif
struct CiGemmArgs {
  const _Float16 *ah, *al, *bh, *bl;  // full plane arrays
  _Float16 *oh, *ol, *oth, *otl;      // outputs: row-major planes (kCiY), transposed planes (kCiX, kCiY)
  float* Kinv;                         // kCiLauum(KL)
  int np_, nt, h, per_dim, nwg;        // per_dim: workgroups per latent dim
  int inst0;                           // trtri: first recursive-doubling instance; kCiTrX: its X tiles per dim
  // kCiLauumKL (the exact KL's reduce, kl_closed.hip): mu [L, np] fp64 and sqrt v [L, np] in; out the
  // partials of K^-1 mu, apart[l][s][p] = sum over column block s of Kinv(p, .) mu (every (s, p) once),
  // and -- if bh -- the fp16 hi / lo planes of B = K^-1 diag(sqrt v) (row stride np) split with the
  // dim's scale bsc[l] (ci_bscale_kernel)
  const double* mu;
  const float* sv;
  float* apart;
  _Float16 *bh_out, *bl_out;
  float* bsc;
  int pre = 0;  // kCiLauum(KL): K^-1's lower tiles are in Kinv already (pipelined lauum): epilogue only
  const int* hbon = nullptr;  // kCiLauumKL: *hbon != 0 -> the binned hyper-gradient (kl_hyper.hip) runs: the full
                              // symmetric K^-1 (the mirror) instead of the S GEMM's B planes
  const int* dimflag = nullptr;  // kCiLauum: only the dims l with dimflag[l] != 0 (the others' workgroups exit)
};

// one halving butterfly step over lane bit D (D <= 16): the lane keeps the half of its N partial sums
// its bit selects and adds the partner's copy of that half
template <int D, int N>
__device__ inline void ci_bfly(float (&x)[32], int lane) {
  const bool up = (lane & D) != 0;
#pragma unroll
  for (int q = 0; q < N / 2; ++q) {
    const float send = up ? x[q] : x[q + N / 2];
    const float keep = up ? x[q + N / 2] : x[q];
    x[q] = keep + __shfl_xor(send, D, 64);
  }
}

// kCiLauumKL: the partials of K^-1 mu from the tile T = acc * inv = (K^-1)_ij (i >= j): the rows,
// apart[l][j][256 i + r] = sum_c T(r, c) mu_j(c), and for i != j the mirror's rows,
// apart[l][i][256 j + c] = sum_r T(r, c) mu_i(r).  smu = mu_i (0..255), mu_j (256..511); spart 6 x 256
// floats of LDS.  Row sums: each lane's 2 columns, then per pair of 32-row blocks a halving butterfly
// over the 32 lanes of a half-wave (31 shuffles; lane t ends with the t-th of the pair's 32 rows of its
// half-wave), then the 4 column waves in a fixed order in LDS; column sums: each lane's 64 rows, the
// other half-wave, the 2 row waves.  fp32: the KL refines K^-1 mu in fp64 after (kl_closed.hip).
__device__ inline void ci_kl_partials(const sx_f32x16 (&acc)[4][2], float inv, const CiGemmArgs& g, int l, int i,
                                      int j, const float* smu, float* spart) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r32 = lane & 31, kh = lane >> 5;
  const int wm = (w >> 2) * 128, wn = (w & 3) * 64;
  const float m0 = smu[kSwB + wn + r32], m1 = smu[kSwB + wn + 32 + r32];
#pragma unroll
  for (int a2 = 0; a2 < 4; a2 += 2) {
    float x[32];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int e = 0; e < 16; ++e) x[16 * a + e] = acc[a2 + a][0][e] * m0 + acc[a2 + a][1][e] * m1;
    ci_bfly<16, 32>(x, lane);
    ci_bfly<8, 16>(x, lane);
    ci_bfly<4, 8>(x, lane);
    ci_bfly<2, 4>(x, lane);
    ci_bfly<1, 2>(x, lane);
    const int a = a2 + (r32 >> 4), e = r32 & 15;
    spart[(w & 3) * kSwB + wm + 32 * a + (e & 3) + 8 * (e >> 2) + 4 * kh] = x[0];
  }
  if (i != j) {
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      float cs = 0.f;
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int e = 0; e < 16; ++e) cs += acc[a][b][e] * smu[sx_row(a, e)];
      cs += __shfl_xor(cs, 32, 64);
      if (kh == 0) spart[(4 + (w >> 2)) * kSwB + wn + 32 * b + r32] = cs;
    }
  }
  __syncthreads();
  const int np_ = g.np_, nt = g.nt;
  float* ap = g.apart + (int64_t)l * nt * np_;
  if (tid < kSwB) {
    const float s = ((spart[tid] + spart[kSwB + tid]) + spart[2 * kSwB + tid]) + spart[3 * kSwB + tid];
    ap[(int64_t)j * np_ + i * kSwB + tid] = s * inv;
  } else if (i != j) {
    const int c = tid - kSwB;
    ap[(int64_t)i * np_ + j * kSwB + c] = (spart[4 * kSwB + c] + spart[5 * kSwB + c]) * inv;
  }
}

// Y^T (k, k) = D_k^T, 64 x 64 piece (pa, pb) of D_k -> block (pb, pa) of tile (k, k) of the chunk-major Y^T
// planes, through tp (2 x 64 x 66 halves of LDS); any block size.  Ends with the writes (no barrier).
__device__ inline void ci_diag_t_piece(const CiScratch& S, int np_, int l, int k, int pa, int pb,
                                       _Float16* __restrict__ YTh, _Float16* __restrict__ YTl, _Float16* tp) {
  const int t = threadIdx.x, nth = blockDim.x;
  const int64_t od = ((int64_t)l * S.nt + k) * kSwBB + (int64_t)(64 * pa) * kSwB + 64 * pb;
  for (int e = t; e < 64 * 8; e += nth) {
    const int r = e >> 3, c = (e & 7) * 8;
    const x3_half8 h = *reinterpret_cast<const x3_half8*>(S.Dh + od + r * kSwB + c);
    const x3_half8 lo = *reinterpret_cast<const x3_half8*>(S.Dl + od + r * kSwB + c);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      tp[r * 66 + c + q] = h[q];
      tp[64 * 66 + r * 66 + c + q] = lo[q];
    }
  }
  __syncthreads();
  for (int e = t; e < 64 * 8; e += nth) {
    const int c = e >> 3, r0 = (e & 7) * 8;
    x3_half8 h, lo;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      h[q] = tp[(r0 + q) * 66 + c];
      lo[q] = tp[64 * 66 + (r0 + q) * 66 + c];
    }
    const int64_t o = c16_off(l, np_, k * kSwB + 64 * pb + c, k * kSwB + 64 * pa + r0);
    *reinterpret_cast<x3_half8*>(YTh + o) = h;
    *reinterpret_cast<x3_half8*>(YTl + o) = lo;
  }
}

// the body of one workgroup of ci_gemm_kernel<MODE>, as workgroup `bid` of its launch, on the caller's
// LDS objects (ci_pair_kernel runs two modes' bodies in one launch)
template <int MODE>
__device__ inline void ci_gemm_body(const CiGemmArgs& g, const CiScratch& S, const int bid, _Float16* __restrict__ lds,
                                    float* __restrict__ sprod, uint32_t* __restrict__ redp, float* __restrict__ kl_mu,
                                    float* __restrict__ kl_sv, float* __restrict__ kl_part) {
  uint32_t& red = *redp;
  const int nt = g.nt, np_ = g.np_;
  int l, i, j, kb0, kb1;
  if constexpr (MODE == kCiLauum || MODE == kCiLauumKL) {
    // XCD-contiguous remap, 4 x 8 blocks of tiles sharing their Y^T panels in an XCD's L2 (small I,
    // the longest K ranges, first)
    const int orig = bid, xcd = orig % 8, q8 = g.nwg / 8, r8 = g.nwg % 8;
    const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
    l = wgid / g.per_dim;
    if (g.dimflag && !g.dimflag[l]) return;  // (uniform, before any barrier)
    sx_tri_blocked(wgid % g.per_dim, nt, i, j);
    kb0 = i;
    kb1 = nt;
  } else if constexpr (MODE == kCiPanel || MODE == kCiU12c) {
    const int L = g.nwg / g.per_dim, t = bid / L, m = g.h;
    l = bid % L;
    if constexpr (MODE == kCiPanel) {
      i = m + 1 + t;
      j = m;
    } else if (t < g.inst0) {
      i = m + 2 + t;
      j = m + 1;
    } else {
      sx_tri(t - g.inst0, i, j);
      i += m + 2;
      j += m + 2;
    }
    kb0 = m;
    kb1 = m + 1;
  } else if constexpr (MODE == kCiTrY || MODE == kCiTrX) {
    // dims interleaved (block b: dim b % L): the first L (m + 1) workgroups of Xupd are row m + 1's tiles
    const int L = g.nwg / g.per_dim, t = bid / L, m = g.h;
    l = bid % L;
    if constexpr (MODE == kCiTrY) {
      i = m;
      j = t;
      if (t >= m) {  // (uniform) a piece of the diagonal tile
        ci_diag_t_piece(S, np_, l, m, (t - m) >> 2, (t - m) & 3, g.oth, g.otl, lds);
        return;
      }
    } else if (t < g.inst0) {
      i = m + 1 + t / (m + 1);
      j = t % (m + 1);
    } else {
      sx_tri(t - g.inst0, i, j);  // Lupd tile (i, j), j <= i <= m
    }
    kb0 = m;
    kb1 = m + 1;
  } else {
    // longest K first over the whole launch (the tiles of a level span K = 1 .. h blocks): block b
    // takes latent dim b % L (an XCD then keeps the dims b % 8 selects, and their panels) and the
    // t = b / L-th tile of a K-descending order -- X: K = o + h - j, so j_off = j - o ascending; Y:
    // K = i - o - h + 1, so i_off = i - o - h descending; then the instance, then the other index
    const int L = g.nwg / g.per_dim, t = bid / L, h = g.h, ninst = g.per_dim / (h * h);
    l = bid % L;
    const int slow = t / (ninst * h), rem = t % (ninst * h), m = g.inst0 + rem / h, fast = rem % h, o = 2 * h * m;
    if constexpr (MODE == kCiX) {
      j = o + slow;
      i = o + h + fast;
    } else {
      i = o + h + (h - 1 - slow);
      j = o + fast;
    }
    if (i >= nt) return;  // (uniform: before any barrier)
    if constexpr (MODE == kCiX) {
      kb0 = j;
      kb1 = o + h;
    } else {
      kb0 = o + h;
      kb1 = i + 1;
    }
  }
  const int nkb = kb1 - kb0;
  // the scale of block pair kb: sA(kb) sB(kb)
  const int64_t sl = (int64_t)l * nt * nt;
  if (threadIdx.x < nkb) {
    const int kb = kb0 + threadIdx.x;
    float sa, sb;
    if constexpr (MODE == kCiX) {
      sa = S.lsc[sl + (int64_t)i * nt + kb];
      sb = S.ysc[sl + (int64_t)kb * nt + j];
    } else if constexpr (MODE == kCiY) {
      sa = S.ysc[sl + (int64_t)i * nt + kb];
      sb = S.xsc[sl + (int64_t)kb * nt + j];
    } else if constexpr (MODE == kCiPanel) {  // (kb = m)
      sa = S.csc[((int64_t)l * nt + kb) * nt + i];
      sb = S.ysc[sl + (int64_t)kb * nt + kb];
    } else if constexpr (MODE == kCiU12c) {  // (kb = m)
      sa = S.lsc[sl + (int64_t)i * nt + kb];
      sb = S.lsc[sl + (int64_t)j * nt + kb];
    } else if constexpr (MODE == kCiTrY) {  // (kb = m = i)
      sa = S.ysc[sl + (int64_t)i * nt + i];
      sb = S.xsc[sl + (int64_t)i * nt + j];
    } else if constexpr (MODE == kCiTrX) {  // (kb = m)
      sa = (int)(bid / (g.nwg / g.per_dim)) < g.inst0 ? S.lsc[sl + (int64_t)i * nt + kb]
                                                            : S.ysc[sl + (int64_t)kb * nt + i];
      sb = S.ysc[sl + (int64_t)kb * nt + j];
    } else {
      sa = S.ysc[sl + (int64_t)kb * nt + i];
      sb = S.ysc[sl + (int64_t)kb * nt + j];
    }
    sprod[threadIdx.x] = sa * sb;
  }
  if (threadIdx.x == 0) red = 0u;
  const int64_t np2 = (int64_t)np_ * np_;
  const int64_t oa = l * np2 + (int64_t)i * kSwB * np_ + (int64_t)kb0 * kSwB;
  const int64_t ob = l * np2 + (int64_t)j * kSwB * np_ + (int64_t)kb0 * kSwB;
  const _Float16* ah = g.ah + oa;
  const _Float16* al = g.al + oa;
  const _Float16* bh = g.bh + ob;
  const _Float16* bl = g.bl + ob;
  sx_f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = sx_f32x16{};
  if constexpr (MODE == kCiLauumKL) {  // mu and sqrt v of row block i (0..255) and column block j
    const int t = threadIdx.x, blk = t < kSwB ? i : j;
    const int64_t p = (int64_t)l * np_ + (int64_t)blk * kSwB + (t & (kSwB - 1));
    kl_mu[t] = (float)g.mu[p];
    kl_sv[t] = g.sv[p];
  }
  float inv;
  if constexpr (kCiC16) {
    // operands: A = L planes (row-major) for X, else chunk-major panels from block kb0 on; B chunk-major
    const int64_t kc0 = (int64_t)kb0 * (kSwB / kC16BK) * kC16Part;
    C16Opnd A = MODE == kCiX || MODE == kCiTrX ? C16Opnd{ah, g.al - g.ah, np_}
                                               : C16Opnd{g.ah + c16_panel(l, np_, i) + kc0, g.al - g.ah, 0};
    C16Opnd B{g.bh + c16_panel(l, np_, j) + kc0, g.bl - g.bh, 0};
    if constexpr (MODE == kCiTrX) {
      if ((int)(bid / (g.nwg / g.per_dim)) >= g.inst0)  // Lupd: A = Y^T planes (i, m)
        A = C16Opnd{g.bh + c16_panel(l, np_, i) + kc0, g.bl - g.bh, 0};
    }
    if constexpr (MODE == kCiPanel) {  // A = C block i (pass m's planes, row-major 256 x 256), B = D_m
      const int64_t oc = (int64_t)l * np_ * kSwB + (int64_t)i * kSwBB, od = ((int64_t)l * nt + kb0) * kSwBB;
      A = C16Opnd{S.Ch[kb0 & 1] + oc, S.Cl[kb0 & 1] - S.Ch[kb0 & 1], kSwB};
      B = C16Opnd{S.Dh + od, S.Dl - S.Dh, kSwB};
    }
    if constexpr (MODE == kCiU12c) {  // A, B = the L planes (i, m), (j, m), row-major (stride np)
      A = C16Opnd{S.Lh + oa, S.Ll - S.Lh, np_};
      B = C16Opnd{S.Lh + ob, S.Ll - S.Lh, np_};
    }
    if constexpr (MODE == kCiTrY) {  // A = D_m (row-major, stride 256), B = X^T row tile j (one chunk-major tile)
      const int64_t od = ((int64_t)l * nt + i) * kSwBB, ox = ((int64_t)l * nt + j) * kSwBB;
      A = C16Opnd{S.Dh + od, S.Dl - S.Dh, kSwB};
      B = C16Opnd{S.XRh[i & 1] + ox, S.XRl[i & 1] - S.XRh[i & 1], 0};
    }
    if ((MODE == kCiLauum || MODE == kCiLauumKL) && g.pre) {  // (uniform) K^-1 tile from the pipelined lauum
      const float* T = g.Kinv + l * np2 + (int64_t)i * kSwB * np_ + (int64_t)j * kSwB;
      const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(T), (short)0, 0x7fffffff,
                                                                          0x00020000);
      const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
      const int vo = (((w >> 2) * 128 + 4 * (lane >> 5)) * np_ + (w & 3) * 64 + (lane & 31)) * 4;
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int e = 0; e < 16; ++e)
#pragma unroll
          for (int b = 0; b < 2; ++b)
            acc[a][b][e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                rt, vo, ((32 * a + (e & 3) + 8 * (e >> 2)) * np_ + 32 * b) * 4, 0));
      __syncthreads();  // (kl_mu / kl_sv written above)
      inv = 1.f;
    } else {
      // lauum and trtri's X step: the K ranges of a launch's tiles END together (lauum: at the last block for every
      // tile; X: at o + h in an instance), so their chunks run from the end (LVAE_CI_KREV=0: in order)
      constexpr bool krev = LVAE_CI_KREV && (MODE == kCiLauum || MODE == kCiLauumKL || MODE == kCiX);
      const int nk = nkb * (kSwB / kC16BK);
      C16BlockRescale rs{sprod, 1.f, krev ? nk : 0};
      c16_gemm<4>(A, B, nk, lds, acc, rs, krev);
      inv = 1.0f / rs.scur;
    }
  } else {
    inv = 1.0f / sx_gemm_scaled(ah, al, bh, bl, np_, nkb, sprod, lds, acc);
  }
  if constexpr (MODE == kCiPanel) {
    const float slc = x3_scale(sw_block_max(ci_acc_absmax(acc) * inv, &red));
    const int64_t ot = l * np2 + (int64_t)i * kSwB * np_ + (int64_t)j * kSwB;
    ci_planes_out_buf(acc, inv, slc, S.Lh + ot, S.Ll + ot, np_);
    if (threadIdx.x == 0) S.lsc[sl + (int64_t)i * nt + j] = slc;
  } else if constexpr (MODE == kCiU12c) {
    const int m = g.h;
    float* At = g.Kinv + l * np2 + (int64_t)i * kSwB * np_ + (int64_t)j * kSwB;
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(At, (short)0, 0x7fffffff, 0x00020000);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int vo = (((w >> 2) * 128 + 4 * (lane >> 5)) * np_ + (w & 3) * 64 + (lane & 31)) * 4;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int e = 0; e < 16; ++e)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[a][b][e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                             ra, vo, ((32 * a + (e & 3) + 8 * (e >> 2)) * np_ + 32 * b) * 4, 2)) -
                         acc[a][b][e] * inv;
    if (j == m + 1) {  // (uniform) column m + 1: pass m + 1's C operand
      const float sc = x3_scale(sw_block_max(ci_acc_absmax(acc), &red));
      const int64_t on = (int64_t)l * np_ * kSwB + (int64_t)i * kSwBB;
      ci_planes_out_buf(acc, 1.f, sc, S.Ch[(m + 1) & 1] + on, S.Cl[(m + 1) & 1] + on, kSwB);
      if (threadIdx.x == 0) S.csc[((int64_t)l * nt + m + 1) * nt + i] = sc;
    } else {
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int e = 0; e < 16; ++e)
#pragma unroll
          for (int b = 0; b < 2; ++b)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[a][b][e]), ra, vo,
                                                  ((32 * a + (e & 3) + 8 * (e >> 2)) * np_ + 32 * b) * 4, 2);
    }
  } else if constexpr (MODE == kCiTrY) {
    const float sy = x3_scale(sw_block_max(ci_acc_absmax(acc) * inv, &red));
    ci_transposed_out(acc, -inv, lds, [&](int c, int r0, f32x4 v) {
      const int64_t o = c16_off(l, np_, j * kSwB + c, i * kSwB + r0);  // Y^T tile (j, m)
      ci_split4(v, sy, g.oth + o, g.otl + o);
    });
    if (threadIdx.x == 0) S.ysc[sl + (int64_t)i * nt + j] = sy;
  } else if constexpr (MODE == kCiTrX) {
    const int m = g.h;
    const bool lup = (int)(bid / (g.nwg / g.per_dim)) >= g.inst0;
    float* Xt = g.Kinv + l * np2 + (int64_t)i * kSwB * np_ + (int64_t)j * kSwB;  // fp32 X / K^-1 tile (i, j)
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(Xt, (short)0, 0x7fffffff, 0x00020000);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int vo = (((w >> 2) * 128 + 4 * (lane >> 5)) * np_ + (w & 3) * 64 + (lane & 31)) * 4;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) acc[a][b] *= inv;
    if (lup ? i < m : j < m) {  // (uniform) the terms so far: X k = j .. m-1, K^-1 k = i .. m-1
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int e = 0; e < 16; ++e)
#pragma unroll
          for (int b = 0; b < 2; ++b)
            acc[a][b][e] += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                rx, vo, ((32 * a + (e & 3) + 8 * (e >> 2)) * np_ + 32 * b) * 4, 0));
    }
    if (!lup && i == m + 1) {  // X_{m+1, j} complete: the split X^T planes of the next rowY
      const float sx = x3_scale(sw_block_max(ci_acc_absmax(acc), &red));
      const int64_t ox = ((int64_t)l * nt + j) * kSwBB;
      _Float16* xh = S.XRh[(m + 1) & 1] + ox;
      _Float16* xl = S.XRl[(m + 1) & 1] + ox;
      ci_transposed_out(acc, 1.f, lds, [&](int c, int r0, f32x4 v) {
        const int64_t o = c16_off(0, kSwB, c, r0);
        ci_split4(v, sx, xh + o, xl + o);
      });
      if (threadIdx.x == 0) S.xsc[sl + (int64_t)i * nt + j] = sx;
    } else {
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int e = 0; e < 16; ++e)
#pragma unroll
          for (int b = 0; b < 2; ++b)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[a][b][e]), rx, vo,
                                                  ((32 * a + (e & 3) + 8 * (e >> 2)) * np_ + 32 * b) * 4, 0);
    }
  } else if constexpr (MODE == kCiX) {
    const float sx = x3_scale(sw_block_max(ci_acc_absmax(acc) * inv, &red));
    const int64_t ot = l * np2 + (int64_t)j * kSwB * np_ + (int64_t)i * kSwB;  // X^T tile (j, i)
    ci_transposed_out(acc, inv, lds, [&](int c, int r0, f32x4 v) {
      const int64_t o = kCiC16 ? c16_off(l, np_, j * kSwB + c, i * kSwB + r0) : ot + (int64_t)c * np_ + r0;
      ci_split4(v, sx, g.oth + o, g.otl + o);
    });
    if (threadIdx.x == 0) S.xsc[sl + (int64_t)i * nt + j] = sx;
  } else if constexpr (MODE == kCiY) {
    const float sy = x3_scale(sw_block_max(ci_acc_absmax(acc) * inv, &red));
    const int64_t ot = l * np2 + (int64_t)i * kSwB * np_ + (int64_t)j * kSwB;   // Y tile (i, j)
    const int64_t ott = l * np2 + (int64_t)j * kSwB * np_ + (int64_t)i * kSwB;  // Y^T tile (j, i)
    if constexpr (kCiC16) {
      const int64_t oc = c16_off(l, np_, i * kSwB, j * kSwB);
      c16_tile_planes_out(acc, [&](int) { return -inv * sy; }, g.oh + oc, g.ol + oc);
    } else {
      ci_planes_out(acc, -inv, sy, g.oh + ot, g.ol + ot, np_);
    }
    ci_transposed_out(acc, -inv, lds, [&](int c, int r0, f32x4 v) {
      const int64_t o = kCiC16 ? c16_off(l, np_, j * kSwB + c, i * kSwB + r0) : ott + (int64_t)c * np_ + r0;
      ci_split4(v, sy, g.oth + o, g.otl + o);
    });
    if (threadIdx.x == 0) S.ysc[sl + (int64_t)i * nt + j] = sy;
  } else {
    // (kCiLauumKL: the tile is scaled in place once -- the epilogue has no registers for a scaled copy)
    if constexpr (MODE == kCiLauumKL) {
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] *= inv;
    }
    const float osc = MODE == kCiLauumKL ? 1.f : inv;
    float* O = g.Kinv + l * np2 + (int64_t)i * kSwB * np_ + (int64_t)j * kSwB;
    float* Ot = g.Kinv + l * np2 + (int64_t)j * kSwB * np_ + (int64_t)i * kSwB;
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(O, (short)0, 0x7fffffff, 0x00020000);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int vo = (((w >> 2) * 128 + 4 * (lane >> 5)) * np_ + (w & 3) * 64 + (lane & 31)) * 4;
    if (!g.pre) {  // (pipelined lauum: the lower tile is already there)
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int e = 0; e < 16; ++e)
#pragma unroll
          for (int b = 0; b < 2; ++b)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[a][b][e] * osc), ro, vo,
                                                  ((32 * a + (e & 3) + 8 * (e >> 2)) * np_ + 32 * b) * 4, 0);
    }
    if constexpr (MODE == kCiLauumKL) {
      ci_kl_partials(acc, 1.f, g, l, i, j, kl_mu, kl_part);
      const int64_t tb = l * np2 + (int64_t)i * kSwB * np_ + (int64_t)j * kSwB;   // B tile (i, j)
      const int64_t tbt = l * np2 + (int64_t)j * kSwB * np_ + (int64_t)i * kSwB;  // B tile (j, i)
      // (uniform) the binned hyper-gradient's plan is on: the mirror of K^-1, no B planes
      const bool hbm = g.bh_out && g.hbon && *g.hbon;
      _Float16* const bho = hbm ? nullptr : g.bh_out;
      _Float16* const blo = hbm ? nullptr : g.bl_out;
      const float sb = bho ? g.bsc[l] : 0.f;  // the dim's split scale of B (ci_bscale_kernel)
      if (bho && kCiBC16) {
        // B(i, j) = T diag(sqrt v_j), column-scaled, straight from the registers into the chunk-major
        // planes (x3_c16.hpp): tile (i, j) is the 128 KB run of chunks 16 j .. 16 j + 15 of row block i
        const int64_t tc = c16_off(l, np_, i * kSwB, j * kSwB);
        c16_tile_planes_out(acc, [&](int b) { return sb * kl_sv[kSwB + sx_col(b)]; }, bho + tc, blo + tc);
      } else if (bho) {
        // B(i, j) = T diag(sqrt v_j): column-scaled, straight from the registers
        const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc(bho + tb, (short)0, 0x7fffffff, 0x00020000);
        const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(blo + tb, (short)0, 0x7fffffff, 0x00020000);
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        const int vb = (((w >> 2) * 128 + 4 * (lane >> 5)) * np_ + (w & 3) * 64 + (lane & 31)) * 2;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const float mc = sb * kl_sv[kSwB + sx_col(b)];
#pragma unroll
          for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              const float y = acc[a][b][e] * mc;
              const _Float16 yh = (_Float16)y;
              const _Float16 yl = (_Float16)(y - (float)yh);
              const int so = ((32 * a + (e & 3) + 8 * (e >> 2)) * np_ + 32 * b) * 2;
              __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, yh), rh, vb, so, 0);
              __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, yl), rl, vb, so, 0);
            }
        }
      }
      // (no mirror of K^-1 here: the exact KL's readers -- kl_alpha_sym_kernel, the Gram adjoint, the
      // diagonal -- read its lower tiles only; the B planes need both halves)
      if (i != j && (bho || hbm || LVAE_KL_MIRROR))
        ci_transposed_out(acc, 1.f, lds, [&](int c, int r0, f32x4 v) {
          if (hbm || LVAE_KL_MIRROR) *reinterpret_cast<f32x4*>(Ot + (int64_t)c * np_ + r0) = v;
          if (bho) {
            const f32x4 s4 = *reinterpret_cast<const f32x4*>(&kl_sv[r0]);
            // B(j, i) row c, columns r0 .. r0 + 3 (one 4-half run of a chunk either way)
            const int64_t o = kCiBC16 ? c16_off(l, np_, j * kSwB + c, i * kSwB + r0) : tbt + (int64_t)c * np_ + r0;
            ci_split4(v * s4, sb, bho + o, blo + o);
          }
        });
    } else if (i != j) {
      ci_transposed_out(acc, inv, lds, [&](int c, int r0, f32x4 v) {
        *reinterpret_cast<f32x4*>(Ot + (int64_t)c * np_ + r0) = v;
      });
    }
  }
}


#define CI_GEMM_LDS                                                                     \
  __shared__ __attribute__((aligned(16))) _Float16 lds[2 * 4 * kSxPart];                \
  __shared__ float sprod[64];                                                           \
  __shared__ uint32_t red;                                                              \
  __shared__ float kl_mu[2 * kSwB], kl_sv[2 * kSwB], kl_part[6 * kSwB]; /* (kCiLauumKL only) */

template <int MODE>
__global__ __launch_bounds__(512) void ci_gemm_kernel(CiGemmArgs g, CiScratch S) {
  CI_GEMM_LDS
  ci_gemm_body<MODE>(g, S, blockIdx.x, lds, sprod, &red, kl_mu, kl_sv, kl_part);
}

// two modes in ONE launch (the pipelined schedule's passes: fewer, fuller launches on the caller's stream):
// workgroups [0, n1) run M1 over g1, the rest M2 over g2
template <int M1, int M2>
__global__ __launch_bounds__(512) void ci_pair_kernel(CiGemmArgs g1, CiGemmArgs g2, CiScratch S, int n1) {
  CI_GEMM_LDS
  if ((int)blockIdx.x < n1)
    ci_gemm_body<M1>(g1, S, blockIdx.x, lds, sprod, &red, kl_mu, kl_sv, kl_part);
  else
    ci_gemm_body<M2>(g2, S, blockIdx.x - n1, lds, sprod, &red, kl_mu, kl_sv, kl_part);
}

// ------------------------------------------------------------------------------------------
// host sequencing
// ------------------------------------------------------------------------------------------
// potrf lookahead schedules (the side stream has the highest priority):
// (a) few latent dims (L <= kCiFuseMaxL): the pivots run back to back on the side stream, each applying
//     the previous pass's update to its own block (ci_pending_update) and waiting only for U2(m-2), the
//     last writer of its block before that:
//       side:  pivot(0);  [wait ev_u2(m-1) (ev_c = prep0 for m = 0);  pivot(m+1);  record ev_piv(m+1)]...
//       main:  prep0;  record ev_c;  [wait ev_piv(m);  panel(m);  U1(m) (without the pivot block) + U2(m), one launch;
//              record ev_u2(m)]...
// (b) many latent dims (the headline L = 16): the chain runs whole on the side stream beside U2:
//       side:  prep0;  pivot(0);  panel(0);  record ev_prep
//       main:  [wait ev_prep;  U1(k) (with the pivot block);  record ev_c;  U2(k)]...
//       side:  [wait ev_c;  pivot(k+1);  panel(k+1);  record ev_prep]...
// Buffers: U1(k) writes C planes (k+1) & 1, read by panel(k+1) (and pivot(k+2)'s pending update in (a));
// their previous readers (panel(k-1), pivot(k)) precede U1(k) on the caller's stream.  The L planes of
// column k are written once (panel(k)) and read by U1(k), U2(k), and trtri; D by the pivots, the panels
// and the diagonal copies.
// Then, on the caller's stream: the diagonal copy, trtri (2 launches per level); lauum is ci_lauum_f32.  (Launching each
// recursive-doubling instance as soon as potrf had produced its blocks -- 2 small launches per
// instance on the caller's stream between the passes -- measured 15.1 vs 14.2 ms per closed step at
// L = 16: the small launches slowed the passes more than the overlap saved.)
size_t ci_scratch_bytes(int np_, int L) { return CiScratch(nullptr, np_, L).bytes; }
int ci_factor_f32(int np_, int L, float* A, void* scratch, _Float16* YT, float* Kinv, double* logdet,
                  int32_t* info, hipStream_t st, float* lout = nullptr);

// potrf + trtri: Y = L^-1 as the Y^T planes YT (+ the per-tile scales in the scratch); A and Kinv are
// overwritten (Kinv holds the X^T planes)
// (lout: potrf only -- no trtri, no pipelined schedule -- with L written in fp32 into lout's lower tiles)
int ci_factor_f32(int np_, int L, float* A, void* scratch, _Float16* YT, float* Kinv, double* logdet,
                  int32_t* info, hipStream_t st, float* lout) {
  if (np_ <= 0 || np_ % kSwB || np_ / kSwB > 64) return -1;
  if (L <= 0) return -2;
  CiScratch S((char*)scratch, np_, L);
  S.lout = lout;
  const int nt = S.nt;
  const int64_t full = (int64_t)L * np_ * np_;
  _Float16* YTh = YT;
  _Float16* YTl = YT + full;
  _Float16* Yh = reinterpret_cast<_Float16*>(A);  // A is dead after potrf: the Y planes
  _Float16* Yl = Yh + full;
  _Float16* XTh = reinterpret_cast<_Float16*>(Kinv);  // Kinv is written last (lauum): the X^T planes until then
  _Float16* XTl = XTh + full;
  auto ok = [](hipError_t e) { return e == hipSuccess; };
  bool pipe = false;
  {
    ProfScope ps(LVAE_PH_POTRF, st);
    std::lock_guard<std::recursive_mutex> lock(side_mutex());
    SideStream* sd = nullptr;
    LVAE_TRY(side_stream(sd));
    (void)zero_async(logdet, sizeof(double) * L, st);
    (void)zero_async(info, sizeof(int32_t) * L, st);
    (void)zero_async(S.cnt, CiScratch::cnt_bytes(L, nt), st);  // the split pivots' tickets
    if (!ok(hipEventRecord(sd->fork, st)) || !ok(hipStreamWaitEvent(sd->s, sd->fork, 0))) return LVAE_ERR_LAUNCH;
    const bool fuse = L <= kCiFuseMaxL;
    const int pmode = lout ? 0 : ci_pipe_mode(np_, L);  // (implies fuse and the XR planes)
    // the split pivot (kCiPvG workgroups per pending pivot); LVAE_PIVOT_SPLIT=0: one workgroup per dim
    static const bool split_env = !getenv("LVAE_PIVOT_SPLIT") || atoi(getenv("LVAE_PIVOT_SPLIT")) != 0;
    const bool split = split_env;
    // LVAE_CI_PAIR=1: the pipelined passes as two ci_pair_kernel launches each instead of four (measured
    // slower: the fused update launch ends later, and the next-but-one pivot waits for it -- scripts/inv_ab.py,
    // L = 2: 2.51 vs 2.18 ms for the inverse)
    static const bool pair = getenv("LVAE_CI_PAIR") && atoi(getenv("LVAE_CI_PAIR")) != 0;
    // LVAE_CI_LOOKAHEAD=1: each pass's trailing update in two launches, the next pivot's column first (the
    // next pivot waits only for that part).  Measured slower (scripts/inv_ab.py, inverse alone: L = 16
    // 5.70 vs 5.59 ms, L = 8 3.60 vs 3.53, L = 4 2.85 vs 2.87; profiles/r4_lookahead_ab.txt): the second
    // launch's tail and the extra launch outweigh the earlier pivot start.  Off by default.
    static const bool la = getenv("LVAE_CI_LOOKAHEAD") && atoi(getenv("LVAE_CI_LOOKAHEAD")) != 0;
    // LVAE_CI_U128=0: the trailing update as whole 256-tiles fused with column m+1's (ci_update_kernel<kCiU12>)
    // instead of the 128 x 128 sub-tile kernel (ci_update128_kernel)
    const bool u128 = getenv("LVAE_CI_U128") && atoi(getenv("LVAE_CI_U128")) != 0;
    // LVAE_CI_URING=1: the fused update on the 16-deep ring (ci_update_ring_kernel) instead of the double-buffered
    // 32-deep stages (ci_update_kernel).  Both opt-in forms measured slower (r6, profiles/r6_update_ab.txt): the ring
    // 211 vs 166 us per launch, the 128 x 128 sub-tiles 116 us for the trailing tiles but + 50 us for column k+1 as
    // its own launch (9.21 vs 9.14 ms per step), or + a 70 us split pass with the column folded in (9.58-9.63 vs 9.22)
    const bool uring = getenv("LVAE_CI_URING") && atoi(getenv("LVAE_CI_URING")) != 0;
    pipe = pmode > 0;
    if (fuse) {
      ci_pivot_kernel<1><<<L, 1024, 0, sd->s>>>(A, np_, 0, S, logdet, info, 0, L, g_pivot_prof);
      if (!ok(hipEventRecord(sd->piv[0], sd->s))) return LVAE_ERR_LAUNCH;
      if (nt > 1) ci_prep0_kernel<<<dim3(nt - 1, L), 256, 0, st>>>(A, np_, S);
      if (!ok(hipEventRecord(sd->c, st))) return LVAE_ERR_LAUNCH;
      for (int m = 0; m < nt; ++m) {
        if (m + 1 < nt) {
          if (!ok(hipStreamWaitEvent(sd->s, m == 0 ? sd->c : sd->u2p[(m - 1) & 1], 0))) return LVAE_ERR_LAUNCH;
          if (split) {
            const int Lr = (L + 7) / 8 * 8;
            ci_pivot_kernel<kCiPvG><<<kCiPvG * Lr, 1024, 0, sd->s>>>(A, np_, m + 1, S, logdet, info, 1, L, g_pivot_prof);
          } else {
            ci_pivot_kernel<1><<<L, 1024, 0, sd->s>>>(A, np_, m + 1, S, logdet, info, 1, L, g_pivot_prof);
          }
          if (!ok(hipEventRecord(sd->piv[(m + 1) & 1], sd->s))) return LVAE_ERR_LAUNCH;
        }
        if (!ok(hipStreamWaitEvent(st, sd->piv[m & 1], 0))) return LVAE_ERR_LAUNCH;
        if (pipe && pair) {
          // two launches per pass: [panel(m) + rowY(m)] then [U1 + U2(m) + Xupd(m) (+ Lupd(m))] -- the
          // caller's stream keeps up with the pivot chain (four separate launches per pass did not)
          ProfScope pt(LVAE_PH_POTRI, st);
          const int npn = nt - m - 1, ny = m + 16;
          CiGemmArgs gp{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, np_, nt, m,
                        max(npn, 1), npn * L, 0};
          CiGemmArgs gy{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, YTh, YTl, nullptr, np_, nt, m, ny, ny * L, 0};
          ci_pair_kernel<kCiPanel, kCiTrY><<<(npn + ny) * L, 512, 0, st>>>(gp, gy, S, npn * L);
          const int n1 = max(nt - m - 2, 0), n2 = max(nt - m - 2, 0) * max(nt - m - 1, 0) / 2, nu = n1 + n2;
          const int perx = (nt - m - 1) * (m + 1), perl = pmode == 2 ? (m + 1) * (m + 2) / 2 : 0;
          CiGemmArgs gu{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, A, np_, nt, m,
                        max(nu, 1), nu * L, n1};
          CiGemmArgs gx{S.Lh, S.Ll, YTh, YTl, nullptr, nullptr, nullptr, nullptr, Kinv, np_, nt, m, max(perx + perl, 1),
                        (perx + perl) * L, perx};
          if (nu + perx + perl > 0) ci_pair_kernel<kCiU12c, kCiTrX><<<(nu + perx + perl) * L, 512, 0, st>>>(gu, gx, S, nu * L);
          if (m + 1 < nt && !ok(hipEventRecord(sd->u2p[m & 1], st))) return LVAE_ERR_LAUNCH;
          continue;
        }
        if (m + 1 < nt) {
          ci_panel_kernel<<<dim3(nt - m - 1, L), 512, 0, st>>>(S, np_, m);
          // column m+1 without the pivot block + the trailing tiles
          const int n1 = nt - m - 2, n2 = (nt - m - 2) * (nt - m - 1) / 2;
          if (n2 > 0 && la && n2 > 1) {
            // lookahead split: first what pivot(m+2) reads -- column m+1 (the next C planes) and the trailing
            // tile (m+2, m+2) (sx_tri_blocked's tile 0) -- then the rest, which runs beside pivot(m+2)
            ProfScope pu(LVAE_PH_SWEEP_UPD, st);  // (both launches: the pass's whole trailing update)
            ci_update_kernel<kCiU12><<<(n1 + 1) * L, 512, 0, st>>>(A, S, np_, m, 1, L, n1, 0);
            if (!ok(hipEventRecord(sd->u2p[m & 1], st))) return LVAE_ERR_LAUNCH;
            ci_update_kernel<kCiU12><<<(n2 - 1) * L, 512, 0, st>>>(A, S, np_, m, n2 - 1, (n2 - 1) * L, 0, 1);
          } else {
            if (n2 > 0) {
              ProfScope pu(LVAE_PH_SWEEP_UPD, st);
              if (u128) {  // column m+1 and the trailing tiles as 128 x 128 sub-tiles, two workgroups per CU; then
                           // column m+1's fp32 tiles split into pass m+1's C planes (each 256-tile's exact-max scale)
                ci_update128_kernel<<<4 * (n1 + n2) * L, 256, 0, st>>>(A, S, np_, m, n2, 4 * (n1 + n2) * L, n1);
                ci_prep0_kernel<<<dim3(n1, L), 256, 0, st>>>(A, np_, S, m + 1);
              } else if (uring) {
                ci_update_ring_kernel<kCiU12><<<(n1 + n2) * L, 512, 0, st>>>(A, S, np_, m, n2, n2 * L, n1);
              } else {
                ci_update_kernel<kCiU12><<<(n1 + n2) * L, 512, 0, st>>>(A, S, np_, m, n2, n2 * L, n1);
              }
            }
            if (!ok(hipEventRecord(sd->u2p[m & 1], st))) return LVAE_ERR_LAUNCH;
          }
        }
        if (pipe) {  // trtri by block rows beside the chain (after U2(m): off pivot(m+2)'s path)
          ProfScope pt(LVAE_PH_POTRI, st);
          const int pery = m + 16;
          CiGemmArgs gy{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, YTh, YTl, nullptr, np_, nt, m, pery,
                        pery * L, 0};
          ci_gemm_kernel<kCiTrY><<<pery * L, 512, 0, st>>>(gy, S);
          // Xupd(m) (+ Lupd(m) in mode 2), one launch
          const int perx = (nt - m - 1) * (m + 1), perl = pmode == 2 ? (m + 1) * (m + 2) / 2 : 0;
          if (perx + perl > 0) {
            CiGemmArgs gx{S.Lh, S.Ll, YTh, YTl, nullptr, nullptr, nullptr, nullptr, Kinv, np_, nt, m, perx + perl,
                          (perx + perl) * L, perx};
            ci_gemm_kernel<kCiTrX><<<(perx + perl) * L, 512, 0, st>>>(gx, S);
          }
        }
      }
    } else {
      if (nt > 1) ci_prep0_kernel<<<dim3(nt - 1, L), 256, 0, sd->s>>>(A, np_, S);
      ci_pivot_kernel<1><<<L, 1024, 0, sd->s>>>(A, np_, 0, S, logdet, info, 0, L, g_pivot_prof);
      if (nt > 1) ci_panel_kernel<<<dim3(nt - 1, L), 512, 0, sd->s>>>(S, np_, 0);
      if (!ok(hipEventRecord(sd->prep, sd->s))) return LVAE_ERR_LAUNCH;
      for (int k = 0; k + 1 < nt; ++k) {
        if (!ok(hipStreamWaitEvent(st, sd->prep, 0))) return LVAE_ERR_LAUNCH;  // pivot(k), panel(k)
        const int n1 = nt - k - 1;  // column k+1 with the pivot block
        ci_update_kernel<kCiU1><<<n1 * L, 512, 0, st>>>(A, S, np_, k, n1, n1 * L);
        if (!ok(hipEventRecord(sd->c, st))) return LVAE_ERR_LAUNCH;
        if (!ok(hipStreamWaitEvent(sd->s, sd->c, 0))) return LVAE_ERR_LAUNCH;
        ci_pivot_kernel<1><<<L, 1024, 0, sd->s>>>(A, np_, k + 1, S, logdet, info, 0, L, g_pivot_prof);
        if (k + 2 < nt) ci_panel_kernel<<<dim3(nt - k - 2, L), 512, 0, sd->s>>>(S, np_, k + 1);
        if (!ok(hipEventRecord(sd->prep, sd->s))) return LVAE_ERR_LAUNCH;
        const int n2 = (nt - k - 2) * (nt - k - 1) / 2;
        if (n2 > 0) {
          ProfScope pu(LVAE_PH_SWEEP_UPD, st);
          if (u128)
            ci_update128_kernel<<<4 * n2 * L, 256, 0, st>>>(A, S, np_, k, n2, 4 * n2 * L);
          else
            ci_update_kernel<kCiU2><<<n2 * L, 512, 0, st>>>(A, S, np_, k, n2, n2 * L);
        }
      }
      if (!ok(hipStreamWaitEvent(st, sd->prep, 0))) return LVAE_ERR_LAUNCH;  // the last pivot
    }
  }
  LVAE_CHECK_LAUNCH();
  if (lout) return 0;
  if (!pipe) {
    // trtri (recursive doubling, 2 launches per level): with lauum (ci_lauum_f32) the rest of potri
    ProfScope ps(LVAE_PH_POTRI, st);
    ci_diag_copy_kernel<<<dim3(16 * nt, L), 256, 0, st>>>(S, np_, Yh, Yl, YTh, YTl);
    for (int h = 1; h < nt; h *= 2) {
      const int ninst = (nt + 2 * h - 1) / (2 * h), per = ninst * h * h, nwg = per * L;
      CiGemmArgs gx{S.Lh, S.Ll, YTh, YTl, nullptr, nullptr, XTh, XTl, nullptr, np_, nt, h, per, nwg, 0};
      ci_gemm_kernel<kCiX><<<nwg, 512, 0, st>>>(gx, S);
      CiGemmArgs gy{Yh, Yl, XTh, XTl, Yh, Yl, YTh, YTl, nullptr, np_, nt, h, per, nwg, 0};
      ci_gemm_kernel<kCiY><<<nwg, 512, 0, st>>>(gy, S);
    }
  }
  LVAE_CHECK_LAUNCH();
  return 0;
}

// bsc[l] = x3_scale(a bound on max |B|), B = K^-1 diag(sqrt v), known BEFORE lauum so that every tile
// of B is split with one scale per dim (the S GEMM then needs no rescaling between K blocks, which cost
// it 10%): |K^-1_ij| <= max_j K^-1_jj = max_j sum_{i >= j} Y_ij^2 <= max_J sum_{I >= J} 256 m_IJ^2, m_IJ <
// 2^14 / ysc(I, J) the max of Y's tile (x3_scale puts it in [2^13, 2^14) ysc^-1).  The bound may be loose
// by ~256 nt: that only moves the lo plane's subnormal floor, an absolute error <= 2^-38 bound per entry
// (far below the split's 2^-22 relative error).  One workgroup of 64 threads per dim.
__global__ __launch_bounds__(64) void ci_bscale_kernel(CiScratch S, const float* __restrict__ sv, int np_,
                                                       float* __restrict__ bsc) {
  const int l = blockIdx.x, t = threadIdx.x, nt = S.nt;
  const float* ys = S.ysc + (int64_t)l * nt * nt;
  float d = 0.f;  // column blocks J = t, t + 64, ...
  for (int J = t; J < nt; J += 64) {
    float c = 0.f;
    for (int I = J; I < nt; ++I) {
      const float m = 16384.f / ys[I * nt + J];
      c += 256.f * m * m;
    }
    d = fmaxf(d, c);
  }
  float v = 0.f;
  for (int i = t; i < np_; i += 64) v = fmaxf(v, sv[(int64_t)l * np_ + i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    d = fmaxf(d, __shfl_xor(d, o, 64));
    v = fmaxf(v, __shfl_xor(v, o, 64));
  }
  if (t == 0) bsc[l] = x3_scale(d * v);
}

// lauum, K^-1 = Y^T Y from ci_factor_f32's Y^T planes.  With mu (the exact KL's reduce): also the
// partials of K^-1 mu (apart) and, if Bh, the planes of B = K^-1 diag(sqrt v) with their scale bsc[L].
int ci_lauum_f32(int np_, int L, void* scratch, const _Float16* YT, float* Kinv, const double* mu, const float* sv,
                 float* apart, _Float16* Bh, float* bsc, hipStream_t st, const int* hbon) {
  if (np_ <= 0 || np_ % kSwB || np_ / kSwB > 64) return -1;
  CiScratch S((char*)scratch, np_, L);
  const int nt = S.nt, per = nt * (nt + 1) / 2, nwg = per * L;
  const int64_t full = (int64_t)L * np_ * np_;
  ProfScope ps(LVAE_PH_POTRI, st);
  CiGemmArgs gl{YT, YT + full, YT, YT + full, nullptr, nullptr, nullptr, nullptr, Kinv, np_, nt, 0, per, nwg, 0};
  gl.pre = ci_pipe_mode(np_, L) == 2;  // (the factor accumulated K^-1 already: the same decision)
  if (mu) {
    gl.mu = mu;
    gl.sv = sv;
    gl.apart = apart;
    gl.bh_out = Bh;
    gl.bl_out = Bh ? Bh + full : nullptr;
    gl.bsc = bsc;
    gl.hbon = hbon;
    if (Bh) ci_bscale_kernel<<<L, 64, 0, st>>>(S, sv, np_, bsc);
    ci_gemm_kernel<kCiLauumKL><<<nwg, 512, 0, st>>>(gl, S);
  } else {
    ci_gemm_kernel<kCiLauum><<<nwg, 512, 0, st>>>(gl, S);
  }
  LVAE_CHECK_LAUNCH();
  return 0;
}

// lauum for the dims with flag[l] != 0 only (device flags: the exact KL's early reduce refines diag K^-1 in fp64
// for those dims before the full lauum runs in the backward, kl_closed.hip); K^-1 tiles + mirror into Kinv
int ci_lauum_flagged_f32(int np_, int L, void* scratch, const _Float16* YT, float* Kinv, const int* flag, hipStream_t st) {
  if (np_ <= 0 || np_ % kSwB || np_ / kSwB > 64) return -1;
  CiScratch S((char*)scratch, np_, L);
  const int nt = S.nt, per = nt * (nt + 1) / 2, nwg = per * L;
  const int64_t full = (int64_t)L * np_ * np_;
  CiGemmArgs gl{YT, YT + full, YT, YT + full, nullptr, nullptr, nullptr, nullptr, Kinv, np_, nt, 0, per, nwg, 0};
  gl.dimflag = flag;
  ci_gemm_kernel<kCiLauum><<<nwg, 512, 0, st>>>(gl, S);
  LVAE_CHECK_LAUNCH();
  return 0;
}

int ci_pipe_mode_of(int np_, int L) { return ci_pipe_mode(np_, L); }

// the per-tile split scales of Y (ysc(l, i, j), both plane orientations) in the factor's scratch
const float* ci_ysc_ptr(void* scratch, int np_, int L) { return CiScratch((char*)scratch, np_, L).ysc; }

// potrf alone (lvae_potrf_f32): A [L, np, np] -> L in A's lower tiles (fp32; zero strict upper part of the
// diagonal tiles; the other upper tiles untouched), log|A|, info
int ci_potrf_f32(int np_, int L, float* A, void* scratch, double* logdet, int32_t* info, hipStream_t st) {
  return ci_factor_f32(np_, L, A, scratch, nullptr, nullptr, logdet, info, st, A);
}

int ci_inverse_f32(int np_, int L, float* A, void* scratch, _Float16* YT, float* Kinv, double* logdet,
                   int32_t* info, hipStream_t st) {
  LVAE_TRY(ci_factor_f32(np_, L, A, scratch, YT, Kinv, logdet, info, st));
  return ci_lauum_f32(np_, L, scratch, YT, Kinv, nullptr, nullptr, nullptr, nullptr, nullptr, st, nullptr);
}

}  // namespace lvae

extern "C" {
// dev only (not in the C ABI header): the pivots' phase timestamps into buf (nt L 8 u64; nullptr: off)
void lvae_dev_pivot_prof(void* buf) { lvae::g_pivot_prof = (unsigned long long*)buf; }
size_t lvae_spd_inv_chol_scratch_size(int np_, int L) {
  // the C-ABI form also needs the Y^T planes (the KL workspace lends its S-operand planes instead)
  return lvae::ci_scratch_bytes(np_, L) + lvae::align256((size_t)L * np_ * np_ * 2 * sizeof(_Float16));
}
int lvae_spd_inv_chol_f32(int np_, int L, float* A, void* scratch, float* Ainv, double* logdet, int32_t* info,
                          void* stream) {
  if (!A) return -3;
  if (!scratch || ((uintptr_t)scratch & 255)) return -4;
  if (!Ainv) return -5;
  if (!logdet) return -6;
  if (!info) return -7;
  if (np_ <= 0 || np_ % lvae::kSwB) return -1;
  char* yt = (char*)scratch + lvae::ci_scratch_bytes(np_, L);
  return lvae::ci_inverse_f32(np_, L, A, scratch, (_Float16*)yt, Ainv, logdet, info, (hipStream_t)stream);
}
}
