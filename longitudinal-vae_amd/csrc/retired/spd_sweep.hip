// spd_sweep.hip -- K^-1 and log|K| of L batched SPD np x np fp32 covariances by a block symmetric
// sweep (Gauss-Jordan on SPD), the Regime B inverse of the exact KL (replaces torch.cholesky +
// cholesky_solve(I) + the log-det, elbo_functions.py:26-29).
//
// Sweep on pivot block k (256 wide), P = A_kk the current Schur complement of the unswept part:
//   A_kk <- -P^-1,   A_ik <- W_i = A_ik P^-1 (i != k),   A_ij <- A_ij - W_i A_kj (i, j != k)
// After every block is swept, A = -K^-1; log|K| = sum_k log|P_k|.  The same n^3 flops as
// Cholesky + trtri + lauum, but in nt = np / 256 uniform passes: every pass is ONE rank-256 update
// of the whole lower triangle (K = 256: twice the reuse of a 128-wide blocked factorisation's
// updates), so factor, triangular inverse and product collapse into one HBM-streaming kernel per pass.
//
// Per pass k (all L latent dims in every launch):
//   pivot(k)  P = A_kk -> -P^-1 into A_kk and the fp16 planes of P^-1 (blocked Cholesky in LDS on
//             fp32 MFMA, one 1024-thread workgroup per dim), log|P|, info, its split scale
//   prepW(k)  W_i = C_i P^-1 from the planes (one 256 x 256 x3 tile GEMM per block), written IN
//             PLACE into the column's tiles (transposed into tile (k, i) for i < k) and as the
//             planes of -W_i; block k+1 (W_{k+1} = tile (k+1, k)) also as block k of pass k+1's C
//   U1(k)     row / column k+1: A_ij += (-W_i) C_j^T, written straight as the planes of pass k+1's C
//             operand (C_i = A_{i,k+1}; at few latent dims per call without the next pivot block,
//             which pivot(k+1) updates itself: see the schedules below)
//   U2(k)     the interior tiles (I, J not in {k, k+1}), pre-split planes DMA-staged, C streamed
//             non-temporally under the MFMAs; the last pass writes -A to Kinv (both triangles)
//   finish    the last swept column and pivot block to Kinv
// (pass 0's C operand, column 0 of the Gram, is split by prep0).  With lookahead: the next pass's
// chain runs on a side stream beside U2(k) (host sequencing below).
//
// Split scales.  Every GEMM operand is split x sc = hi + lo into fp16 planes with a power of two
// sc = x3_scale(max |x|) per 256 x 256 block, taken from the block's EXACT max by the kernel that
// produces it (U1 / prep0 / prepW for C_i, prepW for W_i, the pivot for P^-1): nothing overflows fp16
// whatever the scale of K (entries of K^-1 grow like 1 / noise) and every block keeps its top entries
// at 2^13..2^14.  A tile product W_I C_J^T accumulates in sW_I sC_J units (exact powers of two).
//
// Scratch (spd_sweep_scratch_bytes): planes Wh Wl Ch Cl 2 x [L, np, 256] fp16 (by pass parity),
// Ph Pl [L, 256, 256] fp16, csc / wsc [L, nt, nt] and psc [L, nt] fp32 scales.  A [L, np, np]: lower
// 256-block tiles read, overwritten.  Kinv [L, np, np]: out, full symmetric.  np % 256 == 0.
#include "prof.hpp"
#include "pv_lds.hpp"
#include "side_stream.hpp"

#include <climits>

namespace lvae {

constexpr int kSwT = 128;  // sub-tile of the finish copies

struct SwScratch {
  _Float16 *Wh[2], *Wl[2], *Ch[2], *Cl[2];  // [L][np][256], by pass parity (pass k+1's chain runs beside U2(k))
  _Float16 *Ph[2], *Pl[2];                   // [L][256][256] planes of P^-1 sP, by pass parity
  _Float16 *Xh, *Xl;                         // [L][256][256] the pivot's own W block (schedule (a))
  float* csc;                   // [L][nt][nt] split scale of block i of the C operand of pass k
  float* wsc;                   // [L][nt][nt] split scale of block i of the W operand of pass k
  float* psc;                   // [L][nt]     split scale of P_k^-1
  int nt;
  size_t bytes;
  SwScratch(char* base, int np_, int L) {
    size_t off = 0;
    auto take = [&](size_t b) {
      char* p = base ? base + off : nullptr;
      off += align256(b);
      return p;
    };
    const size_t col = (size_t)L * np_ * kSwB;
    for (int b = 0; b < 2; ++b) {
      Wh[b] = (_Float16*)take(col * 2);
      Wl[b] = (_Float16*)take(col * 2);
      Ch[b] = (_Float16*)take(col * 2);
      Cl[b] = (_Float16*)take(col * 2);
    }
    for (int b = 0; b < 2; ++b) {
      Ph[b] = (_Float16*)take((size_t)L * kSwBB * 2);
      Pl[b] = (_Float16*)take((size_t)L * kSwBB * 2);
    }
    Xh = (_Float16*)take((size_t)L * kSwBB * 2);
    Xl = (_Float16*)take((size_t)L * kSwBB * 2);
    nt = np_ / kSwB;
    csc = (float*)take((size_t)L * nt * nt * 4);
    wsc = (float*)take((size_t)L * nt * nt * 4);
    psc = (float*)take((size_t)L * nt * 4);
    bytes = off;
  }
  __device__ float& c_scale(int l, int k, int i) const { return csc[((int64_t)l * nt + k) * nt + i]; }
  __device__ float& w_scale(int l, int k, int i) const { return wsc[((int64_t)l * nt + k) * nt + i]; }
};


// ------------------------------------------------------------------------------------------
// pivot: T = A_kk (lower triangle read) -> T = -P^-1 (full), the planes of P^-1, log|P|, info, its split scale.
// One 1024-thread workgroup per dim; the 36 lower 32 x 32 blocks of P live in LDS (pitch 33, 152 KB)
// for the whole kernel and every block operation reads its operands straight from LDS: the Cholesky
// as chains of v_mfma_f32_32x32x2f32 (fp32 products and sums: the accuracy of LAPACK spotrf), the
// L^-1 levels of 128 / 256 rows and L^-T L^-1 as x3-split f16 MFMA products with per-block scales
// (pv_mma3, fp32-equivalent):
//   1. blocked right-looking Cholesky P = L L^T, 8 panels q:
//        diagonal block: one wave factors it in registers and inverts its factor (pv_diag), the
//                        diagonal slot then holds L_qq^-1;
//        panel:          L_iq = A_iq L_qq^-T                        (waves 0 .. 6-q)
//        trailing:       A_ij -= L_iq L_jq^T, q < j <= i             (all waves; wave 0 takes
//                        (q+1, q+1) first and factors it right away: the next diagonal factor
//                        overlaps the rest of the trailing update)
//   2. L^-1 in place by recursive doubling over levels of 64, 128, 256 rows (see the code)
//   3. P^-1 = L^-T L^-1, all 36 lower blocks at once (sum_{k >= i} (L^-1)_ki^T (L^-1)_kj), written
//      back after one barrier, then streamed out (both triangles, coalesced) with its split scale.
// The Cholesky form (rather than an explicit-inverse block sweep) keeps the block updates backward
// stable: a 32-wide explicit-inverse update loses cond(P_qq) digits (measured 20x larger K^-1 error).
// ------------------------------------------------------------------------------------------

#ifdef LVAE_PV_TIMING
__device__ unsigned long long g_pv_t[64];
#define PV_T(i) do { if (blockIdx.x == 0 && threadIdx.x == 0) g_pv_t[i] = wall_clock64(); } while (0)
// U2 probes (pass k == 4): per workgroup {start, first chunk staged, loop end, end, summed chunk waits, smid}
__device__ unsigned long long g_u2_t[4096 * 6];
#define U2_T(j, v) do { if (MODE == kSwU2 && k == 4 && threadIdx.x == 0) g_u2_t[wgid * 6 + (j)] = (v); } while (0)
#else
#define U2_T(j, v) do { } while (0)
#define PV_T(i) do { } while (0)
#endif


// The pivot block's own pending update from pass kp = kb - 1 (schedule (a): the pivot waits neither
// for U1 nor for prepW of the previous pass):
//   X = W_kb = C_kb P_kp^-1   (C_kb: block kb of pass kp's C planes, P_kp^-1: the previous pivot's
//                              planes; x3 GEMM, all 64 blocks, 4 per wave), split at its exact max into
//                              the planes of -X (Xh / Xl, this dim's scratch)
//   lf <- A_kk + (-X) C_kb^T  (the 36 lower blocks, kLauum's wave map)
// red: a __shared__ word zeroed by the caller before an earlier barrier.
__device__ inline void pv_pending_update(const float* __restrict__ T, int64_t np_, const SwScratch& S, int l, int kb,
                                         float* __restrict__ lf, uint32_t* red) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, rl = lane & 31, hh = lane >> 5;
  const int kp = kb - 1;
  const int64_t oc = (int64_t)l * np_ * kSwB + (int64_t)kb * kSwBB, op = (int64_t)l * kSwBB;
  const float sc = S.c_scale(l, kp, kb);
  float sxo;  // X's split scale (the same in every thread)
  // X = C_kb P^-1 (P^-1 symmetric: its rows are the B operand)
  {
    const _Float16* src[4] = {S.Ch[kp & 1] + oc, S.Cl[kp & 1] + oc, S.Ph[kp & 1] + op, S.Pl[kp & 1] + op};
    int bi[4], bj[4];
#pragma unroll
    for (int h = 0; h < 4; ++h) bi[h] = (4 * w + h) >> 3, bj[h] = (4 * w + h) & 7;
    pv_f32x16 x[4];
#pragma unroll
    for (int h = 0; h < 4; ++h) x[h] = pv_f32x16{};
    pv_x3_gemm<4, false>(src, lf, bi, bj, x);
    const float inv = 1.0f / (sc * S.psc[(int64_t)l * S.nt + kp]);
    float m = 0.f;
#pragma unroll
    for (int h = 0; h < 4; ++h)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        x[h][e] *= inv;
        m = fmaxf(m, fabsf(x[h][e]));
      }
    const float sx = x3_scale(sw_block_max(m, red));
    _Float16* xh = S.Xh + op;
    _Float16* xl = S.Xl + op;
#pragma unroll
    for (int h = 0; h < 4; ++h)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int r = 32 * bi[h] + pv_row(e, hh), c = 32 * bj[h] + rl;
        const float y = -x[h][e] * sx;
        const _Float16 yh = (_Float16)y;
        xh[r * kSwB + c] = yh;
        xl[r * kSwB + c] = (_Float16)(y - (float)yh);
      }
    sxo = sx;
    __syncthreads();  // the X planes are visible to the workgroup (workgroup-scope release / acquire)
  }
  const float sx = sxo;
  // lf <- A_kk + (-X) C_kb^T on the lower blocks
  const _Float16* src[4] = {S.Xh + op, S.Xl + op, S.Ch[kp & 1] + oc, S.Cl[kp & 1] + oc};
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
  pv_x3_gemm<3, true>(src, lf, bi, bj, acc);
  const float inv = 1.0f / (sx * sc);
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
    for (int e = 0; e < 16; ++e) lf[n * kPvBlk + pv_row(e, hh) * kPvL + rl] = old[h][e] + acc[h][e] * inv;
  }
}

__global__ __launch_bounds__(1024) void sw_pivot_kernel(float* __restrict__ Aall, int np_, int kb, SwScratch S,
                                                        double* __restrict__ logdet, int32_t* __restrict__ info,
                                                        int pending) {
  __shared__ float lf[kPvBlocks * kPvBlk];
  __shared__ uint32_t pmax_s, xmax_s;
  __shared__ float bsc[kPvBlocks];  // split scales of the L^-1 blocks (LAUUM on the f16 cores)
  __shared__ int bad_s;
  const int l = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6, rl = lane & 31, hh = lane >> 5;
  float* T = Aall + (int64_t)l * np_ * np_ + (int64_t)kb * kSwB * np_ + kb * kSwB;
  if (tid == 0) {
    bad_s = INT_MAX;
    pmax_s = 0u;
    xmax_s = 0u;
  }
  PV_T(0);
  // lower blocks -> LDS (row r = tid >> 5 of a block, 32 consecutive columns per 32 threads); all 36
  // loads in flight before the first LDS write.  With `pending` (kb > 0 in the sweep), the block still
  // lacks pass kb-1's update, which is applied here from that pass's planes (pv_pending_update).
  if (pending) {
    __syncthreads();  // xmax_s
    pv_pending_update(T, np_, S, l, kb, lf, &xmax_s);
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
  double ld = 0.0;  // wave 0: sum of log pivots
  int bad = INT_MAX;
  PV_T(1);

  // 1. Cholesky P = L L^T, panel by panel (pv_panel), then the trailing update A_ij -= L_iq L_jq^T
  for (int q = 0; q < 8; ++q) {
    if (w <= 7 - q) {
      pv_panel(lf, q, w, lane, ld, bad);
    } else {
      __syncthreads();  // pv_panel's barrier
    }
    __syncthreads();
    PV_T(2 + 2 * q);
    const int m = 7 - q, nb = m * (m + 1) / 2;
    for (int t = w; t < nb; t += 16) {  // trailing block t, column-major from the diagonal
      int jj = 0, u = t;
      while (u >= m - jj) {
        u -= m - jj;
        ++jj;
      }
      const int j = q + 1 + jj, i = j + u;
      pv_f32x16 acc;
      float* Bij = pv_blk(lf, i, j);
      pv_load(acc, Bij, rl, hh);
      pv_mma<false, false>(acc, pv_blk(lf, i, q), pv_blk(lf, j, q), rl, hh, -1.f);
      pv_store(acc, Bij, rl, hh);
    }
    __syncthreads();
    PV_T(3 + 2 * q);
  }
  // the diagonal factors -> L_ii^-1 (eight waves in parallel)
  if (w < 8) pv_trinv(pv_blk(lf, w, w), lane);
  __syncthreads();
  PV_T(20);

  // 2. L^-1 in place by recursive doubling (the diagonal slots already hold L_ii^-1): at each level,
  //    for the lower-triangular [A 0; B C] of two inverted halves, B <- -C^-1 B A^-1 (X = B A^-1 to
  //    LDS, then -C^-1 X); levels of 64, 128, 256 rows: a chain of 2 + 4 + 8 block products
  if (w < 4) {  // 64: B = L_{2a+1, 2a}
    const int a = 2 * w;
    pv_f32x16 X = {}, Y = {};
    pv_mma<false, true>(X, pv_blk(lf, a + 1, a), pv_blk(lf, a, a), rl, hh);
    const float* Ci = pv_blk(lf, a + 1, a + 1);
#pragma unroll
    for (int s = 0; s < 16; ++s)  // Y = C^-1 X, X straight from the accumulator (K permuted to its rows)
      Y = __builtin_amdgcn_mfma_f32_32x32x2f32(Ci[rl * kPvL + pv_row(s, hh)], X[s], Y, 0, 0, 0);
    pv_store(Y, pv_blk(lf, a + 1, a), rl, hh, -1.f);
  }
  __syncthreads();
  PV_T(24);
  // levels 128 and 256 on the f16 cores (pv_mma3) with per-block split scales: all blocks' at the
  // level start, the X blocks' from their accumulators as they are stored
#pragma unroll 1
  for (int lv = 1; lv <= 2; ++lv) {
    pv_block_scales(lf, bsc, w, lane, rl, hh);
    const int h = 1 << lv;                 // half width in blocks (2, 4)
    const int per = h * h;                 // blocks of B per instance
    const int inst = w / per, t = w % per;
    const bool act = inst < 4 / h;         // 2 instances of 128, 1 of 256
    const int o = 2 * h * inst;            // first block row / column of the instance
    const int i = o + h + t / h, j = o + t % h;
    const int nij = i * (i + 1) / 2 + j;
    pv_f32x16 acc = {};
    if (act)  // X_ij = sum_{k=j}^{o+h-1} L_ik (A^-1)_kj
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
    if (act)  // Y_ij = sum_{k=o+h}^{i} (C^-1)_ik X_kj
      for (int k = o + h; k <= i; ++k) {
        const int a = i * (i + 1) / 2 + k, b = k * (k + 1) / 2 + j;
        pv_mma3<false, true>(acc, lf + a * kPvBlk, lf + b * kPvBlk, bsc[a], bsc[b], rl, hh);
      }
    __syncthreads();
    if (act) pv_store(acc, pv_blk(lf, i, j), rl, hh, -1.f);
    __syncthreads();
  }
  PV_T(21);

  // 3. P^-1 = L^-T L^-1: block n = i (i + 1) / 2 + j costs 8 - i products; longest-processing-time
  //    assignment, 7-8 products per wave, 30 per SIMD; the products on the f16 cores (pv_mma3) with
  //    per-block split scales of L^-1 (bsc)
  pv_block_scales(lf, bsc, w, lane, rl, hh);
  pv_pack_blocks(lf, bsc);
  pv_f32x16 res[3];
#pragma unroll
  for (int h = 0; h < 3; ++h) {
    const int n = kLauum[w][h];
    if (n >= 0) {
      int i = 0;
      while ((i + 1) * (i + 2) / 2 <= n) ++i;
      const int j = n - i * (i + 1) / 2;
      res[h] = pv_f32x16{};
      for (int k = i; k < 8; ++k) {
        const int bi = k * (k + 1) / 2 + i, bj = k * (k + 1) / 2 + j;
        pv_mma3p<true, true>(res[h], lf + bi * kPvBlk, lf + bj * kPvBlk, bsc[bi], bsc[bj], rl, hh);
      }
    }
  }
  {  // max |P^-1| before the planes are written (their split scale)
    float pm = 0.f;
#pragma unroll
    for (int h = 0; h < 3; ++h)
      if (kLauum[w][h] >= 0)
#pragma unroll
        for (int e = 0; e < 16; ++e) pm = fmaxf(pm, fabsf(res[h][e]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) pm = fmaxf(pm, __shfl_xor(pm, o, 64));
    if (lane == 0) atomicMax(&pmax_s, __float_as_uint(pm));
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 3; ++h) {
    const int n = kLauum[w][h];
    if (n >= 0) pv_store(res[h], lf + n * kPvBlk, rl, hh);
  }
  __syncthreads();
  PV_T(22);

  // 4. out: T = -P^-1 (both triangles) and the planes of P^-1 sP for prepW: thread (r0 = tid >> 6,
  //    c = 4 (tid & 63)) writes rows r0, r0 + 16, ... at columns c .. c+3 -- a wave writes one whole
  //    row (1 KB of float4 + 2 x 512 B of half4 per instruction); the LDS reads are consecutive
  //    (lower part) or pitch-33 strided (mirror)
  const int c = 4 * (tid & 63);
  const float sP = x3_scale(__uint_as_float(pmax_s));
  _Float16* ph = S.Ph[kb & 1] + (int64_t)l * kSwBB;
  _Float16* pl = S.Pl[kb & 1] + (int64_t)l * kSwBB;
  for (int r = tid >> 6; r < kSwB; r += 16) {
    f32x4 v, t;
    x3_half4 h4, l4;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int cq = c + q;
      v[q] = r >= cq ? pv_blk(lf, r >> 5, cq >> 5)[(r & 31) * kPvL + (cq & 31)]
                     : pv_blk(lf, cq >> 5, r >> 5)[(cq & 31) * kPvL + (r & 31)];
      t[q] = -v[q];
      const float y = v[q] * sP;
      const _Float16 yh = (_Float16)y;
      h4[q] = yh;
      l4[q] = (_Float16)(y - (float)yh);
    }
    *reinterpret_cast<f32x4*>(T + (int64_t)r * np_ + c) = t;
    *reinterpret_cast<x3_half4*>(ph + r * kSwB + c) = h4;
    *reinterpret_cast<x3_half4*>(pl + r * kSwB + c) = l4;
  }
  if (w == 0 && lane == 0) bad_s = bad;
  __syncthreads();
  PV_T(23);
  if (tid == 0) {
    S.psc[(int64_t)l * S.nt + kb] = sP;
    logdet[l] += ld;
    if (bad_s != INT_MAX && info[l] == 0) info[l] = kb * kSwB + bad_s + 1;
  }
}

// ------------------------------------------------------------------------------------------
// 128 x 128 block visitor: fn(r, c, f32x4 v) for dst element (r, c..c+3) = src[r][c..] (direct)
// or src[c..][r] (transposed, through a 64 x 129 LDS stage per half).  256 threads; lanes of a
// 16-group cover 64 consecutive dst columns of one dst row (coalesced reads and writes).
// ------------------------------------------------------------------------------------------
template <typename Fn>
__device__ inline void blk128_visit(const float* __restrict__ src, int64_t ld, bool trans, float* __restrict__ lds,
                                    Fn fn, int t = threadIdx.x) {
  const int c4 = t & 15, r0 = t >> 4;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (trans) {
      __syncthreads();
#pragma unroll
      for (int i = 0; i < 8; ++i) {  // src rows 64 h + (t >> 5) + 8 i, float4 at column 4 (t & 31)
        const int sr = (t >> 5) + 8 * i, sc = 4 * (t & 31);
        const f32x4 v = *reinterpret_cast<const f32x4*>(src + (int64_t)(64 * h + sr) * ld + sc);
#pragma unroll
        for (int e = 0; e < 4; ++e) lds[sr * 129 + sc + e] = v[e];
      }
      __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = r0 + 16 * i, c = 64 * h + 4 * c4;
      f32x4 v;
      if (trans) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = lds[(4 * c4 + e) * 129 + r];
      } else {
        v = *reinterpret_cast<const f32x4*>(src + (int64_t)r * ld + c);
      }
      fn(r, c, v);
    }
  }
}

__device__ inline void sw_split4(f32x4 v, float s, _Float16* __restrict__ hi, _Float16* __restrict__ lo) {
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

// ------------------------------------------------------------------------------------------
// the pass-0 C operand: blocks i >= 1 of column 0 (tile (i, 0)), each with its own split scale from its
// exact max.  grid (nt - 1, L), 256 threads: one pass for the max, one for the planes.
__global__ __launch_bounds__(256) void sw_prep0_kernel(const float* __restrict__ Aall, int np_, SwScratch S) {
  __shared__ uint32_t red;
  const int l = blockIdx.y, i = blockIdx.x + 1, t = threadIdx.x;
  const float* T = Aall + (int64_t)l * np_ * np_ + (int64_t)i * kSwB * np_;
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
    sw_split4(v, sc, S.Ch[0] + o + r * kSwB + c, S.Cl[0] + o + r * kSwB + c);
  }
  if (t == 0) S.c_scale(l, 0, i) = sc;
}

// ------------------------------------------------------------------------------------------
// 256 x 256 tile in accumulators (value = acc * mul) out TRANSPOSED through the workgroup's 128 KB LDS
// stage, per 128-row half: fn(c, r0, v) gets v = (value(r0 + q, c))_{q < 4} -- row c of the transpose,
// columns r0 .. r0 + 3 -- every (c, r0) once (coalesced 512-B rows whatever fn stores).  Starts with a
// barrier: the caller's last reads of the LDS stage must precede it.
// ------------------------------------------------------------------------------------------
template <typename Fn>
__device__ inline void sx_transposed_out(const sx_f32x16 (&acc)[4][2], float mul, _Float16* lds, Fn fn) {
  float* U = reinterpret_cast<float*>(lds);
  const int tid = threadIdx.x, w = tid >> 6;
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    __syncthreads();  // hh = 0: the caller's last LDS reads; hh = 1: the half-0 readers
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

// ------------------------------------------------------------------------------------------
// prepW(k): W_i = A_ik P^-1 = (C_i sC_i)(P^-1 sP) / (sC_i sP) for i != k: one 512-thread workgroup per
// 256 x 256 block on the pre-split planes (sx_gemm, K = 256), grid (nt - 1, L).  W_i goes IN PLACE
// into the swept column -- tile (i, k), or transposed (through LDS) into tile (k, i) for i < k: the
// column's readers are done (U1 / U2 read only planes) -- and as the planes of -W_i sW_i, sW_i from
// the block's exact max.  W_{k+1} = tile (k+1, k) is also block k of the NEXT pass's C operand
// (column k+1): its transpose goes to that pass's C planes with the same scale.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(512) void sw_prepw_kernel(float* __restrict__ Aall, SwScratch S, int np_, int k) {
  __shared__ __attribute__((aligned(16))) _Float16 lds[2 * 4 * kSxPart];
  __shared__ uint32_t red;
  const int l = blockIdx.y, i = blockIdx.x < k ? blockIdx.x : blockIdx.x + 1;
  const int64_t np2 = (int64_t)np_ * np_, col = (int64_t)np_ * kSwB;
  const int64_t oc = l * col + (int64_t)i * kSwBB, op = (int64_t)l * kSwBB;
  if (threadIdx.x == 0) red = 0u;
  sx_f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = sx_f32x16{};
  sx_gemm(S.Ch[k & 1] + oc, S.Cl[k & 1] + oc, S.Ph[k & 1] + op, S.Pl[k & 1] + op, kSwB, kSwB, lds, acc);
  const float inv = 1.0f / (S.c_scale(l, k, i) * S.psc[(int64_t)l * S.nt + k]);
  float wm = 0.f;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        acc[a][b][e] *= inv;
        wm = fmaxf(wm, fabsf(acc[a][b][e]));
      }
  const float sw = x3_scale(sw_block_max(wm, &red));
  _Float16* wh = S.Wh[k & 1] + oc;
  _Float16* wl = S.Wl[k & 1] + oc;
  float* A = Aall + l * np2;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int r = sx_row(a, e), c = sx_col(b);
        const float v = acc[a][b][e];
        const float y = -v * sw;
        const _Float16 yh = (_Float16)y;
        wh[r * kSwB + c] = yh;
        wl[r * kSwB + c] = (_Float16)(y - (float)yh);
        if (i > k) A[(int64_t)(i * kSwB + r) * np_ + k * kSwB + c] = v;
      }
  if (threadIdx.x == 0) S.w_scale(l, k, i) = sw;
  if (i < k) {  // tile (k, i) = W_i^T
    float* Ot = A + (int64_t)k * kSwB * np_ + i * kSwB;
    sx_transposed_out(acc, 1.0f, lds, [&](int c, int r0, f32x4 v) {
      *reinterpret_cast<f32x4*>(Ot + (int64_t)c * np_ + r0) = v;
    });
  } else if (i == k + 1) {  // block k of the C operand of pass k+1 = W_{k+1}^T
    const int64_t on = l * col + (int64_t)k * kSwBB;
    _Float16* ch = S.Ch[(k + 1) & 1] + on;
    _Float16* cl = S.Cl[(k + 1) & 1] + on;
    sx_transposed_out(acc, 1.0f, lds, [&](int c, int r0, f32x4 v) {
      sw_split4(v, sw, ch + c * kSwB + r0, cl + c * kSwB + r0);
    });
    if (threadIdx.x == 0) S.c_scale(l, k + 1, k) = sw;
  }
}

// ------------------------------------------------------------------------------------------
// update(k): A_IJ += (-W_I) C_J^T on lower 256-tiles (I >= J, I, J != k), K = 256: one 512-thread
// workgroup per 256 x 256 tile on the pre-split fp16 planes (x3_dma.hpp layout and DMA staging,
// double-buffered K chunks of 32).  C enters in 8 chunks of 16 accumulator elements INSIDE the K
// loop (chunk j loaded in step j, added in step j + 2), read and written non-temporally (CAUX = slc:
// the C stream does not evict the planes from L2).  Measured at np = 4096, L = 16: C streaming alone
// ~200 us, the GEMM alone ~200 us, together 293 us per launch (a 256 x 128 half-tile form with two
// workgroups per CU moved 1.5x the plane bytes and took 350-410 us).  Three tile sets (MODE):
//   kSwU2    the interior: I, J not in {k, k+1} -- on the caller's stream, beside
//   kSwU1    row / column k+1 (without the next pivot block in schedule (a)) -- on the caller's stream, ahead of the next
//            pivot and prep (lookahead: those do not wait for the interior update)
//   kSwLast  every tile of the last pass (I, J != k): -result to Kinv (I, J) and its mirror
// ------------------------------------------------------------------------------------------
constexpr int kSwU2 = 0, kSwU1 = 1, kSwLast = 2;
constexpr int kSwFuseMaxL = 8;  // latent dims per call up to which the pivot updates its own block
template <int MODE, int CAUX = MODE == kSwLast ? 0 : 2>
__global__ __launch_bounds__(512) void sw_update_kernel(float* __restrict__ Aall, SwScratch S,
                                                           float* __restrict__ Kinv, int np_, int k,
                                                           int ntl, int nwg) {
  constexpr bool LAST = MODE == kSwLast;
  __shared__ __attribute__((aligned(16))) _Float16 lds[2 * 4 * kSxPart];
  __shared__ uint32_t red;
  if (MODE == kSwU1 && threadIdx.x == 0) red = 0u;
  const int orig = blockIdx.x, xcd = orig % 8, q8 = nwg / 8, r8 = nwg % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int l = wgid / ntl, t = wgid % ntl, nt = np_ / kSwB;
  int I, J;
  if constexpr (MODE == kSwU1) {
    if (ntl == nt - 1) {  // t < k: (k+1, t); t == k: (k+1, k+1); t > k: (t+1, k+1)
      I = t > k ? t + 1 : k + 1;
      J = t > k ? k + 1 : (t < k ? t : k + 1);
    } else {  // without the pivot block (it updates itself): t < k: (k+1, t); t >= k: (t+2, k+1)
      I = t >= k ? t + 2 : k + 1;
      J = t >= k ? k + 1 : t;
    }
  } else if constexpr (MODE == kSwU2) {
    sx_tri_blocked(t, nt - 2, I, J);
    I += I >= k ? 2 : 0;
    J += J >= k ? 2 : 0;
  } else {
    sx_tri_blocked(t, nt - 1, I, J);
    I += I >= k;
    J += J >= k;
  }
  const int64_t np2 = (int64_t)np_ * np_, col = (int64_t)np_ * kSwB;
  float* C = Aall + l * np2 + (int64_t)I * kSwB * np_ + J * kSwB;
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(C, (short)0, 0x7fffffff, 0x00020000);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int vo = (((w >> 2) * 128 + 4 * (lane >> 5)) * np_ + (w & 3) * 64 + (lane & 31)) * 4;
  const int64_t oa = l * col + (int64_t)I * kSwBB, ob = l * col + (int64_t)J * kSwBB;
  const float cs = S.w_scale(l, k, I) * S.c_scale(l, k, J), inv = 1.0f / cs;  // sW_I sC_J units (powers of 2)
  const _Float16* ah = S.Wh[k & 1] + oa;
  const _Float16* al = S.Wl[k & 1] + oa;
  const _Float16* bh = S.Ch[k & 1] + ob;
  const _Float16* bl = S.Cl[k & 1] + ob;
  sx_f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = sx_f32x16{};
  // chunk j = accumulator elements 16 j .. 16 j + 15 (a = i >> 5, e = (i >> 1) & 15, b = i & 1),
  // loaded in step j AFTER that step's plane DMA and added in step j + 2: the counted wait of step
  // j + 1 (vmcnt(16)) retires DMA j + 1 and leaves C chunk j in flight
  float cv[2][16];
  constexpr int nk = kSwB / kSxBK;
  static_assert(nk * 16 == 128, "one C chunk per K step");
#ifdef LVAE_PV_TIMING
  unsigned long long t_wait = 0, t_w0 = wall_clock64();
  U2_T(0, t_w0);
  U2_T(5, (unsigned long long)__smid());
#endif
  sx_issue(ah, al, bh, bl, kSwB, 0, lds);
#pragma unroll
  for (int s = 0; s < nk; ++s) {
#ifdef LVAE_PV_TIMING
    t_w0 = wall_clock64();
#endif
    if (s == 0) SX_WAIT_VM(0);
    else __builtin_amdgcn_s_waitcnt(0x4F70);  // vmcnt(16): DMA s and C chunk s - 2 landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#ifdef LVAE_PV_TIMING
    if (s == 0) U2_T(1, wall_clock64());
    else t_wait += wall_clock64() - t_w0;
#endif
    if (s + 1 < nk) sx_issue(ah, al, bh, bl, kSwB, (s + 1) * kSxBK, lds + ((s + 1) & 1) * 4 * kSxPart);
    if (s >= 2) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int i = 16 * (s - 2) + q, a = i >> 5, e = (i >> 1) & 15, b = i & 1;
        acc[a][b][e] += cv[s & 1][q] * cs;
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
      acc[a][b][e] += cv[j & 1][q] * cs;
    }
#ifdef LVAE_PV_TIMING
  U2_T(2, wall_clock64());
  U2_T(4, t_wait);
#endif
  if constexpr (MODE == kSwU1) {
    if (I == J) {  // the next pivot block (schedule (b)): stored for the pivot
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int e = 0; e < 16; ++e)
#pragma unroll
          for (int b = 0; b < 2; ++b)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[a][b][e] * inv), rc, vo,
                                                  ((32 * a + (e & 3) + 8 * (e >> 2)) * np_ + 32 * b) * 4, CAUX);
    } else {
      // a tile of column k+1 = one block of the next pass's C operand: straight to its planes with the
      // block's own split scale (its fp32 copy is dead: prepW(k+1) overwrites the column in place)
      float mx = 0.f;
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int e = 0; e < 16; ++e) mx = fmaxf(mx, fabsf(acc[a][b][e] * inv));
      const float sc = x3_scale(sw_block_max(mx, &red));
      const int blk = J == k + 1 ? I : J;
      const int64_t on = l * col + (int64_t)blk * kSwBB;
      _Float16* ch = S.Ch[(k + 1) & 1] + on;
      _Float16* cl = S.Cl[(k + 1) & 1] + on;
      if (J == k + 1) {  // tile (I, k+1): block I as is
        const float m = inv * sc;
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              const int r = sx_row(a, e), c = sx_col(b);
              const float y = acc[a][b][e] * m;
              const _Float16 yh = (_Float16)y;
              ch[r * kSwB + c] = yh;
              cl[r * kSwB + c] = (_Float16)(y - (float)yh);
            }
      } else {  // tile (k+1, J): block J is its transpose
        sx_transposed_out(acc, inv, lds, [&](int c, int r0, f32x4 v) {
          sw_split4(v, sc, ch + c * kSwB + r0, cl + c * kSwB + r0);
        });
      }
      if (threadIdx.x == 0) S.c_scale(l, k + 1, blk) = sc;
    }
  } else if constexpr (!LAST) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int e = 0; e < 16; ++e)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[a][b][e] * inv), rc, vo,
                                                ((32 * a + (e & 3) + 8 * (e >> 2)) * np_ + 32 * b) * 4, CAUX);
#ifdef LVAE_PV_TIMING
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    U2_T(3, wall_clock64());
#endif
  } else {
    // -result to Kinv (I, J) (diagonal tiles: lower elements only) and, transposed through LDS, to
    // (J, I): per 128-row half of the tile, U[c][r ^ 4 (c & 31)] = value (r, c), read back as float4
    // runs of 4 rows of one column -> coalesced 512-B rows of (J, I)
    float* O = Kinv + l * np2 + (int64_t)I * kSwB * np_ + J * kSwB;
    float* Ot = Kinv + l * np2 + (int64_t)J * kSwB * np_ + I * kSwB;
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(O, (short)0, 0x7fffffff, 0x00020000);
    const bool diag = I == J;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int e = 0; e < 16; ++e)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          if (!diag || sx_row(a, e) >= sx_col(b))
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(-acc[a][b][e] * inv), ro, vo,
                                                  ((32 * a + (e & 3) + 8 * (e >> 2)) * np_ + 32 * b) * 4, 0);
    float* U = reinterpret_cast<float*>(lds);  // 128 x 256 fp32 = the 128 KB of the K stages
    const int tid = threadIdx.x;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      __syncthreads();  // (hh = 0: every wave's last LDS reads of the GEMM; hh = 1: the half-0 readers)
      if ((w >> 2) == hh) {
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int e = 0; e < 16; ++e)
#pragma unroll
            for (int b = 0; b < 2; ++b) {
              const int rl = sx_row(a, e) - 128 * hh, c = sx_col(b);
              U[c * 128 + (rl ^ ((c & 31) << 2))] = -acc[a][b][e] * inv;
            }
      }
      __syncthreads();
      const int t4 = tid & 31;
#pragma unroll 4
      for (int cc = 0; cc < kSwB; cc += 16) {
        const int c = cc + (tid >> 5), rl = 4 * t4;
        const f32x4 v = *reinterpret_cast<const f32x4*>(&U[c * 128 + (rl ^ ((c & 31) << 2))]);
        float* dst = Ot + (int64_t)c * np_ + 128 * hh + rl;
        if (!diag) {
          *reinterpret_cast<f32x4*>(dst) = v;
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (128 * hh + rl + q >= c) dst[q] = v[q];
        }
      }
    }
  }
}

// last pass: -(swept column nt-1) and -(last pivot block) to Kinv.  grid.x = 4 (2 (nt-1) + 1):
// block w >> 2 < nt-1: Kinv (i, nt-1) = -W_i; < 2 (nt-1): Kinv (nt-1, i) = -W_i^T; else the pivot.
__global__ __launch_bounds__(256) void sw_finish_kernel(const float* __restrict__ Aall, SwScratch S,
                                                        float* __restrict__ Kinv, int np_, int nt) {
  __shared__ float lds[64 * 129];
  const int l = blockIdx.y, w = blockIdx.x, blk = w >> 2, sm = (w >> 1) & 1, sn = w & 1, c = nt - 1;
  const int64_t np2 = (int64_t)np_ * np_;
  const float* A = Aall + l * np2;
  // the last swept column is in place: tile (c, i) = A_ci = W_i^T (i < c)
  const float* src;
  const int64_t ls = np_;
  int64_t r0, c0;
  bool tr = false;
  if (blk < c) {  // Kinv (i, c) = -tile (c, i)^T
    src = A + (int64_t)(c * kSwB + sn * kSwT) * np_ + blk * kSwB + sm * kSwT;
    tr = true;
    r0 = blk * kSwB + sm * kSwT;
    c0 = c * kSwB + sn * kSwT;
  } else if (blk < 2 * c) {  // Kinv (c, i) = -tile (c, i)
    const int i = blk - c;
    src = A + (int64_t)(c * kSwB + sm * kSwT) * np_ + i * kSwB + sn * kSwT;
    r0 = c * kSwB + sm * kSwT;
    c0 = i * kSwB + sn * kSwT;
  } else {
    src = A + (int64_t)(c * kSwB + sm * kSwT) * np_ + c * kSwB + sn * kSwT;
    r0 = c * kSwB + sm * kSwT;
    c0 = c * kSwB + sn * kSwT;
  }
  float* dst = Kinv + l * np2 + r0 * np_ + c0;
  blk128_visit(src, ls, tr, lds,
               [&](int r, int cc, f32x4 v) { *reinterpret_cast<f32x4*>(dst + (int64_t)r * np_ + cc) = -v; });
}

// ------------------------------------------------------------------------------------------
// host sequencing
// ------------------------------------------------------------------------------------------
// Lookahead schedules.  The side stream has the highest priority, so its workgroups are dispatched
// ahead of U2's as CUs free.
// (a) Few latent dims per GPU (L <= kSwFuseMaxL; latent-dim sharding): a pass is bound by its critical
//     chain, so the side stream runs the pivots BACK TO BACK: pivot(m) applies pass m-1's update to its
//     own block itself, computing the W block it needs from the previous pivot's P planes and the C
//     planes (pv_pending_update), and waits only for U2(m-2), the last writer of its block up to pass
//     m-2; prepW, U1 and U2 of pass m follow on the caller's stream once pivot(m) is done:
//       side:  pivot(0);  [wait ev_u2(m-1) (ev_c = prep0 for m = 0);  pivot(m+1);  record ev_piv(m+1)]...
//       main:  prep0;  record ev_c;  [wait ev_piv(m);  prepW(m);  U1(m) (row / column m+1 without the
//              pivot block: pass m+1's C planes);  U2(m);  record ev_u2(m)]...
//     chain per pass: the pivot alone (r2s: 160 us at L = 2 with its 256 x 256 x 256 W block, against
//     133 us pivot + 33 us prepW + ~20 us of launch gaps in r2s's first form).  Events and P planes
//     alternate by pass parity (pivot(m+1) runs beside pass m's prepW, which reads P planes m).
// (b) Many latent dims (the headline L = 16): a pass is bound by total work; the chain runs whole on the
//     side stream beside U2 (measured 0.3 ms per step faster than (a) at L = 16):
//       main:  wait ev_prep;  U1(k) (row / column k+1 with the pivot block);  record ev_c;  U2(k)
//       side:  wait ev_c;  pivot(k+1);  prepW(k+1);  record ev_prep
// Buffers: U1(k) and prepW(k) write the C planes of pass k+1, prepW(k+1) the W planes of pass k+1 and
// block k+1 of pass k+2's C planes, all in the plane set (k+1) & 1 (block k+1 of set k & 1 for the
// latter, whose last readers, U1(k) and pivot(k+1), precede prepW(k+1)); the readers of set (k+1) & 1
// from pass k-1 (U1 / U2(k-1), prepW(k-1), pivot(k)'s pending update) precede its writers on the main
// or the side stream.  pivot(k+1) writes its own block, its X scratch and the P planes of parity
// (k+1) & 1, whose previous readers (prepW(k-1)) precede U2(k-1).
// The side stream and its events: side_stream.hpp (one per device, every enqueue sequence under
// side_mutex(), so host threads cannot interleave their records / waits).  (Disjoint CU masks for the
// two streams were measured 2.6 ms per step slower: every masked queue slowed the rest.)
size_t spd_sweep_scratch_bytes(int np_, int L) { return SwScratch(nullptr, np_, L).bytes; }

int spd_sweep_f32(int np_, int L, float* A, void* scratch, float* Kinv, double* logdet, int32_t* info,
                  hipStream_t st) {
  if (np_ <= 0 || np_ % kSwB) return -1;
  if (L <= 0) return -2;
  std::lock_guard<std::recursive_mutex> lock(side_mutex());
  SideStream* sd = nullptr;
  LVAE_TRY(side_stream(sd));
  SwScratch S((char*)scratch, np_, L);
  const int nt = np_ / kSwB;
  const int ntl2 = (nt - 2) * (nt - 1) / 2, ntll = (nt - 1) * nt / 2;
  auto ok = [](hipError_t e) { return e == hipSuccess; };
  (void)zero_async(logdet, sizeof(double) * L, st);
  (void)zero_async(info, sizeof(int32_t) * L, st);
  if (!ok(hipEventRecord(sd->fork, st)) || !ok(hipStreamWaitEvent(sd->s, sd->fork, 0))) return LVAE_ERR_LAUNCH;
  sw_pivot_kernel<<<L, 1024, 0, sd->s>>>(A, np_, 0, S, logdet, info, 0);
  const bool fuse = L <= kSwFuseMaxL;
  if (fuse) {
    if (!ok(hipEventRecord(sd->piv[0], sd->s))) return LVAE_ERR_LAUNCH;
    if (nt > 1) sw_prep0_kernel<<<dim3(nt - 1, L), 256, 0, st>>>(A, np_, S);  // beside pivot(0)
    if (!ok(hipEventRecord(sd->c, st))) return LVAE_ERR_LAUNCH;
    // schedule (a): the side stream runs the pivots back to back; the caller's stream runs each pass's
    // prepW, U1, U2 once its pivot is done
    for (int m = 0; m < nt; ++m) {
      if (m + 1 < nt) {  // pivot(m+1): block m+1 current up to pass m-1 (U2(m-1); prep0 for m = 0)
        if (!ok(hipStreamWaitEvent(sd->s, m == 0 ? sd->c : sd->u2p[(m - 1) & 1], 0))) return LVAE_ERR_LAUNCH;
        sw_pivot_kernel<<<L, 1024, 0, sd->s>>>(A, np_, m + 1, S, logdet, info, 1);
        if (!ok(hipEventRecord(sd->piv[(m + 1) & 1], sd->s))) return LVAE_ERR_LAUNCH;
      }
      if (!ok(hipStreamWaitEvent(st, sd->piv[m & 1], 0))) return LVAE_ERR_LAUNCH;  // pivot(m)
      if (nt > 1) sw_prepw_kernel<<<dim3(nt - 1, L), 512, 0, st>>>(A, S, np_, m);
      if (m + 1 < nt) {
        if (nt - 2 > 0) sw_update_kernel<kSwU1><<<(nt - 2) * L, 512, 0, st>>>(A, S, Kinv, np_, m, nt - 2, (nt - 2) * L);
        if (ntl2 > 0) {
          ProfScope ps(LVAE_PH_SWEEP_UPD, st);
          sw_update_kernel<kSwU2><<<ntl2 * L, 512, 0, st>>>(A, S, Kinv, np_, m, ntl2, ntl2 * L);
        }
        if (!ok(hipEventRecord(sd->u2p[m & 1], st))) return LVAE_ERR_LAUNCH;
      }
    }
  } else {
    if (nt > 1) {
      sw_prep0_kernel<<<dim3(nt - 1, L), 256, 0, sd->s>>>(A, np_, S);
      sw_prepw_kernel<<<dim3(nt - 1, L), 512, 0, sd->s>>>(A, S, np_, 0);
    }
    if (!ok(hipEventRecord(sd->prep, sd->s))) return LVAE_ERR_LAUNCH;
    for (int k = 0; k + 1 < nt; ++k) {
      if (!ok(hipStreamWaitEvent(st, sd->prep, 0))) return LVAE_ERR_LAUNCH;  // prepW(k)
      sw_update_kernel<kSwU1><<<(nt - 1) * L, 512, 0, st>>>(A, S, Kinv, np_, k, nt - 1, (nt - 1) * L);
      if (!ok(hipEventRecord(sd->c, st))) return LVAE_ERR_LAUNCH;  // U1(k): the C planes of pass k+1
      if (!ok(hipStreamWaitEvent(sd->s, sd->c, 0))) return LVAE_ERR_LAUNCH;
      sw_pivot_kernel<<<L, 1024, 0, sd->s>>>(A, np_, k + 1, S, logdet, info, 0);
      sw_prepw_kernel<<<dim3(nt - 1, L), 512, 0, sd->s>>>(A, S, np_, k + 1);
      if (!ok(hipEventRecord(sd->prep, sd->s))) return LVAE_ERR_LAUNCH;
      if (ntl2 > 0) {
        ProfScope ps(LVAE_PH_SWEEP_UPD, st);
        sw_update_kernel<kSwU2><<<ntl2 * L, 512, 0, st>>>(A, S, Kinv, np_, k, ntl2, ntl2 * L);
      }
    }
  }
  if (!fuse && !ok(hipStreamWaitEvent(st, sd->prep, 0))) return LVAE_ERR_LAUNCH;  // the whole side chain
  if (ntll > 0) sw_update_kernel<kSwLast><<<ntll * L, 512, 0, st>>>(A, S, Kinv, np_, nt - 1, ntll, ntll * L);
  sw_finish_kernel<<<dim3(4 * (2 * (nt - 1) + 1), L), 256, 0, st>>>(A, S, Kinv, np_, nt);
  LVAE_CHECK_LAUNCH();
  return 0;
}

}  // namespace lvae

extern "C" {
#ifdef LVAE_PV_TIMING
int lvae_pv_timing(float* A, int np_, int L, void* scratch, double* logdet, int32_t* info, unsigned long long* out) {
  lvae::SwScratch S((char*)scratch, np_, L);
  lvae::sw_pivot_kernel<<<L, 1024>>>(A, np_, 0, S, logdet, info, 0);
  (void)hipDeviceSynchronize();
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(lvae::g_pv_t), sizeof(unsigned long long) * 64);
}
int lvae_u2_timing(int np_, int L, float* A, void* scratch, float* Kinv, double* logdet, int32_t* info,
                   unsigned long long* out) {
  const int rc = lvae::spd_sweep_f32(np_, L, A, scratch, Kinv, logdet, info, nullptr);
  (void)hipDeviceSynchronize();
  return rc ? rc : (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(lvae::g_u2_t), sizeof(unsigned long long) * 4096 * 6);
}
#endif
size_t lvae_spd_sweep_scratch_size(int np_, int L) { return lvae::spd_sweep_scratch_bytes(np_, L); }
int lvae_spd_sweep_f32(int np_, int L, float* A, void* scratch, float* Kinv, double* logdet, int32_t* info,
                       void* stream) {
  if (!A) return -3;
  if (!scratch || ((uintptr_t)scratch & 255)) return -4;
  if (!Kinv) return -5;
  if (!logdet) return -6;
  if (!info) return -7;
  return lvae::spd_sweep_f32(np_, L, A, scratch, Kinv, logdet, info, (hipStream_t)stream);
}
}
