// pv_lds.hpp -- device helpers of the 256 x 256 pivot-block kernels (one 1024-thread workgroup per
// latent dim, the 36 lower 32 x 32 blocks of the block in LDS): shared by the block sweep
// (spd_sweep.hip) and the blocked Cholesky inverse (chol_inv.hip).  Blocked Cholesky panels as rank-1
// steps inside v_mfma_f32_32x32x2f32 accumulators, the triangular inverse of a 32 x 32 factor, x3
// f16-split block products straight from LDS, and an x3 tile GEMM from global fp16 planes staged
// through the pivot's LDS.
#pragma once
#include "mfma_x3.hpp"
#include "x3_dma.hpp"

#include <climits>

namespace lvae {

constexpr int kSwB = 256;  // pivot block
constexpr int kSwBB = kSwB * kSwB;

// max over a 512- or 1024-thread workgroup of the threads' v >= 0 (red: a __shared__ word zeroed by
// the caller before an earlier barrier); every thread gets the result
__device__ inline float sw_block_max(float v, uint32_t* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(red, __float_as_uint(v));
  __syncthreads();
  return __uint_as_float(*red);
}
constexpr int kPvL = 33;                 // LDS pitch (floats) of a 32 x 32 block
constexpr int kPvBlk = 32 * kPvL;        // floats per block
constexpr int kPvBlocks = 36;            // lower blocks of 8 x 8
__device__ inline float* pv_blk(float* lf, int R, int C) { return lf + (R * (R + 1) / 2 + C) * kPvBlk; }

typedef float pv_f32x16 __attribute__((ext_vector_type(16)));
__device__ inline float pv_rl(float v, int lane) {  // v of lane `lane` (uniform lane index)
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// accumulator element e of a 32x32x2 MFMA block in lane (rl, hh): row (e&3) + 8 (e>>2) + 4 hh, col rl
__device__ inline int pv_row(int e, int hh) { return (e & 3) + 8 * (e >> 2) + 4 * hh; }

__device__ inline void pv_load(pv_f32x16& acc, const float* B, int rl, int hh) {
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = B[pv_row(e, hh) * kPvL + rl];
}
__device__ inline void pv_store(const pv_f32x16& acc, float* B, int rl, int hh, float sgn = 1.f) {
#pragma unroll
  for (int e = 0; e < 16; ++e) B[pv_row(e, hh) * kPvL + rl] = sgn * acc[e];
}
// acc += op(X) op(Y)^T with X, Y 32 x 32 LDS blocks: TX / TY select the transposed operand
//   A[r][k] = TX ? X[k][r] : X[r][k],   B[k][c] = TY ? Y[k][c] : Y[c][k]   (c, r = rl)
// Two interleaved accumulation chains (even / odd k-steps) so consecutive MFMAs do not wait on
// each other's results.
template <bool TX, bool TY>
__device__ inline void pv_mma(pv_f32x16& acc, const float* X, const float* Y, int rl, int hh, float sx = 1.f) {
  pv_f32x16 t = {};
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const int k = 2 * s + hh;
    const float a = TX ? X[k * kPvL + rl] : X[rl * kPvL + k];
    const float b = TY ? Y[k * kPvL + rl] : Y[rl * kPvL + k];
    if (s & 1)
      t = __builtin_amdgcn_mfma_f32_32x32x2f32(sx * a, b, t, 0, 0, 0);
    else
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(sx * a, b, acc, 0, 0, 0);
  }
  acc += t;
}

// acc += op(X) op(Y)^T as pv_mma, on the f16 matrix cores with the 3-product split: each operand is
// scaled by its block's power of two (sX, sY: x3_scale of the block's max |x|), split x s = hi + lo on
// the way from LDS, and the 32 x 32 x 32 product is 2 k-blocks x 3 v_mfma_f32_32x32x16_f16 (vs 16
// v_mfma_f32_32x32x2f32: ~5x the MFMA rate) accumulated in a temporary and unscaled into acc.
// The f16 32x32x16 accumulator layout is that of the 32x32x2 f32 MFMA (pv_row).
template <bool TX, bool TY>
__device__ inline void pv_mma3(pv_f32x16& acc, const float* X, const float* Y, float sX, float sY, int rl, int hh,
                               float sgn = 1.f) {
  pv_f32x16 t = {};
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    x3_half8 aH, aL, bH, bL;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 16 * s + 8 * hh + j;
      const float a = (TX ? X[k * kPvL + rl] : X[rl * kPvL + k]) * sX;
      const float b = (TY ? Y[k * kPvL + rl] : Y[rl * kPvL + k]) * sY;
      const _Float16 ah = (_Float16)a, bh = (_Float16)b;
      aH[j] = ah;
      aL[j] = (_Float16)(a - (float)ah);
      bH[j] = bh;
      bL[j] = (_Float16)(b - (float)bh);
    }
    t = __builtin_amdgcn_mfma_f32_32x32x16_f16(aL, bH, t, 0, 0, 0);
    t = __builtin_amdgcn_mfma_f32_32x32x16_f16(aH, bL, t, 0, 0, 0);
    t = __builtin_amdgcn_mfma_f32_32x32x16_f16(aH, bH, t, 0, 0, 0);
  }
  acc += t * (sgn / (sX * sY));
}

// As pv_mma3 on blocks already split IN PLACE (pv_pack_blocks: each fp32 word replaced by the packed
// fp16 pair (hi | lo << 16) of x s): a fragment is 8 LDS words regrouped by v_perm_b32 into its hi and
// lo halves (1 VALU per element instead of 5).
typedef unsigned int pv_u32x4 __attribute__((ext_vector_type(4)));
template <bool TX, bool TY>
__device__ inline void pv_mma3p(pv_f32x16& acc, const float* X, const float* Y, float sX, float sY, int rl, int hh) {
  pv_f32x16 t = {};
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    unsigned wa[8], wb[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 16 * s + 8 * hh + j;
      wa[j] = __float_as_uint(TX ? X[k * kPvL + rl] : X[rl * kPvL + k]);
      wb[j] = __float_as_uint(TY ? Y[k * kPvL + rl] : Y[rl * kPvL + k]);
    }
    pv_u32x4 ah, al, bh, bl;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      ah[q] = __builtin_amdgcn_perm(wa[2 * q + 1], wa[2 * q], 0x05040100u);
      al[q] = __builtin_amdgcn_perm(wa[2 * q + 1], wa[2 * q], 0x07060302u);
      bh[q] = __builtin_amdgcn_perm(wb[2 * q + 1], wb[2 * q], 0x05040100u);
      bl[q] = __builtin_amdgcn_perm(wb[2 * q + 1], wb[2 * q], 0x07060302u);
    }
    const x3_half8 aH = __builtin_bit_cast(x3_half8, ah), aL = __builtin_bit_cast(x3_half8, al);
    const x3_half8 bH = __builtin_bit_cast(x3_half8, bh), bL = __builtin_bit_cast(x3_half8, bl);
    t = __builtin_amdgcn_mfma_f32_32x32x16_f16(aL, bH, t, 0, 0, 0);
    t = __builtin_amdgcn_mfma_f32_32x32x16_f16(aH, bL, t, 0, 0, 0);
    t = __builtin_amdgcn_mfma_f32_32x32x16_f16(aH, bH, t, 0, 0, 0);
  }
  acc += t * (1.0f / (sX * sY));
}

// every element of the 36 LDS blocks x -> the packed fp16 pair (hi | lo << 16) of x bsc[block], then a
// barrier (the blocks are read only through pv_mma3p afterwards, until overwritten)
__device__ inline void pv_pack_blocks(float* lf, const float* bsc) {
  for (int e = threadIdx.x; e < kPvBlocks * 1024; e += 1024) {
    const int n = e >> 10, r = (e >> 5) & 31, c = e & 31;
    float* p = lf + n * kPvBlk + r * kPvL + c;
    const float y = *p * bsc[n];
    const _Float16 h = (_Float16)y, lo = (_Float16)(y - (float)h);
    *p = __uint_as_float((unsigned)__builtin_bit_cast(unsigned short, h) |
                         ((unsigned)__builtin_bit_cast(unsigned short, lo) << 16));
  }
  __syncthreads();
}

// bsc[n] = x3_scale(max |block n|) for the 36 lower blocks in LDS (wave w: blocks w, w + 16, w + 32),
// then a barrier
__device__ inline void pv_block_scales(const float* lf, float* bsc, int w, int lane, int rl, int hh) {
#pragma unroll
  for (int h = 0; h < 3; ++h) {
    const int n = w + 16 * h;
    if (n < kPvBlocks) {
      float m = 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e) m = fmaxf(m, fabsf(lf[n * kPvBlk + pv_row(e, hh) * kPvL + rl]));
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
      if (lane == 0) bsc[n] = x3_scale(m);
    }
  }
  __syncthreads();
}

// Rank-1 elimination steps inside MFMA accumulators.  A 32 x 32 block held as one accumulator
// (lane (c, hh), element e: row (e&3) + 8 (e>>2) + 4 hh, column c) keeps row p in element e(p) of the
// lanes of half h(p).  An outer product u v^T is then ONE v_mfma_f32_32x32x2f32 whose k-slot h(p)
// carries u (A operand, lanes of half h(p)) and v (B operand, same lanes) and whose other k-slot is
// zero: no value crosses lanes, only the pivot itself (one readlane).
__device__ inline int pv_hh(int r) { return (r >> 2) & 1; }            // half holding row r
__device__ inline int pv_e(int r) { return (r & 3) | ((r >> 3) << 2); }  // its element

// The Cholesky panel q, by waves 0 .. 7-q (wave w: row block i = q + w):
//   every wave factors the diagonal block X = A_qq in its own accumulator, X -= u u^T / d_p (u = row
//   p of X: the Schur complement step; L_qq[:, p] = u / sqrt d_p), and wave w > 0 applies the same
//   steps to Bt = A_iq^T (Bt -= u b^T / d_p, b = row p of Bt = A'_iq[:, p]; L_iq[:, p] = b / sqrt d_p)
// so the panel needs no L_qq^-1 and the whole panel is 32 steps deep.  Wave 0 writes L_qq (zero
// upper part), waves > 0 their L_iq, into LDS; wave 0 also returns sum log d_p and the first
// non-positive pivot.
__device__ inline void pv_panel(float* lf, int q, int w, int lane, double& ld, int& bad) {
  const int rl = lane & 31, hh = lane >> 5, i = q + w;
  float* Dq = pv_blk(lf, q, q);
  float* Bi = pv_blk(lf, i, q);
  pv_f32x16 X, Bt;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int r = pv_row(e, hh);
    X[e] = r >= rl ? Dq[r * kPvL + rl] : Dq[rl * kPvL + r];
    Bt[e] = (w > 0) ? Bi[rl * kPvL + r] : 0.0f;
  }
  float dp = 0.f;  // lane p: pivot d_p
  __syncthreads();  // every panel wave has its copy of A_qq before wave 0 overwrites it with L_qq
#pragma unroll
  for (int p = 0; p < 32; ++p) {
    const int ep = pv_e(p), hp = pv_hh(p);
    const float d = pv_rl(X[ep], p + 32 * hp);
    const float id = __builtin_amdgcn_rcpf(d), is = __builtin_amdgcn_rsqf(d);
    const bool mine = (hh == hp);
    const float u = (mine && rl >= p) ? X[ep] : 0.0f;
    if (w > 0) {
      const float bp = mine ? Bt[ep] : 0.0f;
      if (mine) Bi[rl * kPvL + p] = bp * is;
      Bt = __builtin_amdgcn_mfma_f32_32x32x2f32(-u, bp * id, Bt, 0, 0, 0);
    } else {
      if (mine) Dq[rl * kPvL + p] = u * is;
      if (lane == p) dp = d;
    }
    X = __builtin_amdgcn_mfma_f32_32x32x2f32(-u, u * id, X, 0, 0, 0);
  }
  if (w == 0) {
    const double lv = (lane < 32) ? log((double)dp) : 0.0;
    ld += wave_sum(lv);
    const unsigned long long nb = __ballot(lane < 32 && !(dp > 0.0f && isfinite(dp)));
    if (nb) bad = min(bad, 32 * q + (int)__builtin_ctzll(nb));
  }
}

// the value v of lane (rl, h) in every lane (rl, .): v_permlane32_swap of v with itself gives the lower
// half's values in both halves (first result) and the upper half's (second)
__device__ inline float pv_from_half(float v, int h) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(h ? r[1] : r[0]);
}

// pv_panel with TWO elimination steps per MFMA: rows p and p+1 (p even) sit in the same half of the
// accumulator lanes, so step p+1's vectors follow from step p's by one FMA per lane
//   u1 = X[p+1, :] - X[p, p+1] u0 / d_p,   d_{p+1} = X[p+1, p+1] - X[p, p+1]^2 / d_p   (b1 likewise)
// and the MFMA carries step p in k-slot h(p) and step p+1 in the other one (its operands moved across
// by v_permlane32_swap): 16 MFMAs per panel and block instead of 32 on the dependent chain.
__device__ inline void pv_panel2(float* lf, int q, int w, int lane, double& ld, int& bad) {
  const int rl = lane & 31, hh = lane >> 5, i = q + w;
  float* Dq = pv_blk(lf, q, q);
  float* Bi = pv_blk(lf, i, q);
  pv_f32x16 X, Bt;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int r = pv_row(e, hh);
    X[e] = r >= rl ? Dq[r * kPvL + rl] : Dq[rl * kPvL + r];
    Bt[e] = (w > 0) ? Bi[rl * kPvL + r] : 0.0f;
  }
  float dp = 0.f;  // lane p: pivot d_p
  __syncthreads();  // every panel wave has its copy of A_qq before wave 0 overwrites it with L_qq
#pragma unroll
  for (int p = 0; p < 32; p += 2) {
    const int e0 = pv_e(p), e1 = e0 + 1, hp = pv_hh(p);  // row p + 1: element e0 + 1, same half
    const int lp = p + 32 * hp;
    const float d0 = pv_rl(X[e0], lp), x01 = pv_rl(X[e0], lp + 1), x11 = pv_rl(X[e1], lp + 1);
    const float id0 = __builtin_amdgcn_rcpf(d0), is0 = __builtin_amdgcn_rsqf(d0);
    const float c01 = x01 * id0;
    const float d1 = x11 - x01 * c01;
    const float id1 = __builtin_amdgcn_rcpf(d1), is1 = __builtin_amdgcn_rsqf(d1);
    const bool mine = (hh == hp);
    const float u0 = (mine && rl >= p) ? X[e0] : 0.0f;
    const float u1 = (mine && rl > p) ? X[e1] - c01 * u0 : 0.0f;
    const float u1s = pv_from_half(u1, hp);
    const float a = mine ? u0 : u1s;
    if (w > 0) {
      const float b0 = mine ? Bt[e0] : 0.0f;
      const float b1 = mine ? Bt[e1] - c01 * b0 : 0.0f;
      if (mine) {
        Bi[rl * kPvL + p] = b0 * is0;
        Bi[rl * kPvL + p + 1] = b1 * is1;
      }
      const float b1s = pv_from_half(b1, hp);
      Bt = __builtin_amdgcn_mfma_f32_32x32x2f32(-a, mine ? b0 * id0 : b1s * id1, Bt, 0, 0, 0);
    } else {
      if (mine) {
        Dq[rl * kPvL + p] = u0 * is0;
        Dq[rl * kPvL + p + 1] = u1 * is1;
      }
      if (lane == p) dp = d0;
      if (lane == p + 1) dp = d1;
    }
    X = __builtin_amdgcn_mfma_f32_32x32x2f32(-a, mine ? u0 * id0 : u1s * id1, X, 0, 0, 0);
  }
  if (w == 0) {
    const double lv = (lane < 32) ? log((double)dp) : 0.0;
    ld += wave_sum(lv);
    const unsigned long long nb = __ballot(lane < 32 && !(dp > 0.0f && isfinite(dp)));
    if (nb) bad = min(bad, 32 * q + (int)__builtin_ctzll(nb));
  }
}

// one wave: the lower-triangular factor L in block D -> L^-1 (forward substitution as rank-1 steps:
// Y = I; Y -= a b^T with a = column p of L (a_p = L_pp - 1), b = row p of Y / L_pp: the pivot row
// is rescaled in the same update)
__device__ inline void pv_trinv(float* D, int lane) {
  const int rl = lane & 31, hh = lane >> 5;
  pv_f32x16 y;
#pragma unroll
  for (int e = 0; e < 16; ++e) y[e] = (pv_row(e, hh) == rl) ? 1.0f : 0.0f;
  const float lrr = D[rl * kPvL + rl];
  const float ilr = 1.0f / lrr;  // lane rl: 1 / L_rr
#pragma unroll
  for (int p = 0; p < 32; ++p) {
    const int ep = pv_e(p), hp = pv_hh(p);
    const bool mine = (hh == hp);
    const float Lrp = D[rl * kPvL + p];
    const float a = mine ? ((rl == p) ? Lrp - 1.0f : Lrp) : 0.0f;
    const float b = mine ? y[ep] * pv_rl(ilr, p) : 0.0f;
    y = __builtin_amdgcn_mfma_f32_32x32x2f32(-a, b, y, 0, 0, 0);
  }
  pv_store(y, D, rl, hh);
}

// lower 32 x 32 blocks n = i (i + 1) / 2 + j of the pivot block per wave (up to 3): longest-processing-
// time assignment for the L^-T L^-1 products (block n costs 8 - i), reused as the wave -> block map
// of the fused diagonal-block update
static __constant__ signed char kLauum[16][3] = {{0, -1, -1},  {1, 31, -1},  {2, 32, -1},  {3, 26, -1},
                                          {4, 27, -1},  {5, 28, 33},  {6, 22, 34},  {7, 23, 35},
                                          {8, 24, -1},  {9, 25, -1},  {10, 17, -1}, {11, 18, -1},
                                          {12, 19, -1}, {13, 20, -1}, {14, 21, 29}, {15, 16, 30}};
__device__ inline void pv_ij(int n, int& i, int& j) {
  i = 0;
  while ((i + 1) * (i + 2) / 2 <= n) ++i;
  j = n - i * (i + 1) / 2;
}

// acc[h] += A(I_h) B(J_h)^T over K = 256 on the f16 cores (x3 split) for up to NB 32 x 32 blocks per
// wave (I_h < 0: none), A = (src[0] hi, src[1] lo) and B = (src[2], src[3]) fp16 planes, 256 rows of
// 256 halves each.  K in 4 chunks of 64 staged in the pivot's LDS ([4 parts][256 rows][72 halves]: the
// 144-B row pitch puts a 16-lane ds_read_b128 phase on 16 distinct bank groups); PREF: the next chunk's
// global loads are issued under the current chunk's MFMAs (8 more VGPR quads).  SAMEAB: B = A (only the
// A parts are loaded, B's fragments read from them: half the bytes of X X^T).  BTRI: B is lower
// triangular ([row][k] = 0 for k > row): chunk kc loads only B rows >= kc and skips the blocks J_h whose
// rows all lie above it (the zero upper half of Y_kk in X = C Y_kk^T).  Ends after a barrier only if the
// caller adds one: the staging area is still being read.
constexpr int kPvKC = 64, kPvKP = kPvKC + 8;
template <int NB, bool PREF, bool SAMEAB = false, bool BTRI = false>
__device__ inline void pv_x3_gemm(const _Float16* const* src, float* __restrict__ lf, const int* bi, const int* bj,
                                  pv_f32x16* acc, const int64_t* sld = nullptr) {
  // sld: row stride (halves) of each of the 4 sources (nullptr: kSwB, the [256][256] plane blocks)
  const int tid = threadIdx.x, lane = tid & 63, rl = lane & 31, hh = lane >> 5;
  constexpr int NU = SAMEAB ? 4 : 8;  // 16-B pieces per thread and chunk
  _Float16* st = reinterpret_cast<_Float16*>(lf);
  x3_half8 v[NU];
  auto need = [&](int u, int kc) {  // (thread-dependent) the piece is not a zero of a triangular B
    const int e = tid + 1024 * u, p = e >> 11, row = (e >> 3) & 255;
    return !(BTRI && p >= 2 && row < kc);
  };
  auto load = [&](int kc) {
#pragma unroll
    for (int u = 0; u < NU; ++u) {  // parts x 256 rows x 8 16-B chunks
      const int e = tid + 1024 * u, p = e >> 11, row = (e >> 3) & 255, c8 = e & 7;
      if (need(u, kc)) v[u] = *reinterpret_cast<const x3_half8*>(src[p] + row * (sld ? sld[p] : kSwB) + kc + 8 * c8);
    }
  };
  if (PREF) load(0);
  for (int kc = 0; kc < kSwB; kc += kPvKC) {
    __syncthreads();  // the previous chunk's readers are done
    if (PREF) {
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int e = tid + 1024 * u, p = e >> 11, row = (e >> 3) & 255, c8 = e & 7;
        if (need(u, kc)) *reinterpret_cast<x3_half8*>(st + (p * kSwB + row) * kPvKP + 8 * c8) = v[u];
      }
    } else {  // rounds of 4 (fewer live registers beside a 4-block accumulator set)
#pragma unroll
      for (int q = 0; q < NU / 4; ++q) {
        x3_half8 t[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int e = tid + 1024 * (4 * q + u), p = e >> 11, row = (e >> 3) & 255, c8 = e & 7;
          if (need(4 * q + u, kc))
            t[u] = *reinterpret_cast<const x3_half8*>(src[p] + row * (sld ? sld[p] : kSwB) + kc + 8 * c8);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int e = tid + 1024 * (4 * q + u), p = e >> 11, row = (e >> 3) & 255, c8 = e & 7;
          if (need(4 * q + u, kc)) *reinterpret_cast<x3_half8*>(st + (p * kSwB + row) * kPvKP + 8 * c8) = t[u];
        }
      }
    }
    __syncthreads();
    if (PREF && kc + kPvKC < kSwB) load(kc + kPvKC);
#pragma unroll
    for (int h = 0; h < NB; ++h) {
      if (bi[h] < 0) continue;
      if (BTRI && 32 * bj[h] + 31 < kc) continue;  // (wave-uniform) a zero chunk of the triangular B
      const _Float16* ar = st + (32 * bi[h] + rl) * kPvKP;
      const _Float16* br = st + ((SAMEAB ? 0 : 2 * kSwB) + 32 * bj[h] + rl) * kPvKP;
#pragma unroll
      for (int ks = 0; ks < kPvKC / 16; ++ks) {
        const int ko = 16 * ks + 8 * hh;
        const x3_half8 aH = *reinterpret_cast<const x3_half8*>(ar + ko);
        const x3_half8 aL = *reinterpret_cast<const x3_half8*>(ar + kSwB * kPvKP + ko);
        const x3_half8 bH = *reinterpret_cast<const x3_half8*>(br + ko);
        const x3_half8 bL = *reinterpret_cast<const x3_half8*>(br + kSwB * kPvKP + ko);
        acc[h] = __builtin_amdgcn_mfma_f32_32x32x16_f16(aL, bH, acc[h], 0, 0, 0);
        acc[h] = __builtin_amdgcn_mfma_f32_32x32x16_f16(aH, bL, acc[h], 0, 0, 0);
        acc[h] = __builtin_amdgcn_mfma_f32_32x32x16_f16(aH, bH, acc[h], 0, 0, 0);
      }
    }
  }
}

}  // namespace lvae
