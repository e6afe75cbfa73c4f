// x3_dma.hpp -- 256 x 256 output tiles on the f16 matrix cores with the fp32-accurate 3-product
// split (see mfma_x3.hpp for the error argument), operands PRE-SPLIT in global memory as fp16 hi / lo
// planes [row][k] and staged global -> LDS by DMA (global_load_lds_dwordx4, no VGPR round trip).
// 512 threads = 8 waves (2 along M x 4 along N, 128 x 64 each, 4 x 2 blocks of
// v_mfma_f32_32x32x16_f16, three products per block and k-step).  Shared by syrk_x3.hip (S =
// K^-1 V K^-1) and spd_sweep.hip (the sweep's rank-256 updates).
//
// LDS image of one operand part and chunk: [256 rows][32 halves] (64 B rows), 16-B chunk c of
// row r stored at chunk c ^ ((r >> 2) & 3): a ds_read_b128 phase (16 lanes = 16 consecutive rows,
// one logical chunk) then touches 16 distinct 16-B bank groups.  The swizzle is applied on the
// per-lane GLOBAL address of the DMA (its LDS side is lane-linear).
#pragma once
#include "common.hpp"

namespace lvae {

typedef _Float16 sx_half8 __attribute__((ext_vector_type(8)));
typedef _Float16 sx_half4 __attribute__((ext_vector_type(4)));
typedef float sx_f32x16 __attribute__((ext_vector_type(16)));
typedef float sx_f32x4 __attribute__((ext_vector_type(4)));

constexpr int kSxT = 256;                // output tile edge
constexpr int kSxBK = 32;                // K chunk (halves) per LDS stage
constexpr int kSxPart = kSxT * kSxBK;    // halves per operand part per stage (16 KB)

// linear index t of a lower-triangular tile grid (row-major) -> (I, J), J <= I
__device__ inline void sx_tri(int t, int& I, int& J) {
  int r = (int)((sqrtf(8.0f * (float)t + 1.0f) - 1.0f) * 0.5f);
  while ((r + 1) * (r + 2) / 2 <= t) ++r;
  while (r * (r + 1) / 2 > t) --r;
  I = r;
  J = t - r * (r + 1) / 2;
}

// tile t of the lower triangle of an m x m tile grid in blocked order: row blocks of 4, inside a
// block by column, then row.  64 half-tile workgroups in flight on one XCD then touch ~4 W and ~8 C
// panels (3 MB, inside its 4 MB L2) instead of a few rows x every C panel (row-major order).
__device__ inline void sx_tri_blocked(int t, int m, int& I, int& J) {
  int r, c;
  sx_tri(t, r, c);  // row r of t in row-major order: t lies in row block r / 4 either way
  const int base = (r >> 2) << 2, h = min(4, m - base);
  int u = t - base * (base + 1) / 2;
  if (u < h * base) {
    J = u / h;
    I = base + u % h;
  } else {
    u -= h * base;
    int jj = 0;
    while (u >= h - jj) {
      u -= h - jj;
      ++jj;
    }
    J = base + jj;
    I = J + u;
  }
}

// one stage: 4 parts (A hi, A lo, B hi, B lo) x 16 wave-instructions of 1 KB; wave w issues
// instructions 2w, 2w+1 of every part -> 8 global_load_lds per thread.
__device__ inline void sx_issue(const _Float16* __restrict__ ah, const _Float16* __restrict__ al,
                                const _Float16* __restrict__ bh, const _Float16* __restrict__ bl, int64_t ld, int k0,
                                _Float16* __restrict__ stage) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const _Float16* src[4] = {ah, al, bh, bl};
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int blk = 2 * w + q;                      // 16-row block of the 256-row part
    const int row = 16 * blk + (lane >> 2);
    const int c = (lane & 3) ^ ((row >> 2) & 3);    // logical chunk stored at physical chunk lane&3
    const int64_t go = (int64_t)row * ld + k0 + 8 * c;
#pragma unroll
    for (int p = 0; p < 4; ++p)
      __builtin_amdgcn_global_load_lds((const void*)(src[p] + go), (void*)(stage + p * kSxPart + blk * 512), 16, 0,
                                       0);
  }
}

__device__ inline sx_half8 sx_frag(const _Float16* __restrict__ part, int row, int c) {
  return *reinterpret_cast<const sx_half8*>(part + row * kSxBK + ((c ^ ((row >> 2) & 3)) << 3));
}

#define SX_WAIT_VM(N) __builtin_amdgcn_s_waitcnt(0xF70 | (N))  // vmcnt(N), expcnt / lgkmcnt untouched


// one K chunk (kSxBK halves) of the staged stage: acc[a][b] += A_part rows x B_part rows
__device__ inline void sx_mma_stage(const _Float16* __restrict__ cur, sx_f32x16 (&acc)[4][2]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w >> 2) * 128, wn = (w & 3) * 64;
  const int r32 = lane & 31, kh = lane >> 5;
  const _Float16* pah = cur;
  const _Float16* pal = cur + kSxPart;
  const _Float16* pbh = cur + 2 * kSxPart;
  const _Float16* pbl = cur + 3 * kSxPart;
#pragma unroll
  for (int ks = 0; ks < kSxBK / 16; ++ks) {
    const int c = 2 * ks + kh;
    sx_half8 bH[2], bL[2];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      bH[b] = sx_frag(pbh, wn + 32 * b + r32, c);
      bL[b] = sx_frag(pbl, wn + 32 * b + r32, c);
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const sx_half8 aH = sx_frag(pah, wm + 32 * a + r32, c);
      const sx_half8 aL = sx_frag(pal, wm + 32 * a + r32, c);
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(aL, bH[b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(aH, bL[b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(aH, bH[b], acc[a][b], 0, 0, 0);
      }
    }
  }
}

// acc[a][b] += op(A) op(B)^T over k in [0, K): A = (ah, al) rows, B = (bh, bl) rows, leading dim
// ld halves; lds = 2 * 4 * kSxPart halves (128 KB).  The first stage's DMA is issued here.
__device__ inline void sx_gemm(const _Float16* __restrict__ ah, const _Float16* __restrict__ al,
                               const _Float16* __restrict__ bh, const _Float16* __restrict__ bl, int64_t ld, int K,
                               _Float16* __restrict__ lds, sx_f32x16 (&acc)[4][2]) {
  const int nk = K / kSxBK;
  sx_issue(ah, al, bh, bl, ld, 0, lds);
  for (int s = 0; s < nk; ++s) {
    // one barrier per K-chunk: it retires stage s (every wave waited for its own DMA of it) and
    // every wave's reads of stage s-1, whose buffer then receives stage s+1 while s is multiplied
    SX_WAIT_VM(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + 1 < nk) sx_issue(ah, al, bh, bl, ld, (s + 1) * kSxBK, lds + ((s + 1) & 1) * 4 * kSxPart);
    __builtin_amdgcn_s_setprio(1);
    sx_mma_stage(lds + (s & 1) * 4 * kSxPart, acc);
    __builtin_amdgcn_s_setprio(0);
  }
}

// sx_gemm over nkb whole 256-deep K blocks whose operand planes carry per-block split scales:
// sprod[kb] = sA(kb) sB(kb) (LDS, written before the first barrier here).  The accumulators move to
// the units of each new block at its first chunk (ratios of powers of two: exact); returns the units
// of the last block (value = acc / returned).
__device__ inline float sx_gemm_scaled(const _Float16* __restrict__ ah, const _Float16* __restrict__ al,
                                       const _Float16* __restrict__ bh, const _Float16* __restrict__ bl, int64_t ld,
                                       int nkb, const float* sprod, _Float16* __restrict__ lds,
                                       sx_f32x16 (&acc)[4][2]) {
  constexpr int cpb = 256 / kSxBK;  // K chunks per block
  const int nk = nkb * cpb;
  float scur = 1.f;
  sx_issue(ah, al, bh, bl, ld, 0, lds);
  for (int s = 0; s < nk; ++s) {
    SX_WAIT_VM(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + 1 < nk) sx_issue(ah, al, bh, bl, ld, (s + 1) * kSxBK, lds + ((s + 1) & 1) * 4 * kSxPart);
    if (s % cpb == 0) {
      const float snew = sprod[s / cpb];
      if (s) {
        const float ratio = snew / scur;
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b) acc[a][b] *= ratio;
      }
      scur = snew;
    }
    __builtin_amdgcn_s_setprio(1);
    sx_mma_stage(lds + (s & 1) * 4 * kSxPart, acc);
    __builtin_amdgcn_s_setprio(0);
  }
  return scur;
}

// accumulator element e of block (a, b) in lane: row / column inside the 256 x 256 tile
__device__ inline int sx_row(int a, int e) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  return (w >> 2) * 128 + 32 * a + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
}
__device__ inline int sx_col(int b) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  return (w & 3) * 64 + 32 * b + (lane & 31);
}

}  // namespace lvae
