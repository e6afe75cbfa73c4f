// x3_gemm4.hpp -- 256 x 256 output tiles on the f16 matrix cores with the fp32-accurate 3-product
// split (mfma_x3.hpp), operands PRE-SPLIT in global memory as fp16 hi / lo planes [row][k], staged
// global -> LDS by DMA (global_load_lds_dwordx4) through a FOUR-stage ring of 16-deep K chunks with
// three stages in flight across each barrier (counted vmcnt, raw s_barrier: the DMA latency from
// L2 / MALL is hidden by ~3 chunks of MFMA work instead of one).
//
// 256 threads = 4 waves (2 along M x 2 along N, one per SIMD), each 128 x 128 = 4 x 4 blocks of
// v_mfma_f32_32x32x16_f16 with three products per block and k-step: 48 MFMAs per wave between
// barriers, accumulators in the AGPR half of the unified register file (one wave per SIMD).
//
// LDS image of one operand part and stage: [256 rows][16 halves] (32-B rows); the 16-B chunk h of
// row r is stored at chunk h ^ ((r >> 3) & 1), which puts every ds_read_b128 lane group (16 rows
// of one chunk) on 16 distinct 16-B bank groups.  The swizzle is applied on the per-lane GLOBAL
// address of the DMA (its LDS side is lane-linear).
#pragma once
#include "x3_dma.hpp"

namespace lvae {

constexpr int kG4T = 256;                  // output tile edge
constexpr int kG4BK = 16;                  // K chunk (halves) per stage
constexpr int kG4NS = 4;                   // stages in the ring
constexpr int kG4Part = kG4T * kG4BK;      // halves per operand part per stage (8 KB)
constexpr int kG4Stage = 4 * kG4Part;      // halves per stage (32 KB)
constexpr int kG4Lds = kG4NS * kG4Stage;   // halves of LDS (128 KB)

// one stage: 4 parts (A hi, A lo, B hi, B lo) x 8 wave-instructions of 1 KB (32 rows x 2 chunks);
// wave w issues instructions 2w, 2w+1 of every part -> 8 global_load_lds per thread
__device__ inline void g4_issue(const _Float16* __restrict__ ah, const _Float16* __restrict__ al,
                                const _Float16* __restrict__ bh, const _Float16* __restrict__ bl, int64_t ld, int k0,
                                _Float16* __restrict__ stage) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const _Float16* src[4] = {ah, al, bh, bl};
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int blk = 2 * w + q;  // 32-row block of the 256-row part
    const int row = 32 * blk + (lane >> 1);
    const int c = (lane & 1) ^ ((row >> 3) & 1);  // logical chunk stored at physical chunk lane & 1
    const int64_t go = (int64_t)row * ld + k0 + 8 * c;
#pragma unroll
    for (int p = 0; p < 4; ++p)
      __builtin_amdgcn_global_load_lds((const void*)(src[p] + go), (void*)(stage + p * kG4Part + blk * 512), 16, 0, 0);
  }
}

__device__ inline sx_half8 g4_frag(const _Float16* __restrict__ part, int row, int h) {
  return *reinterpret_cast<const sx_half8*>(part + row * kG4BK + ((h ^ ((row >> 3) & 1)) << 3));
}

// one 16-deep K chunk of a staged stage: acc[a][b] += A rows x B rows (x3)
__device__ inline void g4_mma_stage(const _Float16* __restrict__ cur, sx_f32x16 (&acc)[4][4]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w >> 1) * 128, wn = (w & 1) * 128;
  const int r32 = lane & 31, kh = lane >> 5;
  const _Float16* pah = cur;
  const _Float16* pal = cur + kG4Part;
  const _Float16* pbh = cur + 2 * kG4Part;
  const _Float16* pbl = cur + 3 * kG4Part;
  sx_half8 bH[4], bL[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    bH[b] = g4_frag(pbh, wn + 32 * b + r32, kh);
    bL[b] = g4_frag(pbl, wn + 32 * b + r32, kh);
  }
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const sx_half8 aH = g4_frag(pah, wm + 32 * a + r32, kh);
    const sx_half8 aL = g4_frag(pal, wm + 32 * a + r32, kh);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(aL, bH[b], acc[a][b], 0, 0, 0);
      acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(aH, bL[b], acc[a][b], 0, 0, 0);
      acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(aH, bH[b], acc[a][b], 0, 0, 0);
    }
  }
}

// acc[a][b] += op(A) op(B)^T over k in [0, K) (K % 16 == 0): A = (ah, al) rows, B = (bh, bl) rows,
// leading dim ld halves; lds = kG4Lds halves (the kernel's only __shared__ object, or its first).
// rescale(s, acc): called before chunk s's MFMAs (s > 0, s % (256 / kG4BK) == 0 marks a new 256-block
// of K for callers with per-block split scales; others pass a no-op).
template <typename Rescale>
__device__ inline void g4_gemm(const _Float16* __restrict__ ah, const _Float16* __restrict__ al,
                               const _Float16* __restrict__ bh, const _Float16* __restrict__ bl, int64_t ld, int K,
                               _Float16* __restrict__ lds, sx_f32x16 (&acc)[4][4], Rescale rescale) {
  const int nk = K / kG4BK;
#pragma unroll
  for (int s = 0; s < kG4NS - 1; ++s)
    if (s < nk) g4_issue(ah, al, bh, bl, ld, s * kG4BK, lds + s * kG4Stage);
  for (int s = 0; s < nk; ++s) {
    // stage s landed (this wave's 8 DMAs of it); the stages issued after it (up to 2) stay in flight
    const int after = min(nk - 1, s + kG4NS - 2) - s;
    if (after >= 2) __builtin_amdgcn_s_waitcnt(0x4F70);       // vmcnt(16)
    else if (after == 1) __builtin_amdgcn_s_waitcnt(0x0F78);  // vmcnt(8)
    else __builtin_amdgcn_s_waitcnt(0x0F70);                  // vmcnt(0)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // every wave's DMA of stage s has landed and every wave's reads of stage s-1 have returned: the
    // buffer of stage s-1 takes stage s+3
    __builtin_amdgcn_s_barrier();
    if (s + kG4NS - 1 < nk)
      g4_issue(ah, al, bh, bl, ld, (s + kG4NS - 1) * kG4BK, lds + ((s + kG4NS - 1) % kG4NS) * kG4Stage);
    rescale(s, acc);
    __builtin_amdgcn_s_setprio(1);
    g4_mma_stage(lds + (s % kG4NS) * kG4Stage, acc);
    __builtin_amdgcn_s_setprio(0);
  }
}

// accumulator element e of block (a, b) in lane: row / column inside the 256 x 256 tile
__device__ inline int g4_row(int a, int e) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  return (w >> 1) * 128 + 32 * a + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
}
__device__ inline int g4_col(int b) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  return (w & 1) * 128 + 32 * b + (lane & 31);
}

}  // namespace lvae
