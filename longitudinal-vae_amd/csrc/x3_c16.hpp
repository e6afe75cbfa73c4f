// x3_c16.hpp -- 256 x 256 output tiles on the f16 matrix cores with the fp32-accurate 3-product split
// (mfma_x3.hpp), operands PRE-SPLIT in a K-CHUNK-MAJOR plane layout, staged global -> LDS by DMA through
// a ring of NS 16-deep stages (NS - 3 stay in flight across each barrier, and the DMA of the stage NS - 1
// ahead is issued right after it), each wave's fragments for the next stage read from LDS while the
// MFMAs of the current stage run (no ds_read latency exposed behind a barrier).
//
// Chunk-major layout (c16 planes): a plane of np rows x np columns is stored as
//   [row block R (256 rows)][K chunk c (16 columns)][row r in the block (256)][16 halves]
// so one stage of one operand part (256 rows x 16 k) is ONE contiguous 8 KB block: every DMA piece is a
// whole 1 KB run (full cache lines; the row-major planes' 32-B row segments per 16-deep chunk doubled the
// L2 traffic, syrk_x3.hip).  Inside a row the two 8-half groups are swapped when bit 3 of r is set
// (stored at position kk ^ 8 (r >> 3 & 1)): the producer applies the swizzle, the DMA copies linearly,
// and a ds_read_b128 lane group (16 consecutive rows, one 8-half group) then covers all 64 banks.
//
// 512 threads = 8 waves (2 along M x 4 along N, 128 x 64 each = 4 x 2 blocks of
// v_mfma_f32_32x32x16_f16, three products per block): 24 MFMAs, 12 ds_read_b128 and 4 DMA pieces per
// wave and stage.  The accumulator layout is x3_dma.hpp's (sx_row / sx_col).
#pragma once
#include "x3_dma.hpp"

namespace lvae {

// the S GEMM's operand planes (B = K^-1 diag(sqrt v), written by the exact KL's lauum epilogue) are in
// this layout and the S GEMM runs on this core (false: row-major planes and syrk_tiles_kernel)
constexpr bool kCiBC16 = true;
#ifndef LVAE_C16NS
#define LVAE_C16NS 5
#endif
constexpr int kC16NS = LVAE_C16NS;          // stages of the product S GEMM's ring (-D for dev A/B builds)

constexpr int kC16BK = 16;                  // K chunk (halves) per stage
constexpr int kC16Part = 256 * kC16BK;      // halves per operand part per stage (8 KB)
constexpr int kC16Stage = 4 * kC16Part;     // halves per stage (32 KB)

// offset (halves) of element (row, col) of plane l in the chunk-major layout (np % 256 == 0)
__host__ __device__ inline int64_t c16_off(int64_t l, int np_, int row, int col) {
  const int R = row >> 8, r = row & 255, c = col >> 4, kk = col & 15;
  return l * np_ * np_ + ((int64_t)R * (np_ >> 4) + c) * kC16Part + r * 16 + (kk ^ (((r >> 3) & 1) << 3));
}
// the chunk-major panel of row block R of plane l: stage c starts at + c * kC16Part
__host__ __device__ inline int64_t c16_panel(int64_t l, int np_, int R) {
  return l * np_ * np_ + (int64_t)R * (np_ >> 4) * kC16Part;
}

// one stage: 4 parts x 8 pieces of 1 KB; wave w issues pieces 4 (w & 1) .. + 3 of part w >> 1.  Part p's
// panel is a + (p & 1) lo + (p >> 1) b (halves): uniform integer arithmetic, no select branches.
__device__ inline void c16_issue(const _Float16* __restrict__ a, int64_t lo, int64_t b, int c,
                                 _Float16* __restrict__ stage) {
  // the wave id through readfirstlane: provably uniform, so the LDS base (M0) needs no waterfall loop
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), p = w >> 1;
  const _Float16* g = a + (p & 1) * lo + (p >> 1) * b + (int64_t)c * kC16Part + (w & 1) * 2048 + lane * 8;
  _Float16* d = stage + p * kC16Part + (w & 1) * 2048;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    __builtin_amdgcn_global_load_lds((const void*)(g + q * 512), (void*)(d + q * 512), 16, 0, 0);
}

struct C16Frags {
  sx_half8 aH[4], aL[4], bH[2], bL[2];
};

__device__ inline sx_half8 c16_frag(const _Float16* __restrict__ part, int row, int h) {
  return *reinterpret_cast<const sx_half8*>(part + row * kC16BK + ((h ^ ((row >> 3) & 1)) << 3));
}

__device__ inline void c16_read(const _Float16* __restrict__ st, C16Frags& f) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w >> 2) * 128, wn = (w & 3) * 64, r32 = lane & 31, kh = lane >> 5;
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    f.bH[b] = c16_frag(st + 2 * kC16Part, wn + 32 * b + r32, kh);
    f.bL[b] = c16_frag(st + 3 * kC16Part, wn + 32 * b + r32, kh);
  }
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    f.aH[a] = c16_frag(st, wm + 32 * a + r32, kh);
    f.aL[a] = c16_frag(st + kC16Part, wm + 32 * a + r32, kh);
  }
}

__device__ inline void c16_mma(const C16Frags& f, sx_f32x16 (&acc)[4][2]) {
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.aL[a], f.bH[b], acc[a][b], 0, 0, 0);
      acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.aH[a], f.bL[b], acc[a][b], 0, 0, 0);
      acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.aH[a], f.bH[b], acc[a][b], 0, 0, 0);
    }
}

// vmcnt(n) for n < 64, expcnt / lgkmcnt untouched
template <int N>
__device__ inline void c16_wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt(0x0F70 | (N & 15) | ((N >> 4) << 14));
}
// the issue order of a step's MFMAs and DMA pieces (sched_group_barrier masks: MFMA 0x8, VMEM read 0x20):
// the 4 pieces spread between the MFMAs, so they issue in the MFMAs' shadow instead of as a burst after
// the barrier with the matrix pipe idle
__device__ inline void c16_interleave() {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    __builtin_amdgcn_sched_group_barrier(0x20, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x8, 6, 0);
  }
}

// one ring step: stage s's fragments are in `cur`; stage s+1's are read into `nxt` under the MFMAs, and
// the DMA of stage s+NS-1 is issued.  Every step issues one (branch-free: past the last chunk it re-reads
// chunk nk-1 into the buffer of stage s-1, which no later step reads for real), so stages s+2 .. s+NS-2
// (NS - 3 of them) may stay in flight while stage s+1 must have landed.  The last step reads a stale
// buffer into `nxt` (unused).
template <int NS>
__device__ inline void c16_step(const _Float16* __restrict__ a, int64_t lo, int64_t b, int s, int nk,
                                _Float16* __restrict__ lds, const C16Frags& cur, C16Frags& nxt,
                                sx_f32x16 (&acc)[4][2]) {
  c16_wait_vm<4 * (NS - 3)>();
  // this wave's reads of stage s (into cur, issued a step ago under the MFMAs) retired: a counted wait
  // the compiler sees, so it needs none between the reads below and the MFMAs on cur
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  // every wave's DMA of stage s+1 has landed; every wave's reads of the buffer that stage s+NS-1 takes
  // (stage s-1's, read during step s-2) are retired
  __builtin_amdgcn_s_barrier();
  // the next stage's 12 fragment reads first, fenced from the scheduler (which would otherwise sink them
  // below the MFMAs into the registers the MFMAs free, exposing their latency at the next barrier)
  c16_read(lds + ((s + 1) % NS) * kC16Stage, nxt);
  __builtin_amdgcn_sched_barrier(0);
  c16_issue(a, lo, b, min(s + NS - 1, nk - 1), lds + ((s + NS - 1) % NS) * kC16Stage);
  c16_mma(cur, acc);
  c16_interleave();
}

// acc[a][b] += A B^T over nk 16-deep chunks: A = (a hi, a + lo lo), B = (a + b hi, a + b + lo lo) chunk-major
// panels (stage c of a part at its panel + c * kC16Part); lds = NS * kC16Stage halves, the kernel's only
// __shared__ object; nk even.  Returns with no DMA outstanding.
template <int NS>
__device__ inline void c16_gemm(const _Float16* __restrict__ a, int64_t lo, int64_t b, int nk,
                                _Float16* __restrict__ lds, sx_f32x16 (&acc)[4][2]) {
#pragma unroll
  for (int s = 0; s < NS - 1; ++s) c16_issue(a, lo, b, min(s, nk - 1), lds + s * kC16Stage);
  c16_wait_vm<4 * (NS - 2)>();
  __builtin_amdgcn_s_barrier();
  C16Frags f0, f1;
  c16_read(lds, f0);
  // two steps per trip (nk is even: whole 256-deep blocks of 16 chunks): the fragment sets keep static
  // names (no runtime-indexed register arrays), and no branch between the steps invites the compiler to
  // sink a step's fragment reads past its MFMAs
  for (int s = 0; s < nk; s += 2) {
    c16_step<NS>(a, lo, b, s, nk, lds, f0, f1, acc);
    c16_step<NS>(a, lo, b, s + 1, nk, lds, f1, f0, acc);
  }
  c16_wait_vm<0>();  // the re-read pieces past the last chunk: none may land after the workgroup ends
}

}  // namespace lvae
