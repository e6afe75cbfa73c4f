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
// An operand may also be a plain row-major plane (rows of ld halves, K contiguous; C16Opnd.ld != 0): its
// DMA pieces are then 32 rows x 2 16-B chunks, the chunk swizzle applied on the global address (the
// LDS image is the same), at twice the requests per byte.
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

// one operand of the core: the panel of its 256 rows from the first K chunk of the range on, in the
// chunk-major layout (ld == 0) or row-major (row stride ld halves); lo = lo plane - hi plane (halves)
struct C16Opnd {
  const _Float16* hi;
  int64_t lo;
  int64_t ld;
};

// the DMA addressing of one wave: part p = w >> 1 (A hi, A lo, B hi, B lo), pieces 4 (w & 1) .. + 3 of it
// (32-row blocks).  Piece blk of stage c reads base + c cs + blk bs + lane_off: chunk-major cs = 4096,
// bs = 512, lane_off = 8 lane (1 KB runs); row-major cs = 16, bs = 32 ld, lane_off = row (lane >> 1) and
// logical chunk (lane & 1) ^ (bit 3 of the row) (the swizzle moved to the source).  Set once per GEMM
// from wave-uniform scalars: no branch at the issue.
struct C16Dma {
  const _Float16* g;  // + lane_off, + (w & 1) * 4 blocks
  int64_t cs, bs;
  int doff;           // LDS offset (halves) of the wave's first piece in a stage
  int rev_nk;         // 0: chunks in order; nk: step c reads chunk nk - 1 - c (the K range from its end)
};
__device__ inline C16Dma c16_dma(const C16Opnd& A, const C16Opnd& B) {
  // the wave id through readfirstlane: provably uniform, so the LDS base (M0) needs no waterfall loop
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), p = w >> 1;
  const bool isb = p >= 2;
  const uintptr_t hi = isb ? (uintptr_t)B.hi : (uintptr_t)A.hi;
  const int64_t lo = isb ? B.lo : A.lo, ld = isb ? B.ld : A.ld;
  C16Dma d;
  d.cs = ld ? kC16BK : kC16Part;
  d.bs = ld ? 32 * ld : 512;
  const int64_t lane_off = ld ? (lane >> 1) * ld + 8 * ((lane & 1) ^ ((lane >> 4) & 1)) : 8 * lane;
  d.g = reinterpret_cast<const _Float16*>(hi) + (p & 1) * lo + 4 * (w & 1) * d.bs + lane_off;
  d.doff = p * kC16Part + (w & 1) * 2048;
  d.rev_nk = 0;
  return d;
}
__device__ inline void c16_issue(const C16Dma& d, int c, _Float16* __restrict__ stage) {
  const _Float16* g = d.g + (int64_t)(d.rev_nk ? d.rev_nk - 1 - c : c) * d.cs;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    __builtin_amdgcn_global_load_lds((const void*)(g + q * d.bs), (void*)(stage + d.doff + q * 512), 16, 0, 0);
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
// buffer into `nxt` (unused).  rescale(s, acc) runs first (callers with per-K-block split scales move
// the accumulators to the units of the block that starts at chunk s).
template <int NS, typename Rescale>
__device__ inline void c16_step(const C16Dma& dma, int s, int nk, _Float16* __restrict__ lds, const C16Frags& cur,
                                C16Frags& nxt, sx_f32x16 (&acc)[4][2], Rescale& rescale) {
  rescale(s, acc);
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
  c16_issue(dma, min(s + NS - 1, nk - 1), lds + ((s + NS - 1) % NS) * kC16Stage);
  c16_mma(cur, acc);
  c16_interleave();
}

struct C16NoRescale {
  __device__ void operator()(int, sx_f32x16 (&)[4][2]) const {}
};

// acc[a][b] += A B^T over nk 16-deep chunks (A, B: C16Opnd panels); lds = NS * kC16Stage halves, the
// kernel's only staging object; nk even; rescale(s, acc) at the top of every step (state kept in the
// caller's functor).  rev: the chunks from the last to the first (tiles whose K ranges end together then read
// the same chunks at the same time: the shared panels stay in L2).  Returns with no DMA outstanding.
template <int NS, typename Rescale>
__device__ inline void c16_gemm(const C16Opnd& A, const C16Opnd& B, int nk, _Float16* __restrict__ lds,
                                sx_f32x16 (&acc)[4][2], Rescale& rescale, bool rev = false) {
  C16Dma dma = c16_dma(A, B);
  dma.rev_nk = rev ? nk : 0;
#pragma unroll
  for (int s = 0; s < NS - 1; ++s) c16_issue(dma, min(s, nk - 1), lds + s * kC16Stage);
  c16_wait_vm<4 * (NS - 2)>();
  __builtin_amdgcn_s_barrier();
  C16Frags f0, f1;
  c16_read(lds, f0);
  // two steps per trip (nk is even: whole 256-deep blocks of 16 chunks): the fragment sets keep static
  // names (no runtime-indexed register arrays), and no branch between the steps invites the compiler to
  // sink a step's fragment reads past its MFMAs
  for (int s = 0; s < nk; s += 2) {
    c16_step<NS>(dma, s, nk, lds, f0, f1, acc, rescale);
    c16_step<NS>(dma, s + 1, nk, lds, f1, f0, acc, rescale);
  }
  c16_wait_vm<0>();  // the re-read pieces past the last chunk: none may land after the workgroup ends
}
template <int NS>
__device__ inline void c16_gemm(const C16Opnd& A, const C16Opnd& B, int nk, _Float16* __restrict__ lds,
                                sx_f32x16 (&acc)[4][2]) {
  C16NoRescale none;
  c16_gemm<NS>(A, B, nk, lds, acc, none);
}

// per-K-block split scales (operands split with a power-of-two scale per 256 x 256 block, sprod[kb] =
// sA(kb) sB(kb) in LDS): the accumulators move to the units of each new block at its first chunk (ratios
// of powers of two: exact); value = acc / scur at the end
struct C16BlockRescale {
  const float* sprod;
  float scur;
  int rev_nk = 0;  // (c16_gemm's rev: step s is chunk rev_nk - 1 - s; nk a multiple of 16)
  __device__ void operator()(int s, sx_f32x16 (&acc)[4][2]) {
    const int b = (rev_nk ? rev_nk - 1 - s : s) >> 4;
    if (s == 0) {
      scur = sprod[b];
    } else if ((s & 15) == 0) {
      const float snew = sprod[b], ratio = snew / scur;
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] *= ratio;
      scur = snew;
    }
  }
};

// accumulator tile (value = acc * colmul(b), colmul: the multiplier of the lane's column block b) -> the fp16
// hi / lo planes of one 256 x 256 tile in the chunk-major layout (hi, lo: the tile's base, c16_off of its
// first element: 16 chunks of 8 KB).  Lane (w, lane) holds chunk (w & 3) 4 + 2 b + (lane & 31) / 16, half
// (lane & 15) of rows sx_row(a, e); bit 3 of the row is bit 0 of e >> 2, so the half's swizzle is a
// compile-time choice per e.
template <typename ColMul>
__device__ inline void c16_tile_planes_out(const sx_f32x16 (&acc)[4][2], ColMul colmul, _Float16* __restrict__ hi,
                                           _Float16* __restrict__ lo) {
  const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc(hi, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(lo, (short)0, 0x7fffffff, 0x00020000);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int vb0 = (((w & 3) * 4 + ((lane & 31) >> 4)) * kC16Part + ((w >> 2) * 128 + 4 * (lane >> 5)) * 16) * 2;
  const int vk0 = (lane & 15) * 2, vk1 = ((lane & 15) ^ 8) * 2;
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const float mc = colmul(b);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const float y = acc[a][b][e] * mc;
        const _Float16 yh = (_Float16)y;
        const _Float16 yl = (_Float16)(y - (float)yh);
        const int vo = vb0 + (((e >> 2) & 1) ? vk1 : vk0);
        const int so = (2 * b * kC16Part + (32 * a + (e & 3) + 8 * (e >> 2)) * 16) * 2;
        __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, yh), rh, vo, so, 0);
        __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, yl), rl, vo, so, 0);
      }
  }
}

}  // namespace lvae
