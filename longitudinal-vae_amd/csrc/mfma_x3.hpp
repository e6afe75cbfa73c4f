// mfma_x3.hpp -- fp32-accurate 128x128 tile GEMM on the f16 matrix cores (3-product split).
//
// gfx950 has no xf32: fp32-input MFMA runs at 1/16 of the f16 rate (157 vs 2500 TFLOP/s dense).
// Each fp32 operand x is split once, while it is staged into LDS, into x sc = hi + lo with hi, lo
// fp16 (sc a power of two from a bound on the operand's max |x|, x3_scale: the largest entries
// land in [2^13, 2^14), far from fp16 overflow, and lo stays normal down to 2^-17 of them), and a product is
// hi_a hi_b + hi_a lo_b + lo_a hi_b: three v_mfma_f32_32x32x16_f16 with fp32 accumulation.  The
// dropped lo_a lo_b term and the split leave a relative error ~2^-22 per product -- between fp32
// (2^-24) and anything a 16-bit format gives -- at 3/16 of the fp32-MFMA cost.
//
// Same interface as tile_gemm (mfma_tile.hpp): 256 threads = 2x2 waves of 64x64, the fp32 Frag
// accumulators (the 32x32 C/D layout is dtype-independent on gfx950), fp32 operands in global
// memory with k contiguous (KCONT) or rows contiguous (!KCONT), optional per-k scale of op(A),
// NEG for acc -= op(A) op(B).  K chunks of kX3BK, register prefetch of the next chunk.
//
// f16 operand maps (cdna_hip_programming.md §3): lane l holds A[row l&31][k = 8(l>>5) + j] and
// B[k = 8(l>>5) + j][col l&31], j = 0..7 -- both read as 8 contiguous halves of one LDS row
// [row][k] (pitch kX3BK + 8 halves: 16 lanes of a ds_read_b128 phase start 16 B-groups apart).
#pragma once
#include "mfma_tile.hpp"

namespace lvae {

typedef _Float16 x3_half8 __attribute__((ext_vector_type(8)));
typedef _Float16 x3_half4 __attribute__((ext_vector_type(4)));

#ifndef LVAE_X3_BK
#define LVAE_X3_BK 32
#endif
constexpr int kX3BK = LVAE_X3_BK;              // K chunk per LDS stage
constexpr int kX3Ld = kX3BK + 8;               // LDS row pitch in halves (16-B aligned rows)
constexpr int kX3Op = kTM * kX3Ld;             // halves per operand part (hi or lo)

constexpr int x3_lds_bytes() { return 4 * kX3Op * (int)sizeof(_Float16); }

// x = (hi + lo) / sc: sc is a power of two chosen by the caller from a bound on |x| (x3_scale) so
// that |x sc| stays below 2^14 -- fp16 overflows at 65504 -- and the split stays exact in sc.
__device__ inline void x3_split(float x, float sc, _Float16& hi, _Float16& lo) {
  const float s = x * sc;
  hi = (_Float16)s;
  lo = (_Float16)(s - (float)hi);
}


// Register prefetch of one 128 x kX3BK fp32 chunk (NV = kX3BK / 8 float4 per thread).
//  KCONT (ptr[row * ld + k]): thread t holds rows (t >> 3) + 32 i (i < NV/2... see below), k-quads.
//  !KCONT (ptr[k * ld + row]): thread t loads 4 x 4 blocks rows 4(t&31)..+3 x k 4((t>>5) + 8 q)..+3
//  (coalesced float4 row loads); after a register transpose each row's 4 k are contiguous.
template <bool KCONT>
struct X3Chunk {
  static constexpr int NV = kX3BK / 8;
  f32x4 v[NV];
  __device__ inline void load(const float* __restrict__ base, int64_t ld, int k0) {
    const int t = threadIdx.x;
    if constexpr (KCONT) {
      // kX3BK/4 float4 per row; 256 threads cover 256 * 4 / kX3BK rows per pass
      constexpr int QPR = kX3BK / 4, RPP = 256 / QPR;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int row = t / QPR + RPP * i, q = t % QPR;
        v[i] = *reinterpret_cast<const f32x4*>(base + (int64_t)row * ld + k0 + q * 4);
      }
    } else {
      const int c4 = t & 31, kq = t >> 5;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int kb = 4 * (kq + 8 * (i >> 2)) + (i & 3);
        v[i] = *reinterpret_cast<const f32x4*>(base + (int64_t)(k0 + kb) * ld + c4 * 4);
      }
    }
  }
  __device__ inline void scale_k(const float* __restrict__ s, int k0) {
    const int t = threadIdx.x;
    if constexpr (KCONT) {
      constexpr int QPR = kX3BK / 4;
      const f32x4 sv = *reinterpret_cast<const f32x4*>(s + k0 + (t % QPR) * 4);
#pragma unroll
      for (int i = 0; i < NV; ++i) v[i] *= sv;
    } else {
      const int kq = t >> 5;
#pragma unroll
      for (int i = 0; i < NV; ++i) v[i] *= s[k0 + 4 * (kq + 8 * (i >> 2)) + (i & 3)];
    }
  }
  __device__ inline void negate() {
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = -v[i];
  }
};

// Stage one prefetched fp32 chunk as hi / lo halves of x * sc in [row][k] layout.
template <bool KCONT>
__device__ inline void x3_store(const X3Chunk<KCONT>& c, float sc, _Float16* __restrict__ hi,
                                _Float16* __restrict__ lo) {
  const int t = threadIdx.x;
  if constexpr (KCONT) {
    constexpr int QPR = kX3BK / 4, RPP = 256 / QPR;
#pragma unroll
    for (int i = 0; i < X3Chunk<true>::NV; ++i) {
      const int row = t / QPR + RPP * i, k = (t % QPR) * 4;
      x3_half4 h, l;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        _Float16 a, b;
        x3_split(c.v[i][e], sc, a, b);
        h[e] = a;
        l[e] = b;
      }
      *reinterpret_cast<x3_half4*>(hi + row * kX3Ld + k) = h;
      *reinterpret_cast<x3_half4*>(lo + row * kX3Ld + k) = l;
    }
  } else {
    const int row0 = (t & 31) * 4, kq = t >> 5;
#pragma unroll
    for (int g = 0; g < X3Chunk<false>::NV / 4; ++g) {
      const int k = 4 * (kq + 8 * g);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        x3_half4 h, l;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          _Float16 a, b;
          x3_split(c.v[4 * g + kk][e], sc, a, b);
          h[kk] = a;
          l[kk] = b;
        }
        *reinterpret_cast<x3_half4*>(hi + (row0 + e) * kX3Ld + k) = h;
        *reinterpret_cast<x3_half4*>(lo + (row0 + e) * kX3Ld + k) = l;
      }
    }
  }
}

__device__ inline void x3_mma_chunk(const _Float16* __restrict__ ah, const _Float16* __restrict__ al,
                                    const _Float16* __restrict__ bh, const _Float16* __restrict__ bl, Frag& f) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w >> 1) * 64, wn = (w & 1) * 64;
  const int r = lane & 31, kh = (lane >> 5) * 8;
#pragma unroll
  for (int kk = 0; kk < kX3BK; kk += 16) {
    x3_half8 aH[2], aL[2], bH[2], bL[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int ao = (wm + 32 * q + r) * kX3Ld + kk + kh, bo = (wn + 32 * q + r) * kX3Ld + kk + kh;
      aH[q] = *reinterpret_cast<const x3_half8*>(ah + ao);
      aL[q] = *reinterpret_cast<const x3_half8*>(al + ao);
      bH[q] = *reinterpret_cast<const x3_half8*>(bh + bo);
      bL[q] = *reinterpret_cast<const x3_half8*>(bl + bo);
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        f.acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(aL[a], bH[b], f.acc[a][b], 0, 0, 0);
        f.acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(aH[a], bL[b], f.acc[a][b], 0, 0, 0);
        f.acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(aH[a], bH[b], f.acc[a][b], 0, 0, 0);
      }
  }
}

__device__ inline void frag_scale(Frag& f, float s) {
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) f.acc[a][b][r] *= s;
}

// acc (+/-)= op(A)[128 x K] op(B)[K x 128] over k in [kbeg, kend) (multiples of kX3BK),
// fp32-accurate on the f16 matrix cores.  lds: x3_lds_bytes() bytes, 16-B aligned.  sa / sb: the
// split scales of op(A) / op(B) (x3_scale of a bound on each operand's max |entry|).
template <bool AK, bool BKc, bool NEG = false>
__device__ inline void tile_gemm_x3(const float* __restrict__ A, int64_t lda, const float* __restrict__ B, int64_t ldb,
                                    int kbeg, int kend, Frag& f, _Float16* __restrict__ lds, float sa, float sb,
                                    const float* __restrict__ ascale = nullptr) {
  if (kend <= kbeg) return;
  _Float16* ah = lds;
  _Float16* al = lds + kX3Op;
  _Float16* bh = lds + 2 * kX3Op;
  _Float16* bl = lds + 3 * kX3Op;
  const float sab = sa * sb;
  frag_scale(f, sab);  // accumulate in sa sb units (exact: powers of two)
  X3Chunk<AK> ca;
  X3Chunk<BKc> cb;
  ca.load(A, lda, kbeg);
  cb.load(B, ldb, kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += kX3BK) {
    if (ascale) ca.scale_k(ascale, k0);
    if constexpr (NEG) ca.negate();
    __syncthreads();  // previous chunk fully consumed
    x3_store<AK>(ca, sa, ah, al);
    x3_store<BKc>(cb, sb, bh, bl);
    __syncthreads();
    if (k0 + kX3BK < kend) {
      ca.load(A, lda, k0 + kX3BK);
      cb.load(B, ldb, k0 + kX3BK);
    }
    x3_mma_chunk(ah, al, bh, bl, f);
  }
  frag_scale(f, 1.0f / sab);
}

}  // namespace lvae
