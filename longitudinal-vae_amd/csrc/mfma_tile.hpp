// mfma_tile.hpp -- 128x128 fp32 output tile on CDNA4 f32-input MFMA (v_mfma_f32_32x32x2_f32).
//
// 256 threads = 4 waves arranged 2x2; each wave owns a 64x64 sub-tile = 2x2 MFMA 32x32 blocks
// (4 x f32x16 accumulators = 64 acc registers).  K is consumed in chunks of BK=32 staged through
// LDS, with the next chunk prefetched into registers while the current one is multiplied.
//
// Operand layouts (element (m,k) of op(A), (k,n) of op(B)):
//   KCONT  : ptr[row * ld + k]   (row = m or n; k contiguous)  -> LDS [128][BK+1] (pad -> the
//            32 lanes of a half-wave read 32 rows at one k: banks (33 r + k) mod 32 all distinct)
//   !KCONT : ptr[k * ld + row]   (row contiguous)              -> LDS [BK][128] (lanes read
//            consecutive rows: conflict-free, 16-B aligned float4 stores)
// MFMA 32x32x2 f32 fragments (cdna_hip_programming.md §3): lane l holds A[l&31][l>>5],
// B[l>>5][l&31]; accumulator reg r of lane l is C[(r&3) + 8(r>>2) + 4(l>>5)][l&31].
#pragma once
#include "common.hpp"

namespace lvae {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kTM = 128;  // tile edge
constexpr int kBK = 32;   // K chunk
constexpr int kLdsK = kBK + 1;

template <bool KCONT>
struct OpLds {
  static constexpr int kFloats = KCONT ? kTM * kLdsK : kBK * kTM;
};

// Shared memory needed by one tile GEMM (A and B stages).
template <bool AK, bool BK_>
constexpr int tile_lds_floats() {
  return OpLds<AK>::kFloats + OpLds<BK_>::kFloats;
}

struct Frag {
  f32x16 acc[2][2];
  __device__ inline void zero() {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  }
};

// Register prefetch of one operand chunk: 128 x 32 floats = 4 float4 per thread.
template <bool KCONT>
struct OpChunk {
  f32x4 v[4];
  // base points at element (row 0, k 0) of the tile; k0 = chunk start.
  __device__ inline void load(const float* __restrict__ base, int64_t ld, int k0) {
    const int t = threadIdx.x;
    if constexpr (KCONT) {
      // 8 float4 per row; rows (t>>3) + 32 i
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = (t >> 3) + 32 * i, c4 = t & 7;
        v[i] = *reinterpret_cast<const f32x4*>(base + row * ld + k0 + c4 * 4);
      }
    } else {
      // 32 float4 per k-row; k-rows (t>>5) + 8 i
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = (t >> 5) + 8 * i, c4 = t & 31;
        v[i] = *reinterpret_cast<const f32x4*>(base + (int64_t)(k0 + k) * ld + c4 * 4);
      }
    }
  }
  // optional per-k scaling (A operand of K^-1 V K^-1): s points at scale[k0 .. k0+BK)
  __device__ inline void scale_k(const float* __restrict__ s, int k0) {
    const int t = threadIdx.x;
    if constexpr (KCONT) {
      const int c4 = t & 7;
      const f32x4 sv = *reinterpret_cast<const f32x4*>(s + k0 + c4 * 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] *= sv;
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] *= s[k0 + (t >> 5) + 8 * i];
    }
  }
  __device__ inline void negate() {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = -v[i];
  }
  __device__ inline void store(float* __restrict__ lds) const {
    const int t = threadIdx.x;
    if constexpr (KCONT) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = (t >> 3) + 32 * i, c4 = t & 7;
        float* p = lds + row * kLdsK + c4 * 4;
        p[0] = v[i][0];
        p[1] = v[i][1];
        p[2] = v[i][2];
        p[3] = v[i][3];
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = (t >> 5) + 8 * i, c4 = t & 31;
        *reinterpret_cast<f32x4*>(lds + k * kTM + c4 * 4) = v[i];
      }
    }
  }
};

template <bool KCONT>
__device__ inline float lds_frag(const float* __restrict__ lds, int row, int k) {
  if constexpr (KCONT) return lds[row * kLdsK + k];
  else return lds[k * kTM + row];
}

// Multiply the staged chunk into the accumulators (BK/2 MFMA k-steps x 4 blocks per wave).
template <bool AK, bool BKc>
__device__ inline void mma_chunk(const float* __restrict__ la, const float* __restrict__ lb, Frag& f) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w >> 1) * 64, wn = (w & 1) * 64;
  const int r = lane & 31, kh = lane >> 5;
#pragma unroll
  for (int kk = 0; kk < kBK; kk += 2) {
    const float a0 = lds_frag<AK>(la, wm + r, kk + kh);
    const float a1 = lds_frag<AK>(la, wm + 32 + r, kk + kh);
    const float b0 = lds_frag<BKc>(lb, wn + r, kk + kh);
    const float b1 = lds_frag<BKc>(lb, wn + 32 + r, kk + kh);
    f.acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, f.acc[0][0], 0, 0, 0);
    f.acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, f.acc[0][1], 0, 0, 0);
    f.acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, f.acc[1][0], 0, 0, 0);
    f.acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, f.acc[1][1], 0, 0, 0);
  }
}

// acc += op(A)[128 x K] * op(B)[K x 128] over k in [kbeg, kend) (multiples of BK); NEG: acc -= ...
// A / B point at element (row 0, k 0) of the tile's operand (k offsets are absolute).
// ascale (nullable): per-k scale applied to op(A) (used for K^-1 V K^-1).
template <bool AK, bool BKc, bool NEG = false>
__device__ inline void tile_gemm(const float* __restrict__ A, int64_t lda, const float* __restrict__ B, int64_t ldb,
                                 int kbeg, int kend, Frag& f, float* __restrict__ lds,
                                 const float* __restrict__ ascale = nullptr) {
  float* la = lds;
  float* lb = lds + OpLds<AK>::kFloats;
  if (kend <= kbeg) return;
  OpChunk<AK> ca;
  OpChunk<BKc> cb;
  ca.load(A, lda, kbeg);
  cb.load(B, ldb, kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += kBK) {
    if (ascale) ca.scale_k(ascale, k0);
    if constexpr (NEG) ca.negate();
    __syncthreads();  // previous chunk fully consumed
    ca.store(la);
    cb.store(lb);
    __syncthreads();
    if (k0 + kBK < kend) {
      ca.load(A, lda, k0 + kBK);
      cb.load(B, ldb, k0 + kBK);
    }
    mma_chunk<AK, BKc>(la, lb, f);
  }
}

// acc = C tile (row-major, ld) -- accumulate-into-C GEMMs start from the old tile.
__device__ inline void frag_load(Frag& f, const float* __restrict__ C, int64_t ld) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w >> 1) * 64, wn = (w & 1) * 64;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int col = wn + b * 32 + (lane & 31);
        f.acc[a][b][r] = C[(int64_t)row * ld + col];
      }
}

// Visit every accumulator element: fn(row, col, value) with row/col in [0,128).
template <typename Fn>
__device__ inline void frag_foreach(const Frag& f, Fn fn) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w >> 1) * 64, wn = (w & 1) * 64;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int col = wn + b * 32 + (lane & 31);
        fn(row, col, f.acc[a][b][r]);
      }
}

}  // namespace lvae
