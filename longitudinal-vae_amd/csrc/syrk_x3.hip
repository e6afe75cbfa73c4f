// syrk_x3.hip -- S = K^-1 V K^-1 (lower tiles) for the exact-KL backward, the step's largest GEMM,
// on the f16 matrix cores with the fp32-accurate 3-product split (see mfma_x3.hpp for the error
// argument), specialised for throughput:
//
//   split : B = 256 K^-1 diag(sqrt v) is split ONCE into fp16 hi / lo planes (B = hi + lo; the
//           generic x3 tile GEMM re-splits every operand chunk for every output tile);
//   syrk  : 256 x 256 output tiles, 512 threads = 8 waves (2 along M x 4 along N, 128 x 64 each,
//           4 x 2 blocks of v_mfma_f32_32x32x16_f16, three products per block and k-step);
//           operands staged global -> LDS directly (global_load_lds_dwordx4, no VGPR round trip)
//           into two LDS buffers: one raw s_barrier per K-chunk, after which the next chunk's DMA
//           is issued into the buffer just released and runs under the current chunk's MFMAs.
//
// LDS image of one operand part and chunk: [256 rows][32 halves] (64 B rows), 16-B chunk c of
// row r stored at chunk c ^ ((r >> 2) & 3): a ds_read_b128 phase (16 lanes = 16 consecutive rows,
// one logical chunk) then touches 16 distinct 16-B bank groups.  The swizzle is applied on the
// per-lane GLOBAL address of the DMA (its LDS side is lane-linear).
//
// Blocks are remapped so that each XCD (blockIdx % 8) works through a contiguous range of tiles
// of one latent dim: neighbouring tiles share 256-row panels in that XCD's L2.
#include "common.hpp"

namespace lvae {

typedef _Float16 sx_half8 __attribute__((ext_vector_type(8)));
typedef _Float16 sx_half4 __attribute__((ext_vector_type(4)));
typedef float sx_f32x16 __attribute__((ext_vector_type(16)));
typedef float sx_f32x4 __attribute__((ext_vector_type(4)));

constexpr int kSxT = 256;                // output tile edge
constexpr int kSxBK = 32;                // K chunk (halves) per LDS stage
constexpr int kSxPart = kSxT * kSxBK;    // halves per operand part per stage (16 KB)
constexpr float kSxScale = 256.0f;
constexpr float kSxUnscale = 1.0f / 65536.0f;

// hi / lo planes of B = 256 K^-1 diag(sqrt v): 4 elements per thread
__global__ __launch_bounds__(256) void syrk_split_kernel(const float* __restrict__ Kinv, const float* __restrict__ v,
                                                         _Float16* __restrict__ Bh, _Float16* __restrict__ Bl,
                                                         int np_, int64_t n4) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n4) return;
  const int64_t i0 = e * 4;
  const int64_t per = (int64_t)np_ * np_;
  const int l = (int)(i0 / per);
  const int k = (int)(i0 % np_);
  const sx_f32x4 x = *reinterpret_cast<const sx_f32x4*>(Kinv + i0);
  const sx_f32x4 s = *reinterpret_cast<const sx_f32x4*>(v + (int64_t)l * np_ + k);
  sx_half4 h, lo;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float y = x[q] * sqrtf(s[q]) * kSxScale;
    const _Float16 hh = (_Float16)y;
    h[q] = hh;
    lo[q] = (_Float16)(y - (float)hh);
  }
  *reinterpret_cast<sx_half4*>(Bh + i0) = h;
  *reinterpret_cast<sx_half4*>(Bl + i0) = lo;
}

__device__ inline void sx_tri(int t, int& I, int& J) {
  int r = (int)((sqrtf(8.0f * (float)t + 1.0f) - 1.0f) * 0.5f);
  while ((r + 1) * (r + 2) / 2 <= t) ++r;
  while (r * (r + 1) / 2 > t) --r;
  I = r;
  J = t - r * (r + 1) / 2;
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

__global__ __launch_bounds__(512) void syrk_x3_kernel(const _Float16* __restrict__ Bh, const _Float16* __restrict__ Bl,
                                                      float* __restrict__ S, int np_, int ntl, int nwg) {
  __shared__ __attribute__((aligned(16))) _Float16 lds[2 * 4 * kSxPart];  // 128 KB, the only LDS object
  // XCD-contiguous remap (bijective): blocks sharing blockIdx % 8 take a contiguous wgid range
  const int orig = blockIdx.x, xcd = orig % 8, q8 = nwg / 8, r8 = nwg % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int l = wgid / ntl;
  int I, J;
  sx_tri(wgid % ntl, I, J);
  const int64_t ld = np_;
  const int64_t base = (int64_t)l * np_ * np_;
  const _Float16* ah = Bh + base + (int64_t)I * kSxT * ld;
  const _Float16* al = Bl + base + (int64_t)I * kSxT * ld;
  const _Float16* bh = Bh + base + (int64_t)J * kSxT * ld;
  const _Float16* bl = Bl + base + (int64_t)J * kSxT * ld;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w >> 2) * 128, wn = (w & 3) * 64;
  const int r32 = lane & 31, kh = lane >> 5;

  sx_f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;

  const int nk = np_ / kSxBK;
  sx_issue(ah, al, bh, bl, ld, 0, lds);
  for (int s = 0; s < nk; ++s) {
    // one barrier per K-chunk: it retires stage s (every wave waited for its own DMA of it) and
    // every wave's reads of stage s-1, whose buffer then receives stage s+1 while s is multiplied
    SX_WAIT_VM(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + 1 < nk) sx_issue(ah, al, bh, bl, ld, (s + 1) * kSxBK, lds + ((s + 1) & 1) * 4 * kSxPart);
    const _Float16* cur = lds + (s & 1) * 4 * kSxPart;
    const _Float16* pah = cur;
    const _Float16* pal = cur + kSxPart;
    const _Float16* pbh = cur + 2 * kSxPart;
    const _Float16* pbl = cur + 3 * kSxPart;
    __builtin_amdgcn_s_setprio(1);
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
    __builtin_amdgcn_s_setprio(0);
  }
  // epilogue: C layout of 32x32 blocks -- row (e&3) + 8(e>>2) + 4(lane>>5), col lane&31
  float* C = S + base + (int64_t)(I * kSxT + wm) * ld + J * kSxT + wn;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = 32 * a + (e & 3) + 8 * (e >> 2) + 4 * kh, col = 32 * b + r32;
        C[(int64_t)row * ld + col] = acc[a][b][e] * kSxUnscale;
      }
}

// S (lower 256-tiles of [L, np, np] fp32) = K^-1 diag(v) K^-1; planes: 2 L np^2 halves of scratch.
int syrk_x3_f32(int np_, int L, const float* Kinv, const float* v, _Float16* planes, float* S, hipStream_t st) {
  if (np_ % kSxT) return -1;
  const int64_t per = (int64_t)np_ * np_, n4 = (int64_t)L * per / 4;
  _Float16* Bh = planes;
  _Float16* Bl = planes + (int64_t)L * per;
  syrk_split_kernel<<<cdiv(n4, 256), 256, 0, st>>>(Kinv, v, Bh, Bl, np_, n4);
  const int nt = np_ / kSxT, ntl = nt * (nt + 1) / 2, nwg = ntl * L;
  syrk_x3_kernel<<<nwg, 512, 0, st>>>(Bh, Bl, S, np_, ntl, nwg);
  LVAE_CHECK_LAUNCH();
  return 0;
}

}  // namespace lvae
