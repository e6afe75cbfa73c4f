// syrk_x3.hip -- S = K^-1 V K^-1 (lower tiles) for the exact-KL backward, the step's largest GEMM,
// on the f16 matrix cores with the fp32-accurate 3-product split (see mfma_x3.hpp for the error
// argument), specialised for throughput:
//
//   split : row i of B = K^-1 diag(sqrt v), times sc_i = x3_scale(bound on max_j |B_ij|), is split
//           ONCE into fp16 hi / lo planes by the forward's kl_alpha_kernel (which reads K^-1 anyway); the
//           epilogue divides by sc_i sc_j (the generic x3 tile GEMM would re-split every operand
//           chunk for every output tile);
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
// of one latent dim: neighbouring tiles share 256-row panels in that XCD's L2.  (The blocked order
// of the sweep's update measured 10% slower here: with K = 4096 the panels stream through L2.)
#include "x3_dma.hpp"
#include "x3_gemm4.hpp"

namespace lvae {

__global__ __launch_bounds__(512) void syrk_x3_kernel(const _Float16* __restrict__ Bh, const _Float16* __restrict__ Bl,
                                                      const float* __restrict__ rsc, float* __restrict__ S,
                                                      float* __restrict__ Sx, int np_, int ntl, int nwg, int L,
                                                      int kspan) {
  __shared__ __attribute__((aligned(16))) _Float16 lds[2 * 4 * kSxPart];  // 128 KB, the only LDS object
  // XCD-contiguous remap (bijective): blocks sharing blockIdx % 8 take a contiguous wgid range
  const int orig = blockIdx.x, xcd = orig % 8, q8 = nwg / 8, r8 = nwg % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int sp = wgid / (ntl * L), l = (wgid / ntl) % L;  // K split, latent dim
  int I, J;
  sx_tri(wgid % ntl, I, J);
  const int64_t ld = np_;
  const int64_t base = (int64_t)l * np_ * np_, k0 = (int64_t)sp * kspan;
  const _Float16* ah = Bh + base + (int64_t)I * kSxT * ld + k0;
  const _Float16* al = Bl + base + (int64_t)I * kSxT * ld + k0;
  const _Float16* bh = Bh + base + (int64_t)J * kSxT * ld + k0;
  const _Float16* bl = Bl + base + (int64_t)J * kSxT * ld + k0;
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
  sx_gemm(ah, al, bh, bl, ld, kspan, lds, acc);
  // epilogue: C layout of 32x32 blocks -- row (e&3) + 8(e>>2) + 4(lane>>5), col lane&31
  // per-row split scales of B: S_ij = (B sc)_i (B sc)_j^T / (sc_i sc_j) (exact: powers of two)
  const float* rs = rsc + (int64_t)l * np_;
  float* C = (sp == 0 ? S : Sx + (int64_t)(sp - 1) * L * np_ * np_) + base + (int64_t)(I * kSxT + wm) * ld + J * kSxT + wn;
  float icol[2];
#pragma unroll
  for (int b = 0; b < 2; ++b) icol[b] = 1.0f / rs[J * kSxT + wn + 32 * b + r32];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int row = 32 * a + (e & 3) + 8 * (e >> 2) + 4 * kh;
      const float irow = 1.0f / rs[I * kSxT + wm + row];
#pragma unroll
      for (int b = 0; b < 2; ++b) C[(int64_t)row * ld + 32 * b + r32] = acc[a][b][e] * (irow * icol[b]);
    }
}

// The same S tiles on the 4-wave, 4-stage core (x3_gemm4.hpp): 256 threads, one wave per SIMD with
// 128 x 128 each, 16-deep K chunks with three in flight across every barrier.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void syrk_x4_kernel(
    const _Float16* __restrict__ Bh, const _Float16* __restrict__ Bl, const float* __restrict__ rsc, float* __restrict__ S,
    float* __restrict__ Sx, int np_, int ntl, int nwg, int L, int kspan) {
  __shared__ __attribute__((aligned(16))) _Float16 lds[kG4Lds];  // 128 KB, the only LDS object
  const int orig = blockIdx.x, xcd = orig % 8, q8 = nwg / 8, r8 = nwg % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int sp = wgid / (ntl * L), l = (wgid / ntl) % L;
  int I, J;
  sx_tri(wgid % ntl, I, J);
  const int64_t ld = np_;
  const int64_t base = (int64_t)l * np_ * np_, k0 = (int64_t)sp * kspan;
  const _Float16* ah = Bh + base + (int64_t)I * kG4T * ld + k0;
  const _Float16* al = Bl + base + (int64_t)I * kG4T * ld + k0;
  const _Float16* bh = Bh + base + (int64_t)J * kG4T * ld + k0;
  const _Float16* bl = Bl + base + (int64_t)J * kG4T * ld + k0;
  sx_f32x16 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = sx_f32x16{};
  g4_gemm(ah, al, bh, bl, ld, kspan, lds, acc, [](int, sx_f32x16(&)[4][4]) {});
  const float* rs = rsc + (int64_t)l * np_;
  float* C = (sp == 0 ? S : Sx + (int64_t)(sp - 1) * L * np_ * np_) + base + (int64_t)(I * kG4T) * ld + J * kG4T;
  float icol[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) icol[b] = 1.0f / rs[J * kG4T + g4_col(b)];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int row = g4_row(a, e);
      const float irow = 1.0f / rs[I * kG4T + row];
#pragma unroll
      for (int b = 0; b < 4; ++b) C[(int64_t)row * ld + g4_col(b)] = acc[a][b][e] * (irow * icol[b]);
    }
}

// K splits of the S GEMM: a 256-CU chip holds one 512-thread workgroup per CU (128 KB of LDS), so
// L * nt (nt + 1) / 2 tiles run in ceil(tiles / 256) rounds; with few latent dims per GPU (latent-dim
// sharding) the last round is mostly empty (L = 2: 272 tiles = 2 rounds for 1.06 rounds of work).
// Splitting K into s parts (partials summed by the Gram adjoint, which reads S anyway) runs
// ceil(s tiles / 256) rounds of 1/s the length, s in {2, 4}, taken only where the round count drops
// by more than 30%: a split pays its own prologue / epilogue and s-fold partial traffic (measured at
// np = 4096: L = 2 0.71 -> 0.60 ms with s = 4; L = 4 and L = 8 no gain or slower, L = 1 slower).
int syrk_x3_splits(int np_, int L) {
  const int nt = np_ / kSxT, tiles = L * nt * (nt + 1) / 2;
  auto cost = [&](int s) { return (double)((tiles * s + 255) / 256) / s; };
  int best = 1;
  for (int s : {2, 4})
    if (cost(s) < 0.7 * cost(best)) best = s;
  return best;
}

// S (lower 256-tiles of [L, np, np] fp32) = K^-1 diag(v) K^-1 from the fp16 hi / lo planes of
// B = K^-1 diag(sqrt v) (2 L np^2 halves: hi then lo), row i scaled by rsc[l][i] (kl_alpha_kernel).
// With s = syrk_x3_splits(np, L) > 1 the K-split partials go to S (split 0) and Sx[j - 1] (split j).
int syrk_x3_f32(int np_, int L, const float* rsc, const _Float16* planes, float* S, float* Sx, hipStream_t st) {
  if (np_ % kSxT) return -1;
  const int64_t per = (int64_t)np_ * np_;
  const _Float16* Bh = planes;
  const _Float16* Bl = planes + (int64_t)L * per;
  const int ns = syrk_x3_splits(np_, L);
  if (ns > 1 && !Sx) return -2;
  const int nt = np_ / kSxT, ntl = nt * (nt + 1) / 2, nwg = ntl * L * ns;
  syrk_x3_kernel<<<nwg, 512, 0, st>>>(Bh, Bl, rsc, S, Sx, np_, ntl, nwg, L, np_ / ns);
  LVAE_CHECK_LAUNCH();
  return 0;
}

// dev A/B (not in the C ABI): the S GEMM on the 8-wave 2-stage core (variant 0) or the 4-wave 4-stage
// core (variant 1), no K split
int syrk_dev_variant(int variant, int np_, int L, const float* rsc, const _Float16* planes, float* S, hipStream_t st) {
  if (np_ % kSxT) return -1;
  const int64_t per = (int64_t)np_ * np_;
  const int nt = np_ / kSxT, ntl = nt * (nt + 1) / 2, nwg = ntl * L;
  if (variant == 0)
    syrk_x3_kernel<<<nwg, 512, 0, st>>>(planes, planes + (int64_t)L * per, rsc, S, nullptr, np_, ntl, nwg, L, np_);
  else
    syrk_x4_kernel<<<nwg, 256, 0, st>>>(planes, planes + (int64_t)L * per, rsc, S, nullptr, np_, ntl, nwg, L, np_);
  LVAE_CHECK_LAUNCH();
  return 0;
}

}  // namespace lvae

extern "C" int lvae_dev_syrk(int variant, int np_, int L, const float* rsc, const void* planes, float* S, void* stream) {
  return lvae::syrk_dev_variant(variant, np_, L, rsc, (const _Float16*)planes, S, (hipStream_t)stream);
}
