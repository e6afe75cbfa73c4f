// syrk_x3.hip -- S = K^-1 V K^-1 (lower tiles) for the exact-KL backward, the step's largest GEMM,
// on the f16 matrix cores with the fp32-accurate 3-product split (see mfma_x3.hpp for the error
// argument), specialised for throughput:
//
//   split : B = K^-1 diag(sqrt v) is split ONCE into fp16 hi / lo planes, with one power-of-two scale
//           per latent dim from a bound (ci_bscale_kernel), by the forward's lauum epilogue (which holds
//           the K^-1 tiles in registers anyway: chol_inv.hip, kCiLauumKL); the epilogue divides by its
//           square (the generic x3 tile GEMM would re-split every operand chunk for every output tile).  (r1-r2: one scale per row from a bound, written by a separate pass
//           over K^-1 -- syrk_x3_kernel below, kept for the dev A/B harness);
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
// of one latent dim, in the blocked order of sx_tri_blocked (row blocks of 4, inside a block by
// column): the 32 tiles an XCD runs at once form a 4 x 8 block sharing 4 A and 8 B panels in its L2
// (r3, scripts/gemm_ab.py: 3.19 vs 3.46 ms at np = 4096, L = 16 against the row-major order; 51.1 vs
// 55.9 ms at np = 16384, L = 4).
#include "x3_c16.hpp"

#ifndef LVAE_SYRK_RESERVE
#define LVAE_SYRK_RESERVE 0
#endif
#include "x3_dma.hpp"
#include "x3_gemm4.hpp"

namespace lvae {

template <int ORDER = 0>
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
  if constexpr (ORDER == 0)
    sx_tri(wgid % ntl, I, J);
  else
    sx_tri_blocked(wgid % ntl, np_ / kSxT, I, J);
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

// Variant: 256 x 128 half tiles, TWO independent 256-thread workgroups per CU (72 KB of LDS each),
// each 4 waves of 128 x 64 and a 3-stage ring of 16-deep K chunks (one in flight across each barrier):
// when one workgroup waits at its barrier the other one's MFMAs run.
constexpr int kH2BK = 16, kH2NS = 3;
constexpr int kH2A = 256 * kH2BK, kH2B = 128 * kH2BK;   // halves per A / B plane and stage
constexpr int kH2Stage = 2 * kH2A + 2 * kH2B;          // 24 KB
__device__ inline void h2_issue(const _Float16* __restrict__ ah, const _Float16* __restrict__ al,
                                const _Float16* __restrict__ bh, const _Float16* __restrict__ bl, int64_t ld, int k0,
                                _Float16* __restrict__ stage) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // 24 wave-instructions of 32 rows x 2 chunks: A hi / lo 8 each, B hi / lo 4 each; wave w takes 6
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    const int ins = 6 * w + q;
    const _Float16* src;
    _Float16* dst;
    int blk;
    if (ins < 16) {
      src = ins < 8 ? ah : al;
      blk = ins & 7;
      dst = stage + (ins < 8 ? 0 : kH2A);
    } else {
      src = ins < 20 ? bh : bl;
      blk = (ins - 16) & 3;
      dst = stage + 2 * kH2A + (ins < 20 ? 0 : kH2B);
    }
    const int row = 32 * blk + (lane >> 1);
    const int c = (lane & 1) ^ ((row >> 3) & 1);
    __builtin_amdgcn_global_load_lds((const void*)(src + (int64_t)row * ld + k0 + 8 * c), (void*)(dst + blk * 512), 16,
                                     0, 0);
  }
}

__global__ __launch_bounds__(256, 2) void syrk_h2_kernel(const _Float16* __restrict__ Bh, const _Float16* __restrict__ Bl,
                                                         const float* __restrict__ rsc, float* __restrict__ S, int np_,
                                                         int nth, int nwg, int L) {
  __shared__ __attribute__((aligned(16))) _Float16 lds[kH2NS * kH2Stage];  // 72 KB, the only LDS object
  const int orig = blockIdx.x, xcd = orig % 8, q8 = nwg / 8, r8 = nwg % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int l = wgid / nth, t = wgid % nth;
  // half tiles (I, J2), J2 <= 2 I + 1, in blocks of 4 tile rows (all half columns of a row block first)
  int I, J2;
  {
    int r, c;
    sx_tri(t >> 1, r, c);  // whole-tile lower index, two halves each
    I = r;
    J2 = 2 * c + (t & 1);
  }
  const int ld = np_;
  const int64_t base = (int64_t)l * np_ * np_;
  const _Float16* ah = Bh + base + (int64_t)I * 256 * ld;
  const _Float16* al = Bl + base + (int64_t)I * 256 * ld;
  const _Float16* bh = Bh + base + (int64_t)J2 * 128 * ld;
  const _Float16* bl = Bl + base + (int64_t)J2 * 128 * ld;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w >> 1) * 128, wn = (w & 1) * 64;
  const int r32 = lane & 31, kh = lane >> 5;
  sx_f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = sx_f32x16{};
  const int nk = np_ / kH2BK;
  h2_issue(ah, al, bh, bl, ld, 0, lds);
  if (nk > 1) h2_issue(ah, al, bh, bl, ld, kH2BK, lds + kH2Stage);
  for (int s = 0; s < nk; ++s) {
    if (s + 1 < nk) __builtin_amdgcn_s_waitcnt(0x0F76);  // vmcnt(6): stage s landed, s + 1 in flight
    else __builtin_amdgcn_s_waitcnt(0x0F70);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + 2 < nk) h2_issue(ah, al, bh, bl, ld, (s + 2) * kH2BK, lds + ((s + 2) % kH2NS) * kH2Stage);
    const _Float16* cur = lds + (s % kH2NS) * kH2Stage;
    __builtin_amdgcn_s_setprio(1);
    sx_half8 bH[2], bL[2];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      bH[b] = g4_frag(cur + 2 * kH2A, wn + 32 * b + r32, kh);
      bL[b] = g4_frag(cur + 2 * kH2A + kH2B, wn + 32 * b + r32, kh);
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const sx_half8 aH = g4_frag(cur, wm + 32 * a + r32, kh);
      const sx_half8 aL = g4_frag(cur + kH2A, wm + 32 * a + r32, kh);
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(aL, bH[b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(aH, bL[b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(aH, bH[b], acc[a][b], 0, 0, 0);
      }
    }
    __builtin_amdgcn_s_setprio(0);
  }
  const float* rs = rsc + (int64_t)l * np_;
  float* C = S + base + (int64_t)(I * 256 + wm) * ld + J2 * 128 + wn;
  float icol[2];
#pragma unroll
  for (int b = 0; b < 2; ++b) icol[b] = 1.0f / rs[J2 * 128 + wn + 32 * b + r32];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int row = 32 * a + (e & 3) + 8 * (e >> 2) + 4 * kh;
      const float irow = 1.0f / rs[I * 256 + wm + row];
#pragma unroll
      for (int b = 0; b < 2; ++b) C[(int64_t)row * ld + 32 * b + r32] = acc[a][b][e] * (irow * icol[b]);
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

// The product S GEMM: B's planes split with ONE power-of-two scale per latent dim, bsc[l] (written by the
// exact KL's lauum epilogue, chol_inv.hip), so S = acc / bsc[l]^2.  (Per-tile scales with the
// accumulators rescaled at every K block cost 10% here, scripts/gemm_ab.py.  So did the 8-wave core with
// 16-deep chunks in a 4-stage ring, two chunks in flight across each barrier: 3.55 vs 3.18 ms at
// np = 4096, L = 16 and 87 vs 51 ms at np = 16384, L = 4 -- its 32-B row segments per chunk double the
// L2 traffic.)  Same tile order and K split.
__global__ __launch_bounds__(512) void syrk_tiles_kernel(const _Float16* __restrict__ Bh, const _Float16* __restrict__ Bl,
                                                         const float* __restrict__ bsc, float* __restrict__ S,
                                                         float* __restrict__ Sx, int np_, int ntl, int nwg, int L, int ns) {
  __shared__ __attribute__((aligned(16))) _Float16 lds[2 * 4 * kSxPart];
  const int orig = blockIdx.x, xcd = orig % 8, q8 = nwg / 8, r8 = nwg % 8;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int sp = wgid / (ntl * L), l = (wgid / ntl) % L, nt = np_ / kSxT;
  int I, J;
  sx_tri_blocked(wgid % ntl, nt, I, J);
  const int kb0 = sp * nt / ns, kb1 = (sp + 1) * nt / ns;
  const int64_t ld = np_;
  const int64_t base = (int64_t)l * np_ * np_, k0 = (int64_t)kb0 * kSxT;
  sx_f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = sx_f32x16{};
  if (kb1 > kb0)
    sx_gemm(Bh + base + (int64_t)I * kSxT * ld + k0, Bl + base + (int64_t)I * kSxT * ld + k0,
            Bh + base + (int64_t)J * kSxT * ld + k0, Bl + base + (int64_t)J * kSxT * ld + k0, ld, (kb1 - kb0) * kSxT,
            lds, acc);
  const float sc = bsc[l], inv = 1.0f / (sc * sc);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float* C = (sp == 0 ? S : Sx + (int64_t)(sp - 1) * L * np_ * np_) + base + (int64_t)I * kSxT * ld + J * kSxT;
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(C, (short)0, 0x7fffffff, 0x00020000);
  const int vo = (((w >> 2) * 128 + 4 * (lane >> 5)) * np_ + (w & 3) * 64 + (lane & 31)) * 4;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int e = 0; e < 16; ++e)
#pragma unroll
      for (int b = 0; b < 2; ++b)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[a][b][e] * inv), rc, vo,
                                              ((32 * a + (e & 3) + 8 * (e >> 2)) * np_ + 32 * b) * 4, 0);
}

// The S GEMM on the chunk-major planes (x3_c16.hpp): NS-stage ring of 16-deep chunks, fragments of the
// next chunk read under the current chunk's MFMAs.  Same tile order, K split and epilogue as
// syrk_tiles_kernel.
template <int NS>
__global__ __launch_bounds__(512) void syrk_c16_kernel(const _Float16* __restrict__ Bh, const _Float16* __restrict__ Bl,
                                                       const float* __restrict__ bsc, float* __restrict__ S,
                                                       float* __restrict__ Sx, int np_, int ntl, int nwg, int L, int ns,
                                                       const int* __restrict__ skip) {
  __shared__ __attribute__((aligned(16))) _Float16 lds[NS * kC16Stage];
  if (skip && *skip) return;  // (uniform) the binned hyper-gradient needs no S (kl_hyper.hip)
  // tiles v = blockIdx.x, + gridDim.x, ...: one each with the full grid (nwg workgroups); a grid of fewer
  // (a multiple of 8: v keeps its blockIdx's XCD) leaves CUs to the ConvVAE stream (syrk_tiles_f32)
  for (int v = blockIdx.x; v < nwg; v += gridDim.x) {
    if (v != (int)blockIdx.x) __syncthreads();  // every wave's reads of the previous tile's stages are done
    const int orig = v, xcd = orig % 8, q8 = nwg / 8, r8 = nwg % 8;
    const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
    const int sp = wgid / (ntl * L), l = (wgid / ntl) % L, nt = np_ / kSxT;
    int I, J;
    sx_tri_blocked(wgid % ntl, nt, I, J);
    const int kb0 = sp * nt / ns, kb1 = (sp + 1) * nt / ns;
    const int64_t ld = np_;
    const int64_t base = (int64_t)l * np_ * np_, c0 = (int64_t)kb0 * (kSxT / kC16BK) * kC16Part;
    sx_f32x16 acc[4][2];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) acc[a][b] = sx_f32x16{};
    if (kb1 > kb0) {
      const int64_t pa = c16_panel(l, np_, I) + c0, pb = c16_panel(l, np_, J) + c0;
      c16_gemm<NS>(C16Opnd{Bh + pa, Bl - Bh, 0}, C16Opnd{Bh + pb, Bl - Bh, 0}, (kb1 - kb0) * (kSxT / kC16BK), lds, acc);
    }
    const float sc = bsc[l], inv = 1.0f / (sc * sc);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float* C = (sp == 0 ? S : Sx + (int64_t)(sp - 1) * L * np_ * np_) + base + (int64_t)I * kSxT * ld + J * kSxT;
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(C, (short)0, 0x7fffffff, 0x00020000);
    const int vo = (((w >> 2) * 128 + 4 * (lane >> 5)) * np_ + (w & 3) * 64 + (lane & 31)) * 4;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int e = 0; e < 16; ++e)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[a][b][e] * inv), rc, vo,
                                                ((32 * a + (e & 3) + 8 * (e >> 2)) * np_ + 32 * b) * 4, 0);
  }
}

// CUs the S GEMM leaves free when its tiles outnumber the chip (LVAE_SYRK_RESERVE, default below): the
// exact KL's backward runs the S GEMM on the caller's stream while the encoder backward runs on the ConvVAE
// stream; with one 160 KB-LDS workgroup on every CU those small kernels wait for whole S-GEMM tiles
static int syrk_grid(int nwg) {
  static int cus = -1;
  if (cus < 0) {
    int dev = 0;
    hipDeviceProp_t pr;
    cus = (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&pr, dev) == hipSuccess) ? pr.multiProcessorCount
                                                                                                : 256;
  }
  static const int reserve = getenv("LVAE_SYRK_RESERVE") ? atoi(getenv("LVAE_SYRK_RESERVE")) : LVAE_SYRK_RESERVE;
  if (reserve <= 0 || nwg <= cus) return nwg;
  const int g = (cus - reserve) / 8 * 8;
  return g >= 8 ? g : nwg;
}

int syrk_tiles_f32(int np_, int L, const float* bsc, const _Float16* planes, float* S, float* Sx, hipStream_t st,
                   const int* skip) {
  if (np_ % kSxT) return -1;
  const int64_t per = (int64_t)np_ * np_;
  const int ns = syrk_x3_splits(np_, L);
  if (ns > 1 && !Sx) return -2;
  const int nt = np_ / kSxT, ntl = nt * (nt + 1) / 2, nwg = ntl * L * ns;
  if (kCiBC16)
    syrk_c16_kernel<kC16NS><<<syrk_grid(nwg), 512, 0, st>>>(planes, planes + (int64_t)L * per, bsc, S, Sx, np_, ntl,
                                                            nwg, L, ns, skip);
  else
    syrk_tiles_kernel<<<nwg, 512, 0, st>>>(planes, planes + (int64_t)L * per, bsc, S, Sx, np_, ntl, nwg, L, ns);
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
    syrk_x3_kernel<0><<<nwg, 512, 0, st>>>(planes, planes + (int64_t)L * per, rsc, S, nullptr, np_, ntl, nwg, L, np_);
  else if (variant == 2)
    syrk_x3_kernel<1><<<nwg, 512, 0, st>>>(planes, planes + (int64_t)L * per, rsc, S, nullptr, np_, ntl, nwg, L, np_);
  else if (variant == 4)  // the product kernel (rsc[l * np] read as the dims' scales: ones)
    syrk_tiles_kernel<<<nwg, 512, 0, st>>>(planes, planes + (int64_t)L * per, rsc, S, nullptr, np_, ntl, nwg, L, 1);
  else if (variant == 5)  // chunk-major planes (x3_c16.hpp), 4-stage ring
    syrk_c16_kernel<4><<<nwg, 512, 0, st>>>(planes, planes + (int64_t)L * per, rsc, S, nullptr, np_, ntl, nwg, L, 1,
                                            nullptr);
  else if (variant == 6)  // chunk-major planes, 5-stage ring (all 160 KB of LDS)
    syrk_c16_kernel<5><<<nwg, 512, 0, st>>>(planes, planes + (int64_t)L * per, rsc, S, nullptr, np_, ntl, nwg, L, 1,
                                            nullptr);
  else if (variant == 3)
    syrk_h2_kernel<<<2 * nwg, 256, 0, st>>>(planes, planes + (int64_t)L * per, rsc, S, np_, 2 * ntl, 2 * nwg, L);
  else
    syrk_x4_kernel<<<nwg, 256, 0, st>>>(planes, planes + (int64_t)L * per, rsc, S, nullptr, np_, ntl, nwg, L, np_);
  LVAE_CHECK_LAUNCH();
  return 0;
}

}  // namespace lvae

extern "C" int lvae_dev_syrk(int variant, int np_, int L, const float* rsc, const void* planes, float* S, void* stream) {
  return lvae::syrk_dev_variant(variant, np_, L, rsc, (const _Float16*)planes, S, (hipStream_t)stream);
}
