// kl_hyper.hip -- the exact KL's hyper-parameter gradient WITHOUT S = K^-1 V K^-1 (r5).
//
// d KL / d theta_p = sum_ij G_ij dK_ij / d theta_p,  G = (K^-1 - S - alpha alpha^T) / 2  (elbo_functions.py:22-31
// under autograd).  The product route forms S with an N^3 GEMM (syrk_x3.hip, the step's largest kernel) and
// contracts G with the table adjoint (gram.hip).  For the table family of kernels (every component Cat / Bin
// gates times at most one RBF / periodic factor of an integer-coded covariate -- the reference's whole
// generate_kernel_batched family on integer covariates, GP_model.py:146-236) neither is needed:
//
//   FAR components (no gate on the "big" covariate, e.g. the subject id): dK_ij / d theta depends on the pair only
//   through the bins b(i), b(j), b = (the component's gate covariates' values, the value of its distance dim), so
//       sum_ij X_ij F(b_i, b_j) = sum_bb' F[b][b'] (Phi^T X Phi)[b][b']
//   with Phi the point -> bin indicator, and for the three parts of G
//       Phi^T K^-1 Phi = H Phi,   Phi^T S Phi = H V H^T,   Phi^T alpha alpha^T Phi = a a^T,
//       H = Phi^T K^-1 (bin sums of the rows of K^-1, nbins x N),  a = Phi^T alpha.
//   NEAR components (gated by the big covariate): only pairs inside one run of equal big values contribute,
//       and S's run blocks are X_run V X_run^T from the run's rows X_run of K^-1 (run length <= 64).
//
// So one streaming pass over K^-1 (column slabs of 64, the full symmetric matrix: the KL lauum writes the
// mirror instead of the S GEMM's operand planes) gives H, H V H^T (f64 MFMA) and H Phi per slab, and the near
// runs' X V X^T blocks (f32 MFMA) contracted at once with the derivative tables; a final kernel per latent dim
// adds the slabs in a fixed order (deterministic) and contracts the far part with the tables.  ~ N^2 bytes and
// O(N^2 (bins + run length)) flops per dim instead of the S GEMM's N^3 (CPU prototype: scripts/hyper_bins_proto.py,
// 4e-15 against autograd).  The results land in the table adjoint's per-workgroup slots, so kl_gram_bwd_reduce
// applies the same parameter constants.
//
// Conditions (hb_plan_kernel, on the device; otherwise `on` = 0 and the S GEMM + table adjoint run as before):
// the table path's (covariate flag 2); the Cat gate covariate of the widest range (> 4 values) is "big" (the id),
// the other Cat gates span <= 16 values; its values non-decreasing over the points (runs contiguous) with runs of
// <= 64 points; far binnings <= 4, with <= 128 bins in all, <= 4 blocks of 32 bins and sum nbins^2 <= 4096; <= 8
// parameter slots on near
// components; Bin gate values within 64 of their minimum, distance values within 65535 of theirs (the row keys);
// on the host: the slab kernel's LDS fits (hb_slab_lds).
#include "blkinv.hpp"
#include "gram_tab.hpp"
#include "prof.hpp"

namespace lvae {

constexpr int kHbMaxBin = 4;    // far binnings
constexpr int kHbBins = 128;    // far bins in all
constexpr int kHbBins2 = 4096;  // sum over binnings of nbins^2
constexpr int kHbRun = 64;      // longest run of the big covariate
constexpr int kHbSmall = 16;    // Cat gate covariates other than the big one span at most this many values
constexpr int kHbSmallest = 4;  // the big covariate spans more than this many values
constexpr int kHbNear = 4;      // parameter slots of the near components
constexpr int kHbBlk = 4;       // 32-bin blocks over the far binnings (two one-hot GEMM items per wave of four)
constexpr int kHbT = 64;        // row tile = column slab
constexpr int kHbTP = 68;       // LDS pitch of a tile row (floats: 16-B aligned rows, 16 rows on distinct banks)
constexpr int kHbNB = 24;       // 16 x 16 blocks of a slab's near window (runs ending in the slab: at most 24)
constexpr int kHbNQ = kHbNB / 4;  // near blocks per wave
// the per-(dim, slab) partial record (doubles): M [nb2], Q [nb2] (at kHbBins2), then the tail: the near slots' S
// parts, tr S, the near slots' K^-1 - alpha alpha^T parts (hb_near_kernel, record of row tile I), a = Phi^T alpha
constexpr int kHbNearS = 2 * kHbBins2;
constexpr int kHbNearK = kHbNearS + kHbNear + 1;
constexpr int kHbA = kHbNearK + kHbNear;
constexpr int kHbTail = 2 * kHbNear + 1 + kHbBins;
constexpr int kHbPart = 2 * kHbBins2 + kHbTail;

struct HbDev {
  int on, nbin, big, nbins, nb2, nnear;
  int gmin[kTabMaxBits], grng[kTabMaxBits];                  // gate bit: min value, number of values
  int wmin[kTabMaxG], wrng[kTabMaxG];                        // distance group: min value, number of values
  int bmask[kHbMaxBin], bgrp[kHbMaxBin], boff[kHbMaxBin], bn[kHbMaxBin], b2off[kHbMaxBin];  // far binnings
  int cbin[LVAE_MAX_COMP];                                   // component -> binning, -1: near
  int nslot[kHbNear];                                        // near parameter slots (GramTab porder index)
};

typedef unsigned hb_u32x4 __attribute__((ext_vector_type(4)));

struct HbWs {
  HbDev* dev;
  uint8_t* pbin;  // [kHbMaxBin][np] local bin of every point (255: padding)
  int* rs;        // [np] start of the point's run of the big covariate
  int* re;        // [np] its end (exclusive)
  double* part;   // [L][np / 64][kHbPart] per-slab partials
  float* tab;     // [L][kTabMaxBwdLds] the derivative tables per dim (hb_tab_kernel)
  hb_u32x4* rkey;    // [np] per point: gate values (6 bits each, the big gate's 0), distance values (16 bits each)
  double* hscr;      // [L][np / 64][kHbBins][64] the slab pass's H per workgroup (its epilogue's input)
  double* nscr;      // [L][np / 64][kHbNB][16][16] the slab pass's near S blocks per workgroup (likewise)
  size_t bytes;
  HbWs(char* base, int np_, int L) {
    size_t off = 0;
    auto take = [&](size_t b) {
      char* p = base ? base + off : nullptr;
      off += align256(b);
      return p;
    };
    dev = (HbDev*)take(sizeof(HbDev));
    pbin = (uint8_t*)take((size_t)kHbMaxBin * np_);
    rs = (int*)take((size_t)np_ * sizeof(int));
    re = (int*)take((size_t)np_ * sizeof(int));
    part = (double*)take((size_t)L * (np_ / kHbT) * kHbPart * sizeof(double));
    tab = (float*)take((size_t)L * kTabMaxBwdLds * sizeof(float));
    rkey = (hb_u32x4*)take((size_t)np_ * sizeof(hb_u32x4));
    hscr = (double*)take((size_t)L * (np_ / kHbT) * kHbBins * kHbT * sizeof(double));
    nscr = (double*)take((size_t)L * (np_ / kHbT) * kHbNB * 256 * sizeof(double));
    bytes = off;
  }
};
size_t kl_hyper_bytes(int np_, int L) { return HbWs(nullptr, np_, L).bytes; }
HbDev* kl_hyper_dev(void* base, int np_, int L) { return HbWs((char*)base, np_, L).dev; }

// ------------------------------------------------------------------------------------------
// the plan: one 1024-thread workgroup (x only; after the factor's covariate check)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void hb_plan_kernel(GramTab tb, const double* __restrict__ x, int ldx, int n,
                                                       int np_, const int* __restrict__ covflag, HbWs ws, int enable) {
  __shared__ int lo[kTabMaxBits + kTabMaxG], hi[kTabMaxBits + kTabMaxG];
  __shared__ int fail;
  __shared__ HbDev d;
  const int tid = threadIdx.x, nd = tb.nbits + tb.ng;
  if (*covflag != 2) {  // (uniform) not the table path
    if (tid == 0) ws.dev->on = 0;
    return;
  }
  if (tid < kTabMaxBits + kTabMaxG) {
    lo[tid] = INT_MAX;
    hi[tid] = INT_MIN;
  }
  if (tid == 0) fail = 0;
  __syncthreads();
  for (int q = 0; q < nd; ++q) {  // (uniform) the gate dims, then the distance dims
    const int dim = q < tb.nbits ? tb.bdim[q] : tb.gdim[q - tb.nbits];
    if (dim < 0) continue;
    int mn = INT_MAX, mx = INT_MIN;
    for (int i = tid; i < n; i += 1024) {
      const int v = (int)x[(int64_t)i * ldx + dim];  // (integer-coded: covariate flag 2)
      mn = min(mn, v);
      mx = max(mx, v);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      mn = min(mn, __shfl_xor(mn, o, 64));
      mx = max(mx, __shfl_xor(mx, o, 64));
    }
    if ((tid & 63) == 0) {
      atomicMin(&lo[q], mn);
      atomicMax(&hi[q], mx);
    }
  }
  __syncthreads();
  if (tid == 0) {
    HbDev p{};
    int f = 0;
    p.big = -1;
    for (int b = 0; b < tb.nbits; ++b) {  // big: the Cat gate covariate of the widest range (> kHbSmallest values)
      p.gmin[b] = lo[b];
      p.grng[b] = hi[b] - lo[b] + 1;
      if (tb.bkind[b] == LVAE_CAT && p.grng[b] > kHbSmallest && (p.big < 0 || p.grng[b] > p.grng[p.big])) p.big = b;
    }
    for (int b = 0; b < tb.nbits; ++b)  // a second wide Cat covariate would need bins of its own: not this route
      if (b != p.big && tb.bkind[b] == LVAE_CAT && p.grng[b] > kHbSmall) f = 1;
    for (int g = 0; g < tb.ng; ++g) {
      p.wmin[g] = tb.gdim[g] >= 0 ? lo[tb.nbits + g] : 0;
      p.wrng[g] = tb.gdim[g] >= 0 ? hi[tb.nbits + g] - lo[tb.nbits + g] + 1 : 1;
    }
    for (int r = 0; r < tb.n_comp; ++r) {
      p.cbin[r] = -1;
      if (p.big >= 0 && ((tb.cmask[r] >> p.big) & 1)) continue;  // near
      const int grp = tb.ckind[r] >= 0 ? tb.cgrp[r] : -1;
      int g = 0;
      while (g < p.nbin && !(p.bmask[g] == tb.cmask[r] && p.bgrp[g] == grp)) ++g;
      if (g == p.nbin) {
        if (p.nbin == kHbMaxBin) {
          f = 1;
          break;
        }
        long long nb = grp >= 0 ? p.wrng[grp] : 1;
        for (int b = 0; b < tb.nbits; ++b)
          if ((tb.cmask[r] >> b) & 1) nb *= p.grng[b];
        if (nb > kHbBins) {
          f = 1;
          break;
        }
        p.bmask[g] = tb.cmask[r];
        p.bgrp[g] = grp;
        p.bn[g] = (int)nb;
        p.boff[g] = p.nbins;
        p.b2off[g] = p.nb2;
        p.nbins += (int)nb;
        p.nb2 += (int)(nb * nb);
        ++p.nbin;
      }
      p.cbin[r] = g;
    }
    if (p.nbins > kHbBins || p.nb2 > kHbBins2) f = 1;
    {  // the slab pass's one-hot items: 32-bin blocks of every binning, at most kHbBlk
      int nblk = 0;
      for (int g = 0; g < p.nbin; ++g) nblk += (p.bn[g] + 31) / 32;
      if (nblk > kHbBlk) f = 1;
    }
    for (int k = 0; k < tb.pbeg[tb.ng] && !f; ++k)
      if (p.cbin[tb.pcomp[tb.porder[k]]] < 0) {
        if (p.nnear == kHbNear) f = 1;
        else p.nslot[p.nnear++] = k;
      }
    d = p;
    fail = f;
  }
  __syncthreads();
  // runs of the big covariate (non-decreasing, <= kHbRun points each) and every point's bins
  const int bd = d.big >= 0 ? tb.bdim[d.big] : -1;
  int bad = 0;
  for (int i = tid; i < np_; i += 1024) {
    int s = -1, e = -1;
    if (bd >= 0 && i < n) {
      const double v = x[(int64_t)i * ldx + bd];
      if (i > 0 && x[(int64_t)(i - 1) * ldx + bd] > v) bad = 1;
      s = i;
      while (s > 0 && i - s < kHbRun && x[(int64_t)(s - 1) * ldx + bd] == v) --s;
      e = i + 1;
      while (e < n && e - i < kHbRun && x[(int64_t)e * ldx + bd] == v) ++e;
      if (e - s > kHbRun || (s > 0 && x[(int64_t)(s - 1) * ldx + bd] == v) || (e < n && x[(int64_t)e * ldx + bd] == v))
        bad = 1;
    }
    ws.rs[i] = s;
    ws.re[i] = e;
    hb_u32x4 key = {0u, 0u, 0u, 0u};  // the near pairs' key: gate values (not the big one) and distance values
    if (i < n) {
      for (int b = 0; b < tb.nbits; ++b) {
        const int xv = (int)x[(int64_t)i * ldx + tb.bdim[b]], v = xv - d.gmin[b];
        if (b == d.big) continue;
        if (tb.bkind[b] == LVAE_CAT) {
          if (v < 0 || v > 63) bad = 1;
          key.x |= (unsigned)(v & 63) << (6 * b);
        } else {
          if (xv != 0 && xv != 1) bad = 1;  // (the Bin gate passes when both values are 1: x_i + x_j == 2)
          key.w |= (unsigned)(xv == 1) << b;
        }
      }
      for (int g = 0; g < tb.ng; ++g) {
        if (tb.gdim[g] < 0) continue;
        const int v = (int)x[(int64_t)i * ldx + tb.gdim[g]] - d.wmin[g];
        if (v < 0 || v > 65535) bad = 1;
        const unsigned u = (unsigned)(v & 0xffff);
        if (g == 0) key.y |= u;
        else if (g == 1) key.y |= u << 16;
        else key.z |= u;
      }
    }
    ws.rkey[i] = key;
    for (int g = 0; g < kHbMaxBin; ++g) {
      int idx = 255;
      if (g < d.nbin && i < n) {
        idx = 0;
        for (int b = 0; b < tb.nbits; ++b)
          if ((d.bmask[g] >> b) & 1) idx = idx * d.grng[b] + ((int)x[(int64_t)i * ldx + tb.bdim[b]] - d.gmin[b]);
        if (d.bgrp[g] >= 0) idx = idx * d.wrng[d.bgrp[g]] + ((int)x[(int64_t)i * ldx + tb.gdim[d.bgrp[g]]] - d.wmin[d.bgrp[g]]);
      }
      ws.pbin[(size_t)g * np_ + i] = (uint8_t)idx;
    }
  }
  if (__any(bad) && (tid & 63) == 0) atomicOr(&fail, 1);
  __syncthreads();
  if (tid == 0) {
    HbDev p = d;
    p.on = (!fail && enable) ? 1 : 0;
    *ws.dev = p;
  }
}


// the derivative tables of dim l once (entry per thread), for the slab and final kernels to copy
__global__ __launch_bounds__(256) void hb_tab_kernel(GramTab tb, HbWs ws, const double* __restrict__ params) {
  __shared__ float sp[64];
  const int tid = threadIdx.x, l = blockIdx.y, e = blockIdx.x * 256 + tid;
  if (!ws.dev->on) return;  // (uniform)
  if (tid < tb.n_params) sp[tid] = float(params[(int64_t)l * tb.n_params + tid]);
  __syncthreads();
  if (e < tb.pbeg[tb.ng] * (1 << tb.nbits) * kTabR) ws.tab[(int64_t)l * kTabMaxBwdLds + e] = tab_bwd_entry(tb, sp, e);
}

// a pair's code inside one run of the big covariate, from the two points' keys (hb_plan_kernel): the gate bits
// and the distance per distance group, [bits | d_0 << 8 | d_1 << 16 | d_2 << 24].  Branch-free: the Cat gates' 6-bit
// value fields are compared all at once (a field's OR lands on its low bit, the five low bits are gathered by one
// multiply: 2^(6b) * 2^(5 (4 - b)) = 2^(b + 20), no two products on one bit), the Bin gates pass where both keys
// hold a one (key.w, Bin values are 0 / 1); catbits = the Cat gates' bits
__device__ inline unsigned hb_pair_code(hb_u32x4 ki, hb_u32x4 kj, unsigned catbits, int ng) {
  const unsigned x = ki.x ^ kj.x, x1 = x | (x >> 1), x3 = x1 | (x1 >> 2), x5 = x3 | (x1 >> 4);
  const unsigned fail = (((x5 & 0x1041041u) * 0x108421u) >> 20) & 31u;  // Cat fields that differ
  unsigned c = (catbits & ~fail) | (ki.w & kj.w);
  const unsigned a0 = ki.y & 0xffffu, b0 = kj.y & 0xffffu, a1 = ki.y >> 16, b1 = kj.y >> 16;
  const unsigned a2 = ki.z & 0xffffu, b2 = kj.z & 0xffffu;
  const unsigned d0 = a0 > b0 ? a0 - b0 : b0 - a0, d1 = a1 > b1 ? a1 - b1 : b1 - a1, d2 = a2 > b2 ? a2 - b2 : b2 - a2;
  const unsigned cap = (unsigned)kTabD;  // (0 without a distance dim: both keys' field 0)
  c |= (d0 < cap ? d0 : cap) << 8;
  if (ng > 1) c |= (d1 < cap ? d1 : cap) << 16;
  if (ng > 2) c |= (d2 < cap ? d2 : cap) << 24;
  return c;
}

// the Cat gates' bits (uniform)
__device__ inline unsigned hb_catbits(const GramTab& tb) {
  unsigned m = 0;
#pragma unroll
  for (int b = 0; b < kTabMaxBits; ++b)
    if (b < tb.nbits && tb.bkind[b] == LVAE_CAT) m |= 1u << b;
  return m;
}

// the near slots' tables of dim l into LDS (slot after slot; hb_tab_kernel's) and each slot's distance group
__device__ inline void hb_near_tables(const GramTab& tb, const HbDev& d, const float* __restrict__ gt, int tstride,
                                      float* __restrict__ tab, int* __restrict__ sgrp) {
  const int tid = threadIdx.x;
  if (tid < d.nnear) sgrp[tid] = tb.cgrp[tb.pcomp[tb.porder[d.nslot[tid]]]];
  for (int e = tid; e < d.nnear * tstride; e += blockDim.x) tab[e] = gt[d.nslot[e / tstride] * tstride + e % tstride];
}

// a pair's table entry in near slot k (table base tk = k * tstride)
__device__ inline float hb_near_d(const float* tab, int tk, unsigned code, int grp) {
  return tab[tk + (int)(code & 0xffu) * kTabR + (int)((code >> (8 * (grp + 1))) & 0xffu)];
}

// ------------------------------------------------------------------------------------------
// the near runs' K^-1 and alpha alpha^T parts (no S): workgroup (I, l) takes the pairs of row tile I,
// record (l, I) gets sum over them of (K^-1_ij - alpha_i alpha_j) / 2 * D_k(i, j) per near slot k
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void hb_near_kernel(GramTab tb, HbWs ws, int n, int np_,
                                                      const float* __restrict__ Kinv, const double* __restrict__ alpha) {
  __shared__ HbDev d;
  __shared__ int sgrp[kHbNear];
  __shared__ double red[4][kHbNear];
  extern __shared__ float ntab[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, I = blockIdx.x, l = blockIdx.y, I0 = I * kHbT;
  if (tid == 0) d = *ws.dev;
  __syncthreads();
  if (!d.on) return;  // (uniform)
  const int tstride = (1 << tb.nbits) * kTabR, nnear = d.nnear;
  hb_near_tables(tb, d, ws.tab + (int64_t)l * kTabMaxBwdLds, tstride, ntab, sgrp);
  __syncthreads();
  const float* K = Kinv + (int64_t)l * np_ * np_;
  const double* al = alpha + (int64_t)l * np_;
  const unsigned catbits = hb_catbits(tb);
  double acc[kHbNear];
#pragma unroll
  for (int k = 0; k < kHbNear; ++k) acc[k] = 0.0;
  if (d.big >= 0) {
    for (int e = tid; e < kHbT * kHbRun; e += 256) {
      const int i = I0 + e / kHbRun, jj = e % kHbRun;
      if (i >= n) continue;
      const int s = ws.rs[i], len = ws.re[i] - s;
      if (jj >= len) continue;
      const int j = s + jj;
      const unsigned c = hb_pair_code(ws.rkey[i], ws.rkey[j], catbits, tb.ng);
      const double val = 0.5 * ((double)K[(int64_t)i * np_ + j] - al[i] * al[j]);
#pragma unroll
      for (int k = 0; k < kHbNear; ++k)
        if (k < nnear) acc[k] += val * (double)hb_near_d(ntab, k * tstride, c, sgrp[k]);
    }
  }
#pragma unroll
  for (int k = 0; k < kHbNear; ++k) {
    const double sk = wave_sum(acc[k]);
    if (lane == 0) red[w][k] = sk;
  }
  __syncthreads();
  if (tid < kHbNear)
    ws.part[((int64_t)l * (np_ / kHbT) + I) * kHbPart + kHbNearK + tid] =
        ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
}

// ------------------------------------------------------------------------------------------
// the slab pass: workgroup (J, l) streams column slab J (64 columns) of the full symmetric K^-1 of dim l, 64-row
// tile by tile, and writes its partial record: M_g = H_g V H_g^T, Q_g = H_g Phi_g (the slab's columns), the near
// runs' S parts per near slot, the slab's part of tr S and of a = Phi^T alpha.
//
// 256 threads and < 80 KB of LDS: two workgroups per CU, whose barriers and HBM round trips overlap.
//   tile store: every thread splits its 8 rows x 2 columns exactly into three bf16 pieces (round to nearest:
//     hi + mid + lo = the fp32 value) and writes each column's 8-row chunk of each piece as one 16-byte store into
//     column-major planes (chunks swizzled by the column: conflict-free 16-byte reads and writes), the fp32 tile
//     (x V^(1/2) of its ROWS, column-major) for the near runs, and its tr S part
//   H_g += Phi_g(tile)^T K^-1(tile, slab): one-hot GEMMs on v_mfma_f32_32x32x16_bf16, item = (32-bin block,
//     32-column block), two items per wave (the plan allows at most 4 blocks) held in the accumulators across
//     kHbFold tiles (products exact), then added to the workgroup's fp64 H in the workspace
//   near runs: the workgroup owns the runs ENDING in its columns; K^-1 is symmetric, so a run's S block
//     X_run V X_run^T = sum over all rows m of K^-1(m, run)^T v_m K^-1(m, run) accumulates from the column slab
//     itself, tile by tile: the 16 x 16 blocks of the run window's columns (the slab, plus the previous slab's
//     columns for a run that starts there, loaded in that case only) on v_mfma_f32_16x16x4f32 (k = 16 rows per
//     lane group: 16-byte LDS reads), in fp32 accumulators for kHbFold tiles, then added to fp64 blocks in the
//     workspace; the pair codes and table contraction run ONCE per pair in the epilogue, not per tile
// H and the near blocks reach the workspace by atomics without return (no wait; one lane per entry, so they
// apply in program order: deterministic).  The next tile arrives in registers under the current one's work
// (no branch around a load); the two workgroups of a CU cover each other's HBM round trips and barriers.
// ------------------------------------------------------------------------------------------

#ifdef LVAE_HB_STAMP  // (diagnostic builds only: per-section cycle stamps of the slab pass, printed by workgroup (0, 0))
#define HB_STAMP(t)                                                                   \
  do {                                                                                \
    __builtin_amdgcn_sched_barrier(0);                                                \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");       \
    __builtin_amdgcn_sched_barrier(0);                                                \
  } while (0)
#else
#define HB_STAMP(t) \
  do {              \
  } while (0)
#endif

typedef float hb_f32x2 __attribute__((ext_vector_type(2)));
typedef float hb_f32x4 __attribute__((ext_vector_type(4)));
typedef float hb_f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 hb_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 hb_bf16x2 __attribute__((ext_vector_type(2)));
constexpr int kHbSlabThreads = 256, kHbSlabWaves = kHbSlabThreads / 64;
#ifndef LVAE_HB_FOLD
#define LVAE_HB_FOLD 16
#endif
constexpr int kHbFold = LVAE_HB_FOLD;  // tiles summed in fp32 by the accumulators before the fp64 fold (power of 2)
#ifndef LVAE_HB_DEPTH
#define LVAE_HB_DEPTH 1
#endif
// K^-1 tiles in flight per workgroup (1, 2 or 4): deeper prefetch measured slower (r6, profiles/r6_slab_depth_ab.txt:
// 681 / 708 / 1894 us per launch at 1 / 2 / 4; the extra registers cost the second workgroup per CU at 4)
constexpr int kHbDepth = LVAE_HB_DEPTH;
static_assert(kHbDepth == 1 || kHbDepth == 2 || kHbDepth == 4, "nt = np / 64 is a multiple of 4");

struct HbPre {        // one tile's prefetch
  hb_f32x2 pk[8];     // K^-1 rows 8 (tid >> 5) + u, columns 2 (tid & 31) + 0, 1
  int pbn;            // wave w < nbin: bin of row lane in binning w
  hb_f32x4 vr[2];     // v of rows 8 (tid >> 5) + 0 .. 7 (the near runs' row weights)
};

__device__ inline unsigned hb_pk_bf16(float a, float b) {  // (round to nearest even: v_cvt_pk_bf16_f32)
  const hb_bf16x2 v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(unsigned, v);
}
__device__ inline float hb_bf_lo(unsigned u) { return __uint_as_float(u << 16); }
__device__ inline float hb_bf_hi(unsigned u) { return __uint_as_float(u & 0xffff0000u); }

// dword offset in a bf16 plane of (column c, 8-row chunk k): 32 dwords per column, chunks swizzled by (c >> 1) & 7
__device__ inline int hb_pl_off(int c, int k) { return c * 32 + ((k ^ ((c >> 1) & 7)) << 2); }

// three bf16 pieces of 8 fp32 values, packed by pairs (rows 2 k, 2 k + 1 in dword k)
__device__ inline void hb_split8(const float* a, hb_u32x4& hi, hb_u32x4& mid, hb_u32x4& lo) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float x0 = a[2 * k], x1 = a[2 * k + 1];
    const unsigned h = hb_pk_bf16(x0, x1);
    const float r0 = x0 - hb_bf_lo(h), r1 = x1 - hb_bf_hi(h);
    const unsigned m = hb_pk_bf16(r0, r1);
    const float s0 = r0 - hb_bf_lo(m), s1 = r1 - hb_bf_hi(m);
    hi[k] = h;
    mid[k] = m;
    lo[k] = hb_pk_bf16(s0, s1);
  }
}

__global__ __launch_bounds__(kHbSlabThreads, 2) void hb_slab_kernel(GramTab tb, HbWs ws, int n, int np_,
                                                                    const float* __restrict__ Kinv,
                                                                    const float* __restrict__ vv,
                                                                    const double* __restrict__ alpha, int dbg) {
  __shared__ HbDev d;
  // the near window's fp32 columns x V^(1/2) of the tile's rows, column-major [window column][row]: columns
  // 0 .. 63 the previous slab's (a run starting there only), 64 .. 127 this slab's
  __shared__ __attribute__((aligned(16))) float Tc[2 * kHbT * kHbTP];
  __shared__ __attribute__((aligned(16))) unsigned Pw[3][kHbT * 32];  // the current tile's bf16 planes, column-major
  __shared__ __attribute__((aligned(8))) uint8_t rbin[kHbMaxBin][kHbT];  // bins of the current tile's rows
  __shared__ uint8_t cbin[kHbMaxBin][kHbT];     // bins of the slab's columns
  __shared__ float vs[kHbT];                    // v of the slab's columns
  __shared__ double acol[kHbT];                 // alpha of the slab's columns
  __shared__ hb_u32x4 ckey[2 * kHbT];           // the near window's keys
  __shared__ int rstart[kHbT];                   // start of the run ending at the slab's column e
  __shared__ unsigned long long runends;        // bit e: a run ends at column J0 + e
  __shared__ int nblk, nspan;                    // near window: 16 x 16 blocks (lower), a run from the previous slab
  __shared__ uint8_t blist[kHbNB];               // block t: (bi << 3) | bj, bi >= bj (window column blocks)
  __shared__ int8_t blkid[64];                   // (bi << 3) | bj -> t
  __shared__ int sgrp[kHbNear];
  __shared__ int sbg[kHbBlk], sbb[kHbBlk], nbk;  // 32-bin blocks: binning, block index
  __shared__ double red[kHbSlabWaves][kHbNear + 1];
  extern __shared__ float tab[];                // the near slots' tables
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, J = blockIdx.x, l = blockIdx.y, J0 = J * kHbT;
  if (tid == 0) d = *ws.dev;
  __syncthreads();
  if (!d.on) return;  // (uniform)
  const int tstride = (1 << tb.nbits) * kTabR;
  if (tid < kHbT) {
    vs[tid] = vv[(int64_t)l * np_ + J0 + tid];
    acol[tid] = alpha[(int64_t)l * np_ + J0 + tid];
  }
  for (int e = tid; e < d.nbin * kHbT; e += kHbSlabThreads)
    cbin[e / kHbT][e % kHbT] = ws.pbin[(size_t)(e / kHbT) * np_ + J0 + e % kHbT];
  hb_near_tables(tb, d, ws.tab + (int64_t)l * kTabMaxBwdLds, tstride, tab, sgrp);
  if (tid < 2 * kHbT) {  // the near window's keys (columns J0 - 64 .. J0 + 63)
    const int c = J0 - kHbT + tid;
    ckey[tid] = c >= 0 ? ws.rkey[c] : hb_u32x4{0u, 0u, 0u, 0u};
  }
  if (w == 0) {
    // the runs ending in the slab's columns (lane e: column J0 + e) and the lower 16 x 16 blocks of the window
    // their pairs touch: a run [s, c] (<= 64 points) covers window column blocks (s - J0 + 64) / 16 .. (c - J0 +
    // 64) / 16; at most one run starts in the previous slab, so the union holds at most 15 + 10 - 1 = 24 blocks
    const int c = J0 + lane;
    const bool isend = d.big >= 0 && c < n && ws.re[c] == c + 1;
    const int s0 = isend ? ws.rs[c] : c;
    rstart[lane] = s0;
    const int ba = (s0 - J0 + kHbT) >> 4, bz = (c - J0 + kHbT) >> 4;
    unsigned long long m = 0;
    if (isend)
      for (int bi = ba; bi <= bz; ++bi)
        for (int bj = ba; bj <= bi; ++bj) m |= 1ull << (bi * 8 + bj);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const unsigned lo = __shfl_xor((unsigned)m, o, 64), hi = __shfl_xor((unsigned)(m >> 32), o, 64);
      m |= ((unsigned long long)hi << 32) | lo;
    }
    const unsigned long long ends = __ballot(isend), sp = __ballot(isend && s0 < J0);
    if (lane == 0) {
      runends = ends;
      nspan = sp != 0;
      int t = 0;
      for (int b = 0; b < 64; ++b) {
        blkid[b] = -1;
        if (((m >> b) & 1ull) && t < kHbNB) {
          blkid[b] = (int8_t)t;
          blist[t++] = (uint8_t)b;
        }
      }
      nblk = t;
    }
  }
  if (tid == 0) {  // the 32-bin blocks of the binnings in order (the plan keeps them <= kHbBlk)
    int t = 0;
    for (int g = 0; g < d.nbin; ++g)
      for (int bb = 0; bb * 32 < d.bn[g] && t < kHbBlk; ++bb, ++t) {
        sbg[t] = g;
        sbb[t] = bb;
      }
    nbk = t;
  }
  __syncthreads();
  const float* K = Kinv + (int64_t)l * np_ * np_;
  const int nbin = d.nbin, nnear = d.nnear, nitem = 2 * nbk, nbl = nblk, span = nspan;
  const unsigned catbits = hb_catbits(tb);
  // H items (item = 2 block + column block): wave w takes w and w + 4, both of column block w & 1
  const int cb = w & 1, hh = lane >> 5, col = 32 * cb + (lane & 31);
  const int i0 = w, i1 = w + kHbSlabWaves;
  const bool it0 = i0 < nitem, it1 = i1 < nitem;
  int g0 = 0, b00 = 0, g1 = 0, b01 = 0;
  if (it0) {
    g0 = sbg[i0 >> 1];
    b00 = 32 * sbb[i0 >> 1];
  }
  if (it1) {
    g1 = sbg[i1 >> 1];
    b01 = 32 * sbb[i1 >> 1];
  }
  hb_f32x16 acc0 = {}, acc1 = {};
  // H lives in the workgroup's scratch (fp64): the accumulators are added to it every kHbFold tiles by atomics
  // without return (no wait; one lane per entry, so the adds apply in program order: deterministic), the first
  // fold storing
  double* Hs = ws.hscr + ((int64_t)l * (np_ / kHbT) + J) * kHbBins * kHbT;
  // the near blocks likewise: wave w takes blocks w + 4 q (q < kHbNQ), [t][16 rows][16 columns] in the scratch
  double* Ns = ws.nscr + ((int64_t)l * (np_ / kHbT) + J) * kHbNB * 256;
  const int li = lane & 15, lk = lane >> 4;
  bi_f32x4 nac[kHbNQ];
#pragma unroll
  for (int q = 0; q < kHbNQ; ++q) nac[q] = bi_f32x4{0.f, 0.f, 0.f, 0.f};
  double tS = 0.0;
  const int cp = tid & 31, i8 = tid >> 5;  // this thread's tile part: columns 2 cp + 0, 1; rows 8 i8 + 0..7
  const float v0 = vs[2 * cp], v1 = vs[2 * cp + 1], r0 = sqrtf(v0), r1 = sqrtf(v1);  // (v = exp(log var) > 0)
  const int nt = np_ / kHbT;

  auto fetch = [&](int I, HbPre& p) {
    const int I0 = I * kHbT;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      p.pk[u] = __builtin_nontemporal_load(
          reinterpret_cast<const hb_f32x2*>(K + (int64_t)(I0 + 8 * i8 + u) * np_ + J0 + 2 * cp));
    p.pbn = (int)ws.pbin[(size_t)(w < nbin ? w : 0) * np_ + I0 + lane];  // (used by waves w < nbin only)
    const float* vr = vv + (int64_t)l * np_ + I0 + 8 * i8;
    p.vr[0] = *reinterpret_cast<const hb_f32x4*>(vr);
    p.vr[1] = *reinterpret_cast<const hb_f32x4*>(vr + 4);
  };

  auto fold = [&](hb_f32x16& acc, int g, int b0, bool first) {
    const int nb = d.bn[g];
    double* hc = Hs + (int64_t)d.boff[g] * kHbT + col;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int b = b0 + (e & 3) + 8 * (e >> 2) + 4 * hh;
      if (b < nb) {
        if (first) hc[b * kHbT] = (double)acc[e];
        else unsafeAtomicAdd(hc + b * kHbT, (double)acc[e]);
      }
      acc[e] = 0.f;
    }
  };

  auto body = [&](int I, HbPre& p) {
    const int I0 = I * kHbT;
    // the accumulators go to the fp64 scratch every kHbFold tiles and after the last (the first fold stores)
    const bool fold_now = (I & (kHbFold - 1)) == kHbFold - 1 || I == nt - 1, fold_first = I < kHbFold;
    {  // the tile into LDS: the bf16 planes, the near window's columns; the tr S part (sum_m v_m (K^-1_im)^2)
      float ts = 0.f;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float s0 = p.pk[u][0] * r0, s1 = p.pk[u][1] * r1;
        ts += s0 * s0 + s1 * s1;
      }
      tS += (double)ts;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        float a[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) a[u] = p.pk[u][c];
        hb_u32x4 hi, mid, lo;
        hb_split8(a, hi, mid, lo);
        const int off = hb_pl_off(2 * cp + c, i8);
        *reinterpret_cast<hb_u32x4*>(&Pw[0][off]) = hi;
        *reinterpret_cast<hb_u32x4*>(&Pw[1][off]) = mid;
        *reinterpret_cast<hb_u32x4*>(&Pw[2][off]) = lo;
      }
    }
    if (w < nbin) rbin[w][lane] = (uint8_t)p.pbn;
    if (nbl > 0) {  // (uniform) near runs end in the slab: its columns x v^(1/2) of the rows, column-major
      float sr[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) sr[u] = sqrtf(p.vr[u >> 2][u & 3]);
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        float* dst = &Tc[(kHbT + 2 * cp + c) * kHbTP + 8 * i8];
        *reinterpret_cast<hb_f32x4*>(dst) = hb_f32x4{p.pk[0][c] * sr[0], p.pk[1][c] * sr[1], p.pk[2][c] * sr[2],
                                                     p.pk[3][c] * sr[3]};
        *reinterpret_cast<hb_f32x4*>(dst + 4) = hb_f32x4{p.pk[4][c] * sr[4], p.pk[5][c] * sr[5],
                                                         p.pk[6][c] * sr[6], p.pk[7][c] * sr[7]};
      }
      if (span) {  // (uniform, rare) a run starts in the previous slab: its columns too
        hb_f32x2 q[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          q[u] = *reinterpret_cast<const hb_f32x2*>(K + (int64_t)(I0 + 8 * i8 + u) * np_ + J0 - kHbT + 2 * cp);
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          float* dst = &Tc[(2 * cp + c) * kHbTP + 8 * i8];
          *reinterpret_cast<hb_f32x4*>(dst) = hb_f32x4{q[0][c] * sr[0], q[1][c] * sr[1], q[2][c] * sr[2],
                                                       q[3][c] * sr[3]};
          *reinterpret_cast<hb_f32x4*>(dst + 4) = hb_f32x4{q[4][c] * sr[4], q[5][c] * sr[5], q[6][c] * sr[6],
                                                           q[7][c] * sr[7]};
        }
      }
    }
    __syncthreads();
    // (kHbDepth tiles ahead, in flight under this tile's work and the other workgroup's)
    fetch(I + kHbDepth < nt ? I + kHbDepth : nt - 1, p);
    if (!(dbg & 1) && it0) {
      auto onehot = [&](int g, int b0, int ks) {  // A operand: [bin b0 + (lane & 31)][rows 16 ks + 8 hh + 0..7]
        const unsigned mybin = (unsigned)(b0 + (lane & 31));
        const uint2 rb = *reinterpret_cast<const uint2*>(&rbin[g][16 * ks + 8 * hh]);
        hb_u32x4 a;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const unsigned wd = k < 2 ? rb.x : rb.y, sh = 16 * (k & 1);
          const unsigned lo_ = ((wd >> sh) & 0xffu) == mybin ? 0x3f80u : 0u;
          const unsigned hi_ = ((wd >> (sh + 8)) & 0xffu) == mybin ? 0x3f800000u : 0u;
          a[k] = lo_ | hi_;
        }
        return __builtin_bit_cast(hb_bf16x8, a);
      };
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        // B operands: column col, rows 16 ks + 8 hh + 0..7, the three pieces (shared by the wave's two items)
        const hb_bf16x8 bh = *reinterpret_cast<const hb_bf16x8*>(&Pw[0][hb_pl_off(col, 2 * ks + hh)]);
        const hb_bf16x8 bm = *reinterpret_cast<const hb_bf16x8*>(&Pw[1][hb_pl_off(col, 2 * ks + hh)]);
        const hb_bf16x8 bl = *reinterpret_cast<const hb_bf16x8*>(&Pw[2][hb_pl_off(col, 2 * ks + hh)]);
        const hb_bf16x8 a0 = onehot(g0, b00, ks);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bl, acc0, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bm, acc0, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bh, acc0, 0, 0, 0);
        if (it1) {
          const hb_bf16x8 a1 = onehot(g1, b01, ks);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, bl, acc1, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, bm, acc1, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, bh, acc1, 0, 0, 0);
        }
      }
      if (fold_now) {  // fold the accumulators into H (fp64, the scratch)
        fold(acc0, g0, b00, fold_first);
        if (it1) fold(acc1, g1, b01, fold_first);
      }
    }
    // near blocks: C[r][c] += sum over the tile's 64 rows m of Tc[16 bi + r][m] Tc[16 bj + c][m]; lane group lk
    // takes rows 16 lk .. 16 lk + 15 (the k slots of 16 MFMAs: any row order works when A and B share it)
    if (!(dbg & 2)) {
#pragma unroll
      for (int q = 0; q < kHbNQ; ++q) {
        const int t = w + kHbSlabWaves * q;
        if (t < nbl) {  // (uniform)
          const int bb = blist[t], bi = bb >> 3, bj = bb & 7;
          const float* pa = &Tc[(16 * bi + li) * kHbTP + 16 * lk];
          const float* pb = &Tc[(16 * bj + li) * kHbTP + 16 * lk];
          hb_f32x4 a4[4], b4[4];
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) {
            a4[s4] = *reinterpret_cast<const hb_f32x4*>(pa + 4 * s4);
            b4[s4] = *reinterpret_cast<const hb_f32x4*>(pb + 4 * s4);
          }
          bi_f32x4 x0 = {0.f, 0.f, 0.f, 0.f}, x1 = {0.f, 0.f, 0.f, 0.f};  // (two chains: half the dependency)
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) {
            x0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[s4][0], b4[s4][0], x0, 0, 0, 0);
            x1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[s4][1], b4[s4][1], x1, 0, 0, 0);
            x0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[s4][2], b4[s4][2], x0, 0, 0, 0);
            x1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[s4][3], b4[s4][3], x1, 0, 0, 0);
          }
          nac[q] += x0 + x1;
          if (fold_now) {  // fold into the fp64 blocks: element e = C[4 lk + e][li]
            double* nb = Ns + t * 256 + (4 * lk) * 16 + li;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              if (fold_first) nb[e * 16] = (double)nac[q][e];
              else unsafeAtomicAdd(nb + e * 16, (double)nac[q][e]);
            }
            nac[q] = bi_f32x4{0.f, 0.f, 0.f, 0.f};
          }
        }
      }
    }
    __syncthreads();  // every reader of the planes, the window columns and the bins done before the next store
  };

  // kHbDepth prefetch buffers in rotation (static names: the loop is unrolled by kHbDepth; nt = np / 64 is a
  // multiple of 4)
  HbPre pre[kHbDepth];
#pragma unroll
  for (int u = 0; u < kHbDepth; ++u) fetch(u, pre[u]);
  for (int I = 0; I < nt; I += kHbDepth) {
#pragma unroll
    for (int u = 0; u < kHbDepth; ++u) body(I + u, pre[u]);
  }
  // (the last tile folds too; the scratch's stores and atomics complete and visible to
  // the workgroup before its epilogue reads them)
  __builtin_amdgcn_s_waitcnt(0);  // (vmcnt / lgkmcnt / expcnt 0: this wave's stores and atomics done)
  __threadfence_block();
  __syncthreads();
  // Q_g[b][b'] = sum over the slab's columns m in bin b' of H_g[b][m]: thread (g, b) owns row b (LDS scratch = Tc);
  // a part: thread (g, b) sums alpha over the slab's columns in bin b
  double* Qs = reinterpret_cast<double*>(&Tc[0]);
  for (int e = tid; e < d.nb2; e += kHbSlabThreads) Qs[e] = 0.0;
  __syncthreads();
  double* out = ws.part + ((int64_t)l * nt + J) * kHbPart;
  for (int tb2 = tid; tb2 < d.nbins; tb2 += kHbSlabThreads) {
    int g = 0;
    while (g + 1 < nbin && tb2 >= d.boff[g + 1]) ++g;
    const int b = tb2 - d.boff[g], nb = d.bn[g];
    double* qrow = Qs + d.b2off[g] + b * nb;
    const double* hr = Hs + (int64_t)tb2 * kHbT;
    double as = 0.0;
    for (int m = 0; m < kHbT; ++m) {
      const int bc = cbin[g][m];
      if (bc != 255) qrow[bc] += hr[m];
      if (bc == b) as += acol[m];
    }
    out[kHbA + tb2] = as;
  }
  __syncthreads();
  for (int e = tid; e < d.nb2; e += kHbSlabThreads) out[kHbBins2 + e] = Qs[e];
  // M_g = H_g V H_g^T on v_mfma_f64_16x16x4f64: 16 x 16 blocks dealt to the waves
  for (int g = 0; g < nbin; ++g) {
    const int nb = d.bn[g], nb16 = (nb + 15) >> 4;
    for (int item = w; item < nb16 * nb16; item += kHbSlabWaves) {
      const int bi = item / nb16, bj = item % nb16, li = lane & 15, lk = lane >> 4;
      const int ba = 16 * bi + li, bb = 16 * bj + li;
      const double* ha = Hs + (int64_t)(d.boff[g] + (ba < nb ? ba : 0)) * kHbT;
      const double* hb = Hs + (int64_t)(d.boff[g] + (bb < nb ? bb : 0)) * kHbT;
      bi_f64x4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
      for (int s4 = 0; s4 < kHbT; s4 += 4) {
        const int m = s4 + lk;
        const double a = ba < nb ? ha[m] * (double)vs[m] : 0.0;
        const double b = bb < nb ? hb[m] : 0.0;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {  // C[lk + 4 q][li]
        const int r = 16 * bi + lk + 4 * q, c = 16 * bj + li;
        if (r < nb && c < nb) out[d.b2off[g] + r * nb + c] = acc[q];
      }
    }
  }
  // the near runs' pairs, once each: S_ij from the fp64 blocks, contracted with the near slots' tables through the
  // pair codes (the runs in column order, a run's len^2 ordered pairs dealt to the threads)
  double nacc[kHbNear];
#pragma unroll
  for (int k = 0; k < kHbNear; ++k) nacc[k] = 0.0;
  if (!(dbg & 2)) {
    for (unsigned long long rm = runends; rm; rm &= rm - 1) {
      const int e = __builtin_ctzll(rm), s0 = rstart[e], len = e + 1 - (s0 - J0);
      for (int pq = tid; pq < len * len; pq += kHbSlabThreads) {
        const int wi = s0 - J0 + kHbT + pq / len, wj = s0 - J0 + kHbT + pq % len;  // window columns
        const int lo_ = min(wi, wj), hi_ = max(wi, wj);
        const int t = blkid[((hi_ >> 4) << 3) | (lo_ >> 4)];
        const double sv = t >= 0 ? Ns[t * 256 + (hi_ & 15) * 16 + (lo_ & 15)] : 0.0;  // (t >= 0: <= 24 blocks)
        const unsigned c = hb_pair_code(ckey[wi], ckey[wj], catbits, tb.ng);
        const int cb8 = (int)(c & 0xffu) * kTabR;
#pragma unroll
        for (int k2 = 0; k2 < kHbNear; ++k2) {
          if (k2 >= nnear) break;
          const int g = sgrp[k2];
          nacc[k2] += sv * (double)tab[k2 * tstride + cb8 + (int)((c >> (8 * (g + 1))) & 0xffu)];
        }
      }
    }
  }
  // the near slots' S parts and tr S's part: the waves' sums in a fixed order
#pragma unroll
  for (int k = 0; k < kHbNear; ++k) {
    const double sk = wave_sum(nacc[k]);
    if (lane == 0) red[w][k] = sk;
  }
  {
    const double st = wave_sum(tS);
    if (lane == 0) red[w][kHbNear] = st;
  }
  __syncthreads();
  if (tid <= kHbNear) {
    double t = 0.0;
#pragma unroll
    for (int u = 0; u < kHbSlabWaves; ++u) t += red[u][tid];
    out[kHbNearS + tid] = t;
  }
}

// ------------------------------------------------------------------------------------------
// the final contraction per latent dim: the slabs in a fixed order; raw sums into the table adjoint's slots
// part[l][slot][0] (the other G - 1 zero) for kl_gram_bwd_reduce
// ------------------------------------------------------------------------------------------
constexpr int kNoiseSlotHb = 64, kBwdSlotsHb = 65;  // (gram.hip's kNoiseSlot / kBwdSlots)

// the slab records summed over J in a fixed order, in place into slab 0's record: thread (e, l) owns entry e
__global__ __launch_bounds__(256) void hb_sum_kernel(HbWs ws, int np_) {
  const int i = blockIdx.x * 256 + threadIdx.x, l = blockIdx.y, nt = np_ / kHbT, nb2 = ws.dev->nb2;
  if (!ws.dev->on || i >= 2 * nb2 + kHbTail) return;  // (the written entries only: M, Q, the tail)
  const int e = i < nb2 ? i : i < 2 * nb2 ? kHbBins2 + i - nb2 : 2 * kHbBins2 + i - 2 * nb2;
  double* pl = ws.part + (int64_t)l * nt * kHbPart + e;
  double s = 0.0;
#pragma unroll 16
  for (int J = 0; J < nt; ++J) s += pl[(int64_t)J * kHbPart];
  pl[0] = s;
}

__global__ __launch_bounds__(256) void hb_final_kernel(GramTab tb, HbWs ws, int n, int np_,
                                                       const double* __restrict__ alpha,
                                                       const double* __restrict__ kdiag, double* __restrict__ part,
                                                       int G, int dbg) {
  __shared__ HbDev d;
  __shared__ double Gb[kHbBins2];   // (Q - M - a a^T) / 2 per far bin pair
  __shared__ double raw[kBwdSlotsHb];
  __shared__ double red[4];
  __shared__ double nz;
  extern __shared__ float ftab[];   // the derivative tables
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l = blockIdx.x, nt = np_ / kHbT;
  if (tid == 0) d = *ws.dev;
  __syncthreads();
  if (!d.on) return;  // (uniform)
  if (tid < kBwdSlotsHb) raw[tid] = 0.0;
  const double* al = alpha + (int64_t)l * np_;
  const double* pl = ws.part + (int64_t)l * nt * kHbPart;  // (hb_sum_kernel's sums)
  {
    const float* gt = ws.tab + (int64_t)l * kTabMaxBwdLds;
    for (int e = tid; e < tb.pbeg[tb.ng] * (1 << tb.nbits) * kTabR; e += 256) ftab[e] = gt[e];
  }
  for (int e = tid; e < d.nb2; e += 256) {
    int g = 0;
    while (g + 1 < d.nbin && e >= d.b2off[g + 1]) ++g;
    const int nb = d.bn[g], b = (e - d.b2off[g]) / nb, bc = (e - d.b2off[g]) % nb;
    const double m = pl[e], q = pl[kHbBins2 + e];
    Gb[e] = 0.5 * (q - m - pl[kHbA + d.boff[g] + b] * pl[kHbA + d.boff[g] + bc]);
  }
  // tr G = (sum diag K^-1 - tr S - alpha^T alpha) / 2 (the noise slot)
  {
    double s = 0.0;
    for (int i = tid; i < n; i += 256) s += kdiag[(int64_t)l * np_ + i] - al[i] * al[i];
    s = wave_sum(s);
    if (lane == 0) red[w] = s;
  }
  __syncthreads();
  if (tid == 0) {
    nz = 0.5 * ((((red[0] + red[1]) + red[2]) + red[3]) - pl[kHbNearS + kHbNear]);
    for (int k = 0; k < d.nnear; ++k)  // near slots: -S part / 2 + the K^-1 - alpha alpha^T part
      raw[tb.porder[d.nslot[k]]] = -0.5 * pl[kHbNearS + k] + pl[kHbNearK + k];
  }
  const int tstride = (1 << tb.nbits) * kTabR;
  // far slots: sum over the bin pairs of the slot's binning
  for (int k = 0; k < ((dbg & 16) ? 0 : tb.pbeg[tb.ng]); ++k) {
    const int p = tb.porder[k], r = tb.pcomp[p], g = d.cbin[r];
    if (g < 0) continue;  // (uniform) near
    const int nb = d.bn[g], grp = d.bgrp[g], W = grp >= 0 ? d.wrng[grp] : 1;
    double s = 0.0;
    for (int e = tid; e < nb * nb; e += 256) {
      int b = e / nb, bc = e % nb;
      const int w1 = b % W, w2 = bc % W;
      b /= W;
      bc /= W;
      int bits = 0;
#pragma unroll
      for (int q = kTabMaxBits - 1; q >= 0; --q) {  // the mask's gate values, the last bit fastest (hb_plan_kernel)
        if (q >= tb.nbits || !((d.bmask[g] >> q) & 1)) continue;
        const int v1 = b % d.grng[q] + d.gmin[q], v2 = bc % d.grng[q] + d.gmin[q];
        b /= d.grng[q];
        bc /= d.grng[q];
        const bool pass = tb.bkind[q] == LVAE_CAT ? v1 == v2 : v1 + v2 == 2;
        bits += pass ? (kTabR << q) : 0;
      }
      s += Gb[d.b2off[g] + e] * (double)ftab[k * tstride + bits + abs(w1 - w2)];
    }
    s = wave_sum(s);
    __syncthreads();  // (the previous slot's red read)
    if (lane == 0) red[w] = s;
    __syncthreads();
    if (tid == 0) raw[p] = ((red[0] + red[1]) + red[2]) + red[3];
  }
  __syncthreads();
  if (tid == 0) raw[kNoiseSlotHb] = nz;
  __syncthreads();
  for (int e = tid; e < kBwdSlotsHb * G; e += 256) {
    const int slot = e / G, gg = e % G;
    part[((int64_t)l * kBwdSlotsHb + slot) * G + gg] = gg == 0 ? raw[slot] : 0.0;
  }
}

// ------------------------------------------------------------------------------------------
// host
// ------------------------------------------------------------------------------------------
static int hb_dbg() {  // (timing only: LVAE_HB_DBG bits skip the slab pass's parts -- wrong results)
  const char* v = getenv("LVAE_HB_DBG");
  return v ? atoi(v) : 0;
}

static int hb_enabled() {  // (read per call: A/B runs and tests switch it inside one process)
  const char* v = getenv("LVAE_KL_HYPER");
  return !v || atoi(v) != 0;
}

// the slab kernel's LDS: static + H + the near slots' tables (at most kHbNear of them); 0 = does not fit
static size_t hb_slab_lds(const GramTab& tb) {
  static size_t stat = 0;
  if (!stat) {
    hipFuncAttributes a;
    if (hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&hb_slab_kernel)) != hipSuccess) return 0;
    stat = a.sharedSizeBytes;
  }
  const int ns = tb.pbeg[tb.ng] < kHbNear ? tb.pbeg[tb.ng] : kHbNear;
  const size_t dyn = (size_t)ns * (1 << tb.nbits) * kTabR * sizeof(float);
  return stat + dyn <= 160 * 1024 ? (dyn ? dyn : 4) : 0;
}

// the host's part of the conditions: the table family, the route enabled, the slab kernel's LDS fits
static bool hb_host_ok(const lvae_kernel_spec* spec, GramTab& tb) {
  return gram_tab_build(spec, tb) && hb_enabled() && hb_slab_lds(tb) > 0;
}

// the plan and the pair codes (after kl_gram_fill's covariate check, on the same stream)
int kl_hyper_plan(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int np_, int L, void* wsbase,
                  const int* covflag, hipStream_t st) {
  HbWs ws((char*)wsbase, np_, L);
  GramTab tb;
  if (!hb_host_ok(spec, tb)) {
    if (zero_async(ws.dev, sizeof(HbDev), st) != 0) return LVAE_ERR_LAUNCH;
    return 0;
  }
  hb_plan_kernel<<<1, 1024, 0, st>>>(tb, x, ldx, n, np_, covflag, ws, 1);
  LVAE_CHECK_LAUNCH();
  return 0;
}

// the binned hyper-gradient (raw sums into part, the table adjoint's layout with G workgroup slots); its kernels
// exit at once when the plan is off
int kl_hyper_bwd(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int np_, int L, const double* params,
                 const float* Kinv, const float* v, const double* alpha, const double* kdiag, void* wsbase, double* part,
                 int G, hipStream_t st) {
  (void)x;
  (void)ldx;
  HbWs ws((char*)wsbase, np_, L);
  GramTab tb;
  // (not hb_host_ok: LVAE_KL_HYPER is the forward's decision, recorded in the plan's device flag -- the kernels
  // below exit at once when it is off -- so a change of the variable between forward and backward cannot leave
  // the S-GEMM half skipped and this half unlaunched)
  if (!gram_tab_build(spec, tb) || hb_slab_lds(tb) == 0) return 0;
  const size_t tabb = (size_t)tb.pbeg[tb.ng] * (1 << tb.nbits) * kTabR * sizeof(float);
  const size_t sdyn = hb_slab_lds(tb), ndyn = sdyn;
  const int nt = np_ / kHbT;
  hb_tab_kernel<<<dim3((unsigned)((tabb / sizeof(float) + 255) / 256), L), 256, 0, st>>>(tb, ws, params);
  hb_near_kernel<<<dim3(nt, L), 256, ndyn, st>>>(tb, ws, n, np_, Kinv, alpha);
  {
    ProfScope ps(LVAE_PH_HB_SLAB, st);
    hb_slab_kernel<<<dim3(nt, L), kHbSlabThreads, sdyn, st>>>(tb, ws, n, np_, Kinv, v, alpha, hb_dbg());
  }
  hb_sum_kernel<<<dim3((2 * kHbBins2 + kHbTail + 255) / 256, L), 256, 0, st>>>(ws, np_);
  hb_final_kernel<<<L, 256, tabb, st>>>(tb, ws, n, np_, alpha, kdiag, part, G, hb_dbg());
  LVAE_CHECK_LAUNCH();
  return 0;
}

}  // namespace lvae

extern "C" int lvae_kl_closed_hyper_state(int n, int L, const void* workspace, int32_t* on, void* stream) {
  if (n <= 0) return -1;
  if (L <= 0) return -2;
  if (!workspace) return -3;
  if (!on) return -4;
  size_t kl_hyper_offset_in_kl_ws(int np_, int L);
  const int np_ = (n + 255) / 256 * 256;
  const char* hb = (const char*)workspace + kl_hyper_offset_in_kl_ws(np_, L);
  const lvae::HbWs ws(const_cast<char*>(hb), np_, L);
  if (lvae::copy_words_async(on, &ws.dev->on, sizeof(int32_t), (hipStream_t)stream) != 0) return LVAE_ERR_LAUNCH;
  return 0;
}
