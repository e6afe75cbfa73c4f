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
// <= 64 points; far binnings <= 4, with <= 128 bins
// in all and sum nbins^2 <= 4096; <= 8 parameter slots on near components.
#include "blkinv.hpp"
#include "gram_tab.hpp"

namespace lvae {

constexpr int kHbMaxBin = 4;    // far binnings
constexpr int kHbBins = 128;    // far bins in all
constexpr int kHbBins2 = 4096;  // sum over binnings of nbins^2
constexpr int kHbRun = 64;      // longest run of the big covariate
constexpr int kHbSmall = 16;    // Cat gate covariates other than the big one span at most this many values
constexpr int kHbSmallest = 4;  // the big covariate spans more than this many values
constexpr int kHbNear = 8;      // parameter slots of the near components
constexpr int kHbT = 64;        // row tile = column slab
constexpr int kHbTP = 65;       // LDS pitch of a tile row (floats)
constexpr int kHbQ = 16;        // covariate columns staged
constexpr int kHbPart = 2 * kHbBins2 + kHbNear + 1;  // doubles per (dim, slab) partial record

struct HbDev {
  int on, nbin, big, nbins, nb2, nnear;
  int gmin[kTabMaxBits], grng[kTabMaxBits];                  // gate bit: min value, number of values
  int wmin[kTabMaxG], wrng[kTabMaxG];                        // distance group: min value, number of values
  int bmask[kHbMaxBin], bgrp[kHbMaxBin], boff[kHbMaxBin], bn[kHbMaxBin], b2off[kHbMaxBin];  // far binnings
  int cbin[LVAE_MAX_COMP];                                   // component -> binning, -1: near
  int nslot[kHbNear];                                        // near parameter slots (GramTab porder index)
};

struct HbWs {
  HbDev* dev;
  uint8_t* pbin;  // [kHbMaxBin][np] local bin of every point (255: padding)
  int* rs;        // [np] start of the point's run of the big covariate
  int* re;        // [np] its end (exclusive)
  double* part;   // [L][np / 64][kHbPart] per-slab partials
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


// ------------------------------------------------------------------------------------------
// the slab pass: workgroup (J, l) streams column slab J (64 columns) of the full symmetric K^-1 of dim l, 64-row
// tile by tile, and writes its partial record: M_g = H_g V H_g^T, Q_g = H_g Phi_g (the slab's columns), the near
// runs' parts per near slot and the slab's part of tr S.
// ------------------------------------------------------------------------------------------
__device__ inline int hb_row_slot(int row) { return (row >> 6) & 1; }

// an LDS fp64 add whose return value is not used (ds_add_f64): a wave's adds to one address apply in program order
__device__ inline void hb_lds_add(double* p, double v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

constexpr int kHbPre = (kHbQ * kHbT + 255) / 256;  // covariate values a thread prefetches per tile
typedef float hb_f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void hb_slab_kernel(GramTab tb, HbWs ws, const double* __restrict__ x, int ldx,
                                                      int n, int np_, int qs, const double* __restrict__ params,
                                                      const float* __restrict__ Kinv, const float* __restrict__ vv,
                                                      const double* __restrict__ alpha) {
  __shared__ HbDev d;
  __shared__ __attribute__((aligned(16))) float T[2][kHbT * kHbTP];  // the row tiles of the window (slot = (row / 64) & 1)
  __shared__ float cov[2][kHbQ][kHbT];          // their covariates
  __shared__ double alr[2][kHbT];               // their alpha
  __shared__ float vs[kHbT];                    // v of the slab's columns
  __shared__ float sp[64];
  __shared__ int runs[kHbT], runl[kHbT], nrun;
  __shared__ int sbdim[kTabMaxBits], sbkind[kTabMaxBits];  // the gates (LDS copies: no kernarg loads in loops)
  __shared__ int snoff[kHbNear], sngd[kHbNear];            // near slot: its table offset, its distance dim
  __shared__ uint8_t cbin[kHbMaxBin][kHbT];     // bins of the slab's columns
  __shared__ double red[4][kHbNear + 1];
  extern __shared__ double hdyn[];              // H [kHbBins][64] (fp64), then the derivative tables (fp32)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, J = blockIdx.x, l = blockIdx.y, J0 = J * kHbT;
  if (tid == 0) d = *ws.dev;
  __syncthreads();
  if (!d.on) return;  // (uniform)
  double* H = hdyn;
  float* tab = reinterpret_cast<float*>(hdyn + kHbBins * kHbT);
  const int tstride = (1 << tb.nbits) * kTabR, nbits = tb.nbits;
  if (tid < tb.n_params) sp[tid] = float(params[(int64_t)l * tb.n_params + tid]);
  for (int e = tid; e < d.nbins * kHbT; e += 256) H[e] = 0.0;
  if (tid < kHbT) vs[tid] = vv[(int64_t)l * np_ + J0 + tid];
  if (tid < kTabMaxBits) {
    sbdim[tid] = tid < nbits ? tb.bdim[tid] : 0;
    sbkind[tid] = tid < nbits ? tb.bkind[tid] : 0;
  }
  if (tid < d.nnear) {
    const int kk = d.nslot[tid];
    snoff[tid] = kk * tstride;
    sngd[tid] = tb.gdim[tb.cgrp[tb.pcomp[tb.porder[kk]]]];
  }
  for (int e = tid; e < d.nbin * kHbT; e += 256) cbin[e / kHbT][e % kHbT] = ws.pbin[(size_t)(e / kHbT) * np_ + J0 + e % kHbT];
  __syncthreads();
  tab_build_bwd(tb, sp, tab);
  const float* K = Kinv + (int64_t)l * np_ * np_;
  const double* al = alpha + (int64_t)l * np_;
  const int nbin = d.nbin, nnear = d.nnear, bigon = d.big >= 0;
  const int myoff = w < nbin ? d.boff[w] : 0;
  double nacc[kHbNear];
#pragma unroll
  for (int k = 0; k < kHbNear; ++k) nacc[k] = 0.0;
  double tS = 0.0;
  const int nt = np_ / kHbT;
  // software pipeline: tile I + 1's K^-1 rows, covariates, alpha, bins and run ends in registers during tile I
  hb_f32x4 pk[4];
  float pc[kHbPre];
  double pa = 0.0;
  int pbn = 255, pre_ = -1, prs = -1;
  auto fetch = [&](int I) {
    const int I0 = I * kHbT;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + 256 * u, r = e >> 4, c4 = (e & 15) * 4;
      pk[u] = __builtin_nontemporal_load(reinterpret_cast<const hb_f32x4*>(K + (int64_t)(I0 + r) * np_ + J0 + c4));
    }
#pragma unroll
    for (int u = 0; u < kHbPre; ++u) {
      const int e = tid + 256 * u, q = e / kHbT, r = e % kHbT;
      pc[u] = (q < qs && I0 + r < n) ? float(x[(int64_t)(I0 + r) * ldx + q]) : 0.f;
    }
    if (tid < kHbT) pa = al[I0 + tid];
    pbn = w < nbin ? (int)ws.pbin[(size_t)w * np_ + I0 + lane] : 255;
    if (w == 0 && bigon) {
      pre_ = ws.re[I0 + lane];
      prs = ws.rs[I0 + lane];
    }
  };
  fetch(0);
  for (int I = 0; I < nt; ++I) {
    const int I0 = I * kHbT, sl = I & 1;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + 256 * u, r = e >> 4, c4 = (e & 15) * 4;
      float* t = &T[sl][r * kHbTP + c4];
      t[0] = pk[u][0];
      t[1] = pk[u][1];
      t[2] = pk[u][2];
      t[3] = pk[u][3];
    }
#pragma unroll
    for (int u = 0; u < kHbPre; ++u) {
      const int e = tid + 256 * u, q = e / kHbT, r = e % kHbT;
      if (q < kHbQ) cov[sl][q][r] = pc[u];
    }
    if (tid < kHbT) alr[sl][tid] = pa;
    const int bn = pbn;  // (wave w < nbin: the bin of row lane in binning w)
    if (w == 0) {        // the runs of the big covariate ending in this tile
      const int i = I0 + lane;
      const bool last = bigon && i < n && pre_ == i + 1;
      const unsigned long long m = __ballot(last);
      if (last) {
        const int k = __popcll(m & ((1ull << lane) - 1));
        runs[k] = prs;
        runl[k] = i + 1 - prs;
      }
      if (lane == 0) nrun = __popcll(m);
    }
    __syncthreads();
    if (I + 1 < nt) fetch(I + 1);  // (in flight under this tile's work)
    // H_w[bin(i)][m] += K^-1_im: wave w owns binning w, lane m column m; the rows in order (ds_add_f64 without
    // return: no dependent latency, program order per address -> a fixed summation order)
    if (w < nbin) {
      const float* tr = &T[sl][lane];
#pragma unroll 16
      for (int r = 0; r < kHbT; ++r) {
        const int b = __builtin_amdgcn_readlane(bn, r);
        if (b != 255) hb_lds_add(&H[(myoff + b) * kHbT + lane], (double)tr[r * kHbTP]);
      }
    }
    {  // the slab's part of tr S = sum_m v_m sum_i (K^-1_im)^2: wave w, rows = w (mod 4)
      float ts = 0.f;
#pragma unroll
      for (int r = w; r < kHbT; r += 4) {
        const float t = T[sl][r * kHbTP + lane];
        ts += t * t;
      }
      tS += (double)ts * (double)vs[lane];
    }
    // near runs ending in this tile: 16 x 16 blocks (bi, bj) of X V X^T on v_mfma_f32_16x16x4f32, block items dealt
    // to the waves; each lane's 4 pairs contracted at once with the near slots' tables
    {
      int item = w;
      const int nr = nrun;
      for (int k = 0; k < nr; ++k) {
        const int s0 = runs[k], len = runl[k], nb16 = (len + 15) >> 4;
        for (; item < nb16 * nb16; item += 4) {
          const int bi = item / nb16, bj = item % nb16;
          const int li = lane & 15, lk = lane >> 4;
          const int ra = s0 + 16 * bi + li, rb = s0 + 16 * bj + li;  // the lane's A row, B column
          const bool va = 16 * bi + li < len, vb = 16 * bj + li < len;
          const float* ta = &T[hb_row_slot(ra)][(ra & 63) * kHbTP];
          const float* tb2 = &T[hb_row_slot(rb)][(rb & 63) * kHbTP];
          bi_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
          for (int s4 = 0; s4 < kHbT; s4 += 4) {
            const int m = s4 + lk;
            const float a = va ? ta[m] * vs[m] : 0.f;
            const float b = vb ? tb2[m] : 0.f;
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
          }
          // lane: C[4 lk + q][li] -> pair (i, j) = (s0 + 16 bi + 4 lk + q, s0 + 16 bj + li)
          const int j = s0 + 16 * bj + li, sj = hb_row_slot(j), rj = j & 63;
          const bool jin = j >= J0 && j < J0 + kHbT;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int ioff = 16 * bi + 4 * lk + q, i = s0 + ioff;
            if (ioff >= len || !vb) continue;
            const int si = hb_row_slot(i), ri = i & 63;
            // the pair's gate bits (tab_bits on one element)
            int bits = 0;
#pragma unroll
            for (int b = 0; b < kTabMaxBits; ++b) {
              if (b >= nbits) break;
              const float xi = cov[si][sbdim[b]][ri], xj = cov[sj][sbdim[b]][rj];
              const bool pass = sbkind[b] == LVAE_CAT ? xi == xj : xi + xj == 2.f;
              bits += pass ? (kTabR << b) : 0;
            }
            double val = -0.5 * (double)acc[q];  // the S part (this slab's columns)
            if (jin)                             // the K^-1 and alpha alpha^T parts: once, by the slab holding column j
              val += 0.5 * ((double)T[si][ri * kHbTP + (j - J0)] - alr[si][ri] * alr[sj][rj]);
#pragma unroll
            for (int k2 = 0; k2 < kHbNear; ++k2) {
              if (k2 >= nnear) break;
              const int gd = sngd[k2];
              const int dist = gd >= 0 ? (int)fabsf(cov[si][gd][ri] - cov[sj][gd][rj]) : 0;
              nacc[k2] += val * (double)tab[snoff[k2] + bits + dist];
            }
          }
        }
        item -= nb16 * nb16;  // (this wave's next item index in the following run's block list)
      }
    }
    __syncthreads();  // every reader of slot sl done before tile I + 2 overwrites it (and the run list)
  }
  // Q_g[b][b'] = sum over the slab's columns m in bin b' of H_g[b][m]: thread (g, b) owns row b (LDS scratch = T)
  double* Qs = reinterpret_cast<double*>(&T[0][0]);
  for (int e = tid; e < d.nb2; e += 256) Qs[e] = 0.0;
  __syncthreads();
  if (tid < d.nbins) {
    int g = 0;
    while (g + 1 < nbin && tid >= d.boff[g + 1]) ++g;
    const int b = tid - d.boff[g], nb = d.bn[g];
    double* qrow = Qs + d.b2off[g] + b * nb;
    for (int m = 0; m < kHbT; ++m) {
      const int bc = cbin[g][m];
      if (bc != 255) qrow[bc] += H[tid * kHbT + m];
    }
  }
  __syncthreads();
  double* out = ws.part + ((int64_t)l * nt + J) * kHbPart;
  for (int e = tid; e < d.nb2; e += 256) out[kHbBins2 + e] = Qs[e];
  // M_g = H_g V H_g^T on v_mfma_f64_16x16x4f64: 16 x 16 blocks dealt to the waves
  for (int g = 0; g < nbin; ++g) {
    const int nb = d.bn[g], nb16 = (nb + 15) >> 4;
    for (int item = w; item < nb16 * nb16; item += 4) {
      const int bi = item / nb16, bj = item % nb16, li = lane & 15, lk = lane >> 4;
      const int ba = 16 * bi + li, bb = 16 * bj + li;
      const double* ha = H + (int64_t)(d.boff[g] + (ba < nb ? ba : 0)) * kHbT;
      const double* hb = H + (int64_t)(d.boff[g] + (bb < nb ? bb : 0)) * kHbT;
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
  // the near slots' and tr S's parts: the waves' sums in a fixed order
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
  if (tid <= kHbNear) out[2 * kHbBins2 + tid] = ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
}

// ------------------------------------------------------------------------------------------
// the final contraction per latent dim: the slabs in a fixed order; raw sums into the table adjoint's slots
// part[l][slot][0] (the other G - 1 zero) for kl_gram_bwd_reduce
// ------------------------------------------------------------------------------------------
constexpr int kNoiseSlotHb = 64, kBwdSlotsHb = 65;  // (gram.hip's kNoiseSlot / kBwdSlots)

__global__ __launch_bounds__(256) void hb_final_kernel(GramTab tb, HbWs ws, int n, int np_,
                                                       const double* __restrict__ params,
                                                       const double* __restrict__ alpha,
                                                       const double* __restrict__ kdiag, double* __restrict__ part,
                                                       int G) {
  __shared__ HbDev d;
  __shared__ float sp[64];
  __shared__ double Gb[kHbBins2];   // (Q - M - a a^T) / 2 per far bin pair
  __shared__ double av[kHbBins];    // a = Phi^T alpha
  __shared__ double raw[kBwdSlotsHb];
  __shared__ double red[4];
  extern __shared__ float ftab[];   // the derivative tables
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l = blockIdx.x, nt = np_ / kHbT;
  if (tid == 0) d = *ws.dev;
  __syncthreads();
  if (!d.on) return;  // (uniform)
  if (tid < tb.n_params) sp[tid] = float(params[(int64_t)l * tb.n_params + tid]);
  if (tid < kBwdSlotsHb) raw[tid] = 0.0;
  const double* al = alpha + (int64_t)l * np_;
  {  // a[b]: thread b scans the points in order, 256 at a time through LDS (fixed order)
    __shared__ double ach[256];
    __shared__ uint8_t bch[kHbMaxBin][256];
    int g = 0;
    while (tid < d.nbins && g + 1 < d.nbin && tid >= d.boff[g + 1]) ++g;
    const int b = tid - d.boff[g];
    double s = 0.0;
    for (int i0 = 0; i0 < n; i0 += 256) {
      __syncthreads();
      ach[tid] = i0 + tid < n ? al[i0 + tid] : 0.0;
      for (int q = 0; q < d.nbin; ++q) bch[q][tid] = i0 + tid < n ? ws.pbin[(size_t)q * np_ + i0 + tid] : 255;
      __syncthreads();
      if (tid < d.nbins)
        for (int k = 0; k < 256; ++k)
          if (bch[g][k] == b) s += ach[k];
    }
    if (tid < d.nbins) av[tid] = s;
  }
  __syncthreads();
  tab_build_bwd(tb, sp, ftab);
  const double* pl = ws.part + (int64_t)l * nt * kHbPart;
  for (int e = tid; e < d.nb2; e += 256) {
    int g = 0;
    while (g + 1 < d.nbin && e >= d.b2off[g + 1]) ++g;
    const int nb = d.bn[g], b = (e - d.b2off[g]) / nb, bc = (e - d.b2off[g]) % nb;
    double m = 0.0, q = 0.0;
    for (int J = 0; J < nt; ++J) {
      m += pl[(int64_t)J * kHbPart + e];
      q += pl[(int64_t)J * kHbPart + kHbBins2 + e];
    }
    Gb[e] = 0.5 * (q - m - av[d.boff[g] + b] * av[d.boff[g] + bc]);
  }
  // tr G = (sum diag K^-1 - tr S - alpha^T alpha) / 2 (the noise slot): the first two sums here
  __shared__ double nz;
  {
    double s = 0.0;
    for (int i = tid; i < n; i += 256) s += kdiag[(int64_t)l * np_ + i] - al[i] * al[i];
    s = wave_sum(s);
    if (lane == 0) red[w] = s;
  }
  __syncthreads();
  if (tid == 0) {
    double ts = 0.0;
    for (int J = 0; J < nt; ++J) ts += pl[(int64_t)J * kHbPart + 2 * kHbBins2 + kHbNear];
    nz = 0.5 * ((((red[0] + red[1]) + red[2]) + red[3]) - ts);
    // near slots: the slabs' parts in order
    for (int k = 0; k < d.nnear; ++k) {
      double sk = 0.0;
      for (int J = 0; J < nt; ++J) sk += pl[(int64_t)J * kHbPart + 2 * kHbBins2 + k];
      raw[tb.porder[d.nslot[k]]] = sk;
    }
  }
  const int tstride = (1 << tb.nbits) * kTabR;
  // far slots: sum over the bin pairs of the slot's binning
  for (int k = 0; k < tb.pbeg[tb.ng]; ++k) {
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
      for (int q = tb.nbits - 1; q >= 0; --q) {  // the mask's gate values, the last bit fastest (hb_plan_kernel)
        if (!((d.bmask[g] >> q) & 1)) continue;
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
static int hb_enabled() {  // (read per call: A/B runs and tests switch it inside one process)
  const char* v = getenv("LVAE_KL_HYPER");
  return !v || atoi(v) != 0;
}

// the plan (after kl_gram_fill's covariate check, on the same stream); tb valid only with tab_ok
int kl_hyper_plan(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int np_, int L, void* wsbase,
                  const int* covflag, hipStream_t st) {
  HbWs ws((char*)wsbase, np_, L);
  GramTab tb;
  const bool ok = gram_tab_build(spec, tb) && hb_enabled();
  int qs = 0;
  for (int r = 0; r < spec->n_comp; ++r)
    for (int f = 0; f < spec->n_fac[r]; ++f) qs = spec->dim[r][f] + 1 > qs ? spec->dim[r][f] + 1 : qs;
  if (!ok || qs > kHbQ) {
    if (hipMemsetAsync(ws.dev, 0, sizeof(HbDev), st) != hipSuccess) return LVAE_ERR_LAUNCH;
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
  HbWs ws((char*)wsbase, np_, L);
  GramTab tb;
  if (!gram_tab_build(spec, tb) || !hb_enabled()) return 0;
  int qs = 0;
  for (int r = 0; r < spec->n_comp; ++r)
    for (int f = 0; f < spec->n_fac[r]; ++f) qs = spec->dim[r][f] + 1 > qs ? spec->dim[r][f] + 1 : qs;
  if (qs > kHbQ) return 0;
  const size_t tabb = (size_t)tb.pbeg[tb.ng] * (1 << tb.nbits) * kTabR * sizeof(float);
  hb_slab_kernel<<<dim3(np_ / kHbT, L), 256, kHbBins * kHbT * sizeof(double) + tabb, st>>>(tb, ws, x, ldx, n, np_, qs,
                                                                                        params, Kinv, v, alpha);
  hb_final_kernel<<<L, 256, tabb, st>>>(tb, ws, n, np_, params, alpha, kdiag, part, G);
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
  if (hipMemcpyAsync(on, &ws.dev->on, sizeof(int32_t), hipMemcpyDeviceToDevice, (hipStream_t)stream) != hipSuccess)
    return LVAE_ERR_LAUNCH;
  return 0;
}
