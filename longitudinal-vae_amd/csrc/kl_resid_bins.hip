// kl_resid_bins.hip -- the exact KL's fp64 residual r = mu - K a0 (kl_gram_resid, gram.hip) in O(N W)
// instead of O(N^2) when the covariates are integer-coded.
//
// Every component of the reference's kernel family (GP_model.py:146-236: Cat / Bin kernels, RBF, their
// products, the missing-value Bin masks) is a product of gates (Cat: x_i == x_j, Bin: x_i + x_j == 2) and
// at most one continuous factor phi(x_i[d], x_j[d]) (RBF / periodic of the distance, or linear x_i x_j).
// With integer covariates -- gate values in [0, R), continuous values in a window [c0, c0 + W), W <= 64 --
// the points fall into G W bins (G = the product of the gates' ranges): j's bin is (its gate values, its
// continuous value), and
//   (K_r a)_i = s_r sum_{c < W} phi(x_i[d], c0 + c) H_r[g(i)][c],   H_r[g][c] = sum_{j in bin (g, c)} w_j a_j
// where g(i) is the gate tuple j must have to pass i's gates (Cat: x_i[d]; Bin: 2 - x_i[d]) and w_j = 1
// (w_j = x_j[d] and phi = x_i[d] for a linear factor, W = 1).  Three launches:
//   rb_plan_kernel  one workgroup per component: checks the conditions on x (else flags the component, and
//                   kl_gram_resid falls back to its tiled O(N^2) kernel), bins the points, sorts (bin, j)
//                   keys (bitonic, in LDS) into CSR bin lists -- so every H sum runs in a fixed order
//   rb_hist_kernel  H_r[l][bin] over its CSR list, fp64, deterministic
//   rb_eval_kernel  r_i = mu_i - noise a_i - sum_r (K_r a)_i from per-(dim, component) fp64 phi tables
// Exact arithmetic aside from the order of the fp64 sums (the same terms as the tiled kernel).
#include <stdlib.h>

#include "common.hpp"

namespace lvae {

constexpr int kRbMaxN = 16384;     // points the in-LDS sort handles (keys: bin << 16 | j)
constexpr int kRbMaxW = 64;        // continuous window
constexpr int kRbMaxBins = 16384;  // bins per component (G W)
constexpr int kRbMaxGates = 3;

struct RbComp {
  int ok;                     // 1: this component is binned
  int ngate;
  int gdim[kRbMaxGates], gbin[kRbMaxGates], grange[kRbMaxGates], gstride[kRbMaxGates];
  int ckind, cdim, c0, W;     // continuous factor (ckind -1: none)
  int nb;                     // bins = G W
  int base;                   // this component's first bin in the H / offset arrays
};

// workspace laid out for a capacity of np points (the caller's padded size)
struct RbWs {
  RbComp* comp;   // [n_comp]
  int* ok;        // [1] all components binned (written by the plan; read by every launch)
  int* off;       // [n_comp][kRbMaxBins + 1] CSR offsets
  int* mem;       // [n_comp][np] point index at each sorted position
  int* pbin;      // [n_comp][np] bin at each sorted position
  double* seg;    // [L][n_comp][np] segment sums ending at a sorted position (rb_seg_kernel)
  double* H;      // [L][n_comp][kRbMaxBins]
  size_t bytes;
  RbWs(char* base, int np_, int L, int ncomp) {
    size_t o = 0;
    auto take = [&](size_t b) {
      char* p = base ? base + o : nullptr;
      o += align256(b);
      return p;
    };
    comp = (RbComp*)take(sizeof(RbComp) * LVAE_MAX_COMP);
    ok = (int*)take(sizeof(int));
    off = (int*)take(sizeof(int) * (size_t)ncomp * (kRbMaxBins + 1));
    mem = (int*)take(sizeof(int) * (size_t)ncomp * np_);
    pbin = (int*)take(sizeof(int) * (size_t)ncomp * np_);
    seg = (double*)take(sizeof(double) * (size_t)L * ncomp * np_);
    H = (double*)take(sizeof(double) * (size_t)L * ncomp * kRbMaxBins);
    bytes = o;
  }
};

size_t kl_resid_bins_bytes(int np_, int L, int ncomp) { return RbWs(nullptr, np_, L, ncomp).bytes; }

// structure the host can check: every component at most one continuous factor, at most kRbMaxGates gates
bool kl_resid_bins_spec_ok(const lvae_kernel_spec* s, int n) {
  if (n > kRbMaxN || n < 1) return false;
  for (int r = 0; r < s->n_comp; ++r) {
    int nc = 0, ng = 0;
    for (int f = 0; f < s->n_fac[r]; ++f) {
      const int k = s->kind[r][f];
      if (k == LVAE_CAT || k == LVAE_BIN) ++ng;
      else ++nc;
    }
    if (nc > 1 || ng > kRbMaxGates) return false;
  }
  return true;
}

__device__ inline int rb_block_min(int v, int* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  if ((threadIdx.x & 63) == 0) atomicMin(red, v);
  __syncthreads();
  return *red;
}
__device__ inline int rb_block_max(int v, int* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(red, v);
  __syncthreads();
  return *red;
}

__global__ void rb_init_kernel(int* ok) {
  if (threadIdx.x == 0) *ok = 1;
}

// one workgroup (1024 threads) per component r; n <= kRbMaxN
__global__ __launch_bounds__(1024) void rb_plan_kernel(DevSpec s, const double* __restrict__ x, int ldx, int n,
                                                       int np_, RbWs ws) {
  __shared__ uint32_t keys[kRbMaxN];
  __shared__ int red[8];
  __shared__ int bad_s;
  const int r = blockIdx.x, t = threadIdx.x;
  if (t < 8) red[t] = (t & 1) ? INT_MIN : INT_MAX;
  if (t == 0) bad_s = 0;
  __syncthreads();
  RbComp c{};
  c.ckind = -1;
  for (int f = 0; f < s.n_fac[r]; ++f) {
    const int k = s.kind[r][f];
    if (k == LVAE_CAT || k == LVAE_BIN) {
      c.gdim[c.ngate] = s.dim[r][f];
      c.gbin[c.ngate] = k == LVAE_BIN;
      ++c.ngate;
    } else {
      c.ckind = k;
      c.cdim = s.dim[r][f];
    }
  }
  // ranges: every gate value an integer in [0, 65535]; the continuous values integers in a window <= 64
  // (a linear factor needs no integrality: it is folded into the bin weights)
  int bad = 0;
  int gmax[kRbMaxGates] = {0, 0, 0}, cmin = INT_MAX, cmax = INT_MIN;
  for (int j = t; j < n; j += 1024) {
    const double* xj = x + (int64_t)j * ldx;
    for (int q = 0; q < c.ngate; ++q) {
      const double v = xj[c.gdim[q]];
      bad |= !(v == rint(v) && v >= 0.0 && v < 65536.0);
      if (!bad) gmax[q] = max(gmax[q], (int)v);
    }
    if (c.ckind == LVAE_RBF || c.ckind == LVAE_PER) {
      const double v = xj[c.cdim];
      bad |= !(v == rint(v) && fabs(v) < 1048576.0);
      if (!bad) {
        cmin = min(cmin, (int)v);
        cmax = max(cmax, (int)v);
      }
    }
  }
  if (__any(bad) && (t & 63) == 0) atomicOr(&bad_s, 1);
  int G = 1;
  for (int q = 0; q < c.ngate; ++q) {
    c.grange[q] = rb_block_max(gmax[q], &red[2 * q + 1]) + 1;
  }
  if (c.ckind == LVAE_RBF || c.ckind == LVAE_PER) {
    c.c0 = rb_block_min(cmin, &red[6]);
    c.W = rb_block_max(cmax, &red[7]) - c.c0 + 1;
  } else {
    c.c0 = 0;
    c.W = 1;
  }
  __syncthreads();
  bool ok = !bad_s && c.W <= kRbMaxW && n <= kRbMaxN;
  for (int q = c.ngate - 1; q >= 0 && ok; --q) {
    c.gstride[q] = G;
    if ((int64_t)G * c.grange[q] * c.W > kRbMaxBins) ok = false;
    G *= c.grange[q];
  }
  c.nb = G * c.W;
  c.base = r * kRbMaxBins;
  c.ok = ok;
  if (t == 0) ws.comp[r] = c;
  if (!ok) {
    if (t == 0) *ws.ok = 0;  // (every writer stores 0)
    return;                  // (uniform)
  }
  // keys (bin << 16 | j), padded to a power of two with 0xFFFFFFFF, sorted ascending in LDS
  int M = 1;
  while (M < n) M <<= 1;
  for (int j = t; j < M; j += 1024) {
    uint32_t key = 0xFFFFFFFFu;
    if (j < n) {
      const double* xj = x + (int64_t)j * ldx;
      int g = 0;
      for (int q = 0; q < c.ngate; ++q) g += (int)xj[c.gdim[q]] * c.gstride[q];
      const int cc = c.W > 1 ? (int)xj[c.cdim] - c.c0 : 0;
      key = ((uint32_t)(g * c.W + cc) << 16) | (uint32_t)j;
    }
    keys[j] = key;
  }
  __syncthreads();
  for (int k = 2; k <= M; k <<= 1)
    for (int jj = k >> 1; jj > 0; jj >>= 1) {
      for (int i = t; i < M; i += 1024) {
        const int ixj = i ^ jj;
        if (ixj > i) {
          const uint32_t a = keys[i], b = keys[ixj];
          if ((a > b) == ((i & k) == 0)) {
            keys[i] = b;
            keys[ixj] = a;
          }
        }
      }
      __syncthreads();
    }
  int* mem = ws.mem + (int64_t)r * np_;
  int* pbin = ws.pbin + (int64_t)r * np_;
  for (int p = t; p < n; p += 1024) {
    mem[p] = (int)(keys[p] & 0xFFFFu);
    pbin[p] = (int)(keys[p] >> 16);
  }
  // CSR offsets: off[b] = #keys with bin < b (binary search over the sorted bins)
  int* off = ws.off + (int64_t)r * (kRbMaxBins + 1);
  for (int b = t; b <= c.nb; b += 1024) {
    int lo = 0, hi = n;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if ((int)(keys[mid] >> 16) < b) lo = mid + 1;
      else hi = mid;
    }
    off[b] = lo;
  }
}

// The bin sums in two fixed-order stages, so a bin of any size costs O(size / 64):
// rb_seg_kernel: each wave takes 64 sorted positions, forms w_j a[l][j] and a segmented inclusive scan
// over runs of equal bin (6 shuffle steps); the lane ending a run within the wave stores the run's sum
// at its position.  Grid (np / 256, n_comp, L).
__global__ __launch_bounds__(256) void rb_seg_kernel(const double* __restrict__ x, int ldx, int n, int np_,
                                                     RbWs ws, const double* __restrict__ alpha) {
  const int r = blockIdx.y, l = blockIdx.z, p = blockIdx.x * 256 + threadIdx.x, lane = threadIdx.x & 63;
  if (!*ws.ok) return;
  const RbComp c = ws.comp[r];
  double v = 0.0;
  int b = -1 - lane;  // the padding: runs of one
  if (p < n) {
    const int j = ws.mem[(int64_t)r * np_ + p];
    b = ws.pbin[(int64_t)r * np_ + p];
    v = (c.ckind == LVAE_LIN ? x[(int64_t)j * ldx + c.cdim] : 1.0) * alpha[(int64_t)l * np_ + j];
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double u = __shfl_up(v, o, 64);
    const int bu = __shfl_up(b, o, 64);
    if (lane >= o && bu == b) v += u;
  }
  const int bn = __shfl_down(b, 1, 64);
  if (p < n && (lane == 63 || bn != b)) ws.seg[((int64_t)l * gridDim.y + r) * np_ + p] = v;
}

// rb_hist_kernel: H[l][base + b] = the run sums of bin b over the 64-position blocks its sorted range
// [off[b], off[b + 1]) touches, in block order.  Grid (kRbHistG, n_comp, L), bins strided over it.
constexpr int kRbHistG = 4;
__global__ __launch_bounds__(256) void rb_hist_kernel(int np_, RbWs ws) {
  const int r = blockIdx.y, l = blockIdx.z;
  if (!*ws.ok) return;
  const RbComp c = ws.comp[r];
  const int* off = ws.off + (int64_t)r * (kRbMaxBins + 1);
  const double* seg = ws.seg + ((int64_t)l * gridDim.y + r) * np_;
  double* H = ws.H + (int64_t)l * gridDim.y * kRbMaxBins + c.base;
  for (int b = blockIdx.x * 256 + threadIdx.x; b < c.nb; b += kRbHistG * 256) {
    const int p0 = off[b], p1 = off[b + 1];
    double h = 0.0;
    for (int e = p0 | 63; e < p1 - 1; e += 64) h += seg[e];  // runs ending at a block's last lane
    if (p1 > p0) h += seg[p1 - 1];
    H[b] = h;
  }
}

// res[l][i] = mu[l][i] - noise a_i - sum_r s_r sum_c phi_r(x_i, c0 + c) H_r[g(i)][c]; 0 on the padding.
// grid (np / 256, L); phi tables per (component, |distance|) in fp64 (the same functions as the tiled
// kernel's factor64_at).
__global__ __launch_bounds__(256) void rb_eval_kernel(DevSpec s, const double* __restrict__ x, int ldx, int n,
                                                      int np_, RbWs ws, const double* __restrict__ params,
                                                      const double* __restrict__ noise,
                                                      const double* __restrict__ alpha,
                                                      const double* __restrict__ muc, double* __restrict__ res) {
  __shared__ double phi[LVAE_MAX_COMP][kRbMaxW];
  const int l = blockIdx.y, t = threadIdx.x, i = blockIdx.x * 256 + t;
  if (!*ws.ok) return;
  const double* pl = params + (int64_t)l * s.n_params;
  for (int e = t; e < s.n_comp * kRbMaxW; e += 256) {
    const int r = e / kRbMaxW, d = e % kRbMaxW;
    double v = 1.0;
    for (int f = 0; f < s.n_fac[r]; ++f) {
      const int k = s.kind[r][f], pi = s.param_idx[r][f];
      if (k == LVAE_RBF) v = exp(-0.5 * (double)d * (double)d / (pl[pi] * pl[pi]));
      if (k == LVAE_PER) {
        const double sn = sin((double)d * (M_PI / pl[pi + 1]));
        v = exp(-2.0 / (pl[pi] * pl[pi]) * sn * sn);
      }
    }
    phi[r][d] = v * pl[s.scale_idx[r]];
  }
  __syncthreads();
  if (i >= np_) return;
  const int64_t li = (int64_t)l * np_ + i;
  if (i >= n) {
    res[li] = 0.0;
    return;
  }
  const double* xi = x + (int64_t)i * ldx;
  const double* H = ws.H + (int64_t)l * s.n_comp * kRbMaxBins;
  double acc = noise[l] * alpha[li];
  for (int r = 0; r < s.n_comp; ++r) {
    const RbComp c = ws.comp[r];
    int g = 0;
    bool in = true;
    for (int q = 0; q < c.ngate; ++q) {
      const int v = c.gbin[q] ? 2 - (int)xi[c.gdim[q]] : (int)xi[c.gdim[q]];
      in = in && v >= 0 && v < c.grange[q];
      g += v * c.gstride[q];
    }
    if (!in) continue;
    const double* h = H + c.base + g * c.W;
    if (c.ckind == LVAE_RBF || c.ckind == LVAE_PER) {
      const int ci = (int)xi[c.cdim] - c.c0;
      double sr = 0.0;
      for (int cc = 0; cc < c.W; ++cc) sr += phi[r][abs(ci - cc)] * h[cc];
      acc += sr;
    } else if (c.ckind == LVAE_LIN) {
      acc += phi[r][0] * xi[c.cdim] * h[0];
    } else {
      acc += phi[r][0] * h[0];
    }
  }
  res[li] = muc[li] - acc;
}

// the binned path runs iff the spec qualifies (kl_resid_bins_spec_ok) and LVAE_RESID_BINS is not "0"
bool kl_resid_bins_enabled(const lvae_kernel_spec* spec, int n) {
  static const bool on = !getenv("LVAE_RESID_BINS") || atoi(getenv("LVAE_RESID_BINS")) != 0;
  return on && kl_resid_bins_spec_ok(spec, n);
}

// the plan (depends on x only; kl_closed.hip enqueues it on the side stream during the factorisation)
int kl_resid_bins_plan(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int np_, int L, void* wsbuf,
                       hipStream_t st) {
  RbWs ws((char*)wsbuf, np_, L, spec->n_comp);
  rb_init_kernel<<<1, 64, 0, st>>>(ws.ok);
  rb_plan_kernel<<<spec->n_comp, 1024, 0, st>>>(to_dev(spec), x, ldx, n, np_, ws);
  LVAE_CHECK_LAUNCH();
  return 0;
}

// the bin sums and the residual, after the plan; *okflag = the plan's device flag (1: every component
// was binned -- else these kernels exit at once and the caller's tiled kernels, given the flag, run)
int kl_resid_bins(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int np_, int L,
                  const double* params, const double* noise, const double* alpha0, const double* muc, double* res,
                  void* wsbuf, int** okflag, hipStream_t st) {
  const DevSpec ds = to_dev(spec);
  RbWs ws((char*)wsbuf, np_, L, spec->n_comp);
  *okflag = ws.ok;
  const int nc = spec->n_comp;
  rb_seg_kernel<<<dim3(cdiv(np_, 256), nc, L), 256, 0, st>>>(x, ldx, n, np_, ws, alpha0);
  rb_hist_kernel<<<dim3(kRbHistG, nc, L), 256, 0, st>>>(np_, ws);
  rb_eval_kernel<<<dim3(cdiv(np_, 256), L), 256, 0, st>>>(ds, x, ldx, n, np_, ws, params, noise, alpha0, muc, res);
  LVAE_CHECK_LAUNCH();
  return 0;
}

}  // namespace lvae
