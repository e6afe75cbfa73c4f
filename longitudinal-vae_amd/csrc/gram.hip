// gram.hip -- additive-kernel Gram assembly and its adjoint (GP_model.py:31-144; kernel_gen.py:9-310).
//
// Forward: one 256-thread workgroup per 64x64 output tile of one (batch, latent-dim) slice; the two
// covariate row blocks are staged in LDS (coalesced fp64 reads of the [n, Q] index arrays), each
// thread produces 16 elements of one column (consecutive lanes -> consecutive columns, so the
// stores are coalesced).  The Gram is HBM-write-bound: per element 4 B (f32) / 8 B (f64) out.
#include "gram_bwd.hpp"

namespace lvae {

constexpr int kGT = 64;     // Gram tile edge
constexpr int kMaxQ = 32;   // staged covariate columns

template <int MC, int MF, typename T>
__global__ __launch_bounds__(256) void gram_kernel(DevSpec s, lvae_xview x1, lvae_xview x2, int L, int n1, int n2,
                                                   int qs, const double* __restrict__ params,
                                                   const double* __restrict__ diag, T* __restrict__ out,
                                                   int64_t osb, int64_t osl, int64_t ldo) {
  __shared__ double sx1[kGT * kMaxQ];
  __shared__ double sx2[kGT * kMaxQ];
  __shared__ T sp[64];
  const int bl = blockIdx.z, b = bl / L, l = bl % L;
  const int i0 = blockIdx.y * kGT, j0 = blockIdx.x * kGT;
  const int tid = threadIdx.x;
  if (tid < s.n_params) sp[tid] = T(params[(int64_t)l * s.n_params + tid]);
  const double* p1 = x1.ptr + b * x1.stride_b + l * x1.stride_l;
  const double* p2 = x2.ptr + b * x2.stride_b + l * x2.stride_l;
  for (int e = tid; e < kGT * qs; e += 256) {
    const int r = e / qs, q = e % qs;
    sx1[r * kMaxQ + q] = (i0 + r < n1) ? p1[(int64_t)(i0 + r) * x1.ld + q] : 0.0;
    sx2[r * kMaxQ + q] = (j0 + r < n2) ? p2[(int64_t)(j0 + r) * x2.ld + q] : 0.0;
  }
  __syncthreads();
  const int jj = tid & 63, j = j0 + jj;
  if (j >= n2) return;
  const T dg = diag ? T(diag[l]) : T(0);
  T* o = out + b * osb + l * osl;
#pragma unroll 4
  for (int k = 0; k < kGT / 4; ++k) {
    const int ii = (tid >> 6) + 4 * k, i = i0 + ii;
    if (i >= n1) continue;
    T v = kernel_eval<MC, MF, T>(s, &sx1[ii * kMaxQ], &sx2[jj * kMaxQ], sp);
    if (i == j) v += dg;
    o[(int64_t)i * ldo + j] = v;
  }
}

// Adjoint, generic strided G (fp64), several Grams in one launch (the Hensman backward contracts
// four: K0xz, K0zz, K0_p with spec0 and B_p with spec1).  Stage 1: grid (chunks over all jobs, L),
// each workgroup takes kGBChunk consecutive elements of one job's [nb, n1, n2] G, accumulates the
// per-slot sums of g dk/dparam in registers, reduces them over its waves, and writes one partial
// row part[l][chunk][slot] (slot NS-1: sum of the diagonal of G, the noise adjoint).  Stage 2: one
// workgroup per latent dim sums the chunks of every (job, slot) and adds them to the job's dparams /
// ddiag in a fixed order -- deterministic, and no single-workgroup loop over the whole Gram.
constexpr int kGBMaxJobs = 4;
constexpr int kGBChunk = 1024;  // elements per workgroup (4 per thread)


struct GramBwdJobs {
  DevSpec s[2];
  GramBwdJob j[kGBMaxJobs];
  int njobs, total_chunks;
};

template <int MC, int MF>
__global__ __launch_bounds__(256) void gram_bwd_part_kernel(GramBwdJobs J, int L, double* __restrict__ part) {
  constexpr int NS = MC + MC * MF * 2 + 1;
  __shared__ double sp[64];
  __shared__ double wred[4][NS];
  const int c = blockIdx.x, l = blockIdx.y, tid = threadIdx.x;
  int jb = 0;
  while (jb + 1 < J.njobs && c >= J.j[jb + 1].chunk0) ++jb;
  const GramBwdJob& job = J.j[jb];
  const DevSpec& s = J.s[job.spec];
  if (tid < job.n_params) sp[tid] = job.params[(int64_t)l * job.n_params + tid];
  __syncthreads();
  double acc_s[MC];
  double acc_f[MC][MF][2];
#pragma unroll
  for (int r = 0; r < MC; ++r) {
    acc_s[r] = 0.0;
#pragma unroll
    for (int f = 0; f < MF; ++f) acc_f[r][f][0] = acc_f[r][f][1] = 0.0;
  }
  double dd = 0.0;
  const int64_t per_b = (int64_t)job.n1 * job.n2, total = per_b * job.nb;
  const int64_t e0 = (int64_t)(c - job.chunk0) * kGBChunk;
  for (int64_t e = e0 + tid; e < e0 + kGBChunk && e < total; e += 256) {
    const int b = (int)(e / per_b);
    const int64_t rem = e - b * per_b;
    const int i = (int)(rem / job.n2), j = (int)(rem - (int64_t)i * job.n2);
    const double g = job.G[b * job.gsb + l * job.gsl + i * job.ldg + j];
    if (g == 0.0) continue;
    const double* xi = job.x1.ptr + b * job.x1.stride_b + l * job.x1.stride_l + i * job.x1.ld;
    const double* xj = job.x2.ptr + b * job.x2.stride_b + l * job.x2.stride_l + j * job.x2.ld;
    kernel_grad_acc<MC, MF, double, double>(s, xi, xj, sp, g, acc_s, acc_f);
    if (i == j) dd += g;
  }
  const int w = tid >> 6, lane = tid & 63;
#pragma unroll
  for (int r = 0; r < MC; ++r) {
    const double v = wave_sum(acc_s[r]);
    if (lane == 0) wred[w][r] = v;
#pragma unroll
    for (int f = 0; f < MF; ++f)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const double u = wave_sum(acc_f[r][f][q]);
        if (lane == 0) wred[w][MC + (r * MF + f) * 2 + q] = u;
      }
  }
  {
    const double v = wave_sum(dd);
    if (lane == 0) wred[w][NS - 1] = v;
  }
  __syncthreads();
  double* out = part + ((int64_t)l * J.total_chunks + c) * NS;
  for (int sl = tid; sl < NS; sl += 256) out[sl] = wred[0][sl] + wred[1][sl] + wred[2][sl] + wred[3][sl];
}

template <int MC, int MF>
__global__ __launch_bounds__(256) void gram_bwd_sum_kernel(GramBwdJobs J, const double* __restrict__ part) {
  constexpr int NS = MC + MC * MF * 2 + 1;
  __shared__ double red[kGBMaxJobs][NS];
  const int l = blockIdx.x, tid = threadIdx.x;
  for (int t = tid; t < J.njobs * NS; t += 256) {
    const int jb = t / NS, sl = t % NS;
    const GramBwdJob& job = J.j[jb];
    double v = 0.0;
    for (int c = job.chunk0; c < job.chunk0 + job.nchunks; ++c) v += part[((int64_t)l * J.total_chunks + c) * NS + sl];
    red[jb][sl] = v;
  }
  __syncthreads();
  if (tid != 0) return;
  for (int jb = 0; jb < J.njobs; ++jb) {
    const GramBwdJob& job = J.j[jb];
    const DevSpec& s = J.s[job.spec];
    for (int sl = 0; sl < NS - 1; ++sl) {
      const int pi = slot_param<MC, MF>(s, sl);
      if (pi >= 0) job.dparams[(int64_t)l * job.n_params + pi] += red[jb][sl];
    }
    if (job.ddiag) job.ddiag[l] += red[jb][NS - 1];
  }
}

// ------------------------------------------------------------------------------------------
// Column-vectorised tile evaluation for the Regime B kernels.  Thread (w, jj) of a 256-thread
// workgroup owns column jj of a 64x64 tile and rows ii = w + 4k, k < 16.  The (uniform) spec is
// walked once per 16 elements instead of once per element, each factor is applied to all 16
// rows at once (row covariates are wave-uniform LDS broadcasts), and RBF factors use the native
// exp2 with a per-factor constant: ~30 VALU ops per element instead of a spec interpreter per
// element.  Category comparisons and covariate differences stay in fp64 (exact 0/1, as the
// reference's double compare).
// ------------------------------------------------------------------------------------------
constexpr int kTK = kGT / 4;  // rows per thread
constexpr float kLog2e = 1.4426950408889634f;

template <int MC, int MF>
__device__ __attribute__((always_inline)) inline void tile_kernel_f32(const DevSpec& s, const double* __restrict__ sx1, int ii0,
                                       const double* __restrict__ xj, const float* __restrict__ p,
                                       float (&out)[kTK]) {
#pragma unroll
  for (int k = 0; k < kTK; ++k) out[k] = 0.f;
#pragma unroll
  for (int r = 0; r < MC; ++r) {
    const bool on_r = r < s.n_comp;
    float prod[kTK];
    const float sc = p[s.scale_idx[r]];
#pragma unroll
    for (int k = 0; k < kTK; ++k) prod[k] = sc;
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      if (!on_r || f >= s.n_fac[r]) continue;
      const int d = s.dim[r][f];
      const double b = xj[d];
      const int kind = s.kind[r][f];
      if (kind == LVAE_CAT) {
#pragma unroll
        for (int k = 0; k < kTK; ++k) prod[k] = (sx1[(ii0 + 4 * k) * kMaxQ + d] == b) ? prod[k] : 0.f;
      } else if (kind == LVAE_BIN) {
#pragma unroll
        for (int k = 0; k < kTK; ++k) prod[k] = (sx1[(ii0 + 4 * k) * kMaxQ + d] + b == 2.0) ? prod[k] : 0.f;
      } else if (kind == LVAE_RBF) {
        const float ell = p[s.param_idx[r][f]];
        const float c = -0.5f * kLog2e / (ell * ell);
#pragma unroll
        for (int k = 0; k < kTK; ++k) {
          const float df = float(sx1[(ii0 + 4 * k) * kMaxQ + d] - b);
          prod[k] *= __builtin_amdgcn_exp2f(c * df * df);
        }
      } else if (kind == LVAE_PER) {
        const float ell = p[s.param_idx[r][f]], per = p[s.param_idx[r][f] + 1];
        const float c = -2.f * kLog2e / (ell * ell), w = float(M_PI) / per;
#pragma unroll
        for (int k = 0; k < kTK; ++k) {
          const float sn = sinf(w * float(fabs(sx1[(ii0 + 4 * k) * kMaxQ + d] - b)));
          prod[k] *= __builtin_amdgcn_exp2f(c * sn * sn);
        }
      } else {  // LVAE_LIN
#pragma unroll
        for (int k = 0; k < kTK; ++k) prod[k] *= float(sx1[(ii0 + 4 * k) * kMaxQ + d] * b);
      }
    }
    if (on_r) {
#pragma unroll
      for (int k = 0; k < kTK; ++k) out[k] += prod[k];
    }
  }
}

// acc_s[r] += sum_k g_k dk/dscale_r ; acc_f[r][f][q] += sum_k g_k dk/dparam_q(r,f)   (same walk as above;
// the factor derivatives are recomputed in a second pass so only prod[] stays live)
template <int MC, int MF>
__device__ __attribute__((always_inline)) inline void tile_kernel_grad_f32(const DevSpec& s, const double* __restrict__ sx1, int ii0,
                                            const double* __restrict__ xj, const float* __restrict__ p,
                                            const float (&g)[kTK], double* __restrict__ wrow, int lane) {
#pragma unroll
  for (int r = 0; r < MC; ++r) {
    const bool on_r = r < s.n_comp;
    float gp[kTK];
#pragma unroll
    for (int k = 0; k < kTK; ++k) gp[k] = g[k];
    // pass 1: gp = g * prod_f phi_f
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      if (!on_r || f >= s.n_fac[r]) continue;
      const int d = s.dim[r][f];
      const double b = xj[d];
      const int kind = s.kind[r][f];
      if (kind == LVAE_CAT) {
#pragma unroll
        for (int k = 0; k < kTK; ++k) gp[k] = (sx1[(ii0 + 4 * k) * kMaxQ + d] == b) ? gp[k] : 0.f;
      } else if (kind == LVAE_BIN) {
#pragma unroll
        for (int k = 0; k < kTK; ++k) gp[k] = (sx1[(ii0 + 4 * k) * kMaxQ + d] + b == 2.0) ? gp[k] : 0.f;
      } else if (kind == LVAE_RBF) {
        const float ell = p[s.param_idx[r][f]];
        const float c = -0.5f * kLog2e / (ell * ell);
#pragma unroll
        for (int k = 0; k < kTK; ++k) {
          const float df = float(sx1[(ii0 + 4 * k) * kMaxQ + d] - b);
          gp[k] *= __builtin_amdgcn_exp2f(c * df * df);
        }
      } else if (kind == LVAE_PER) {
        const float ell = p[s.param_idx[r][f]], per = p[s.param_idx[r][f] + 1];
        const float c = -2.f * kLog2e / (ell * ell), w = float(M_PI) / per;
#pragma unroll
        for (int k = 0; k < kTK; ++k) {
          const float sn = sinf(w * float(fabs(sx1[(ii0 + 4 * k) * kMaxQ + d] - b)));
          gp[k] *= __builtin_amdgcn_exp2f(c * sn * sn);
        }
      } else {
#pragma unroll
        for (int k = 0; k < kTK; ++k) gp[k] *= float(sx1[(ii0 + 4 * k) * kMaxQ + d] * b);
      }
    }
    float ts = 0.f;
#pragma unroll
    for (int k = 0; k < kTK; ++k) ts += gp[k];
    if (on_r) {
      const float v = wave_sum(ts);
      if (lane == 0) wrow[r] = v;
    }
    const float sc = p[s.scale_idx[r]];
    // pass 2: d log phi_f / d param for the parametrised factors
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      if (!on_r || f >= s.n_fac[r]) continue;
      const int kind = s.kind[r][f];
      if (kind != LVAE_RBF && kind != LVAE_PER) { } else {
      const int d = s.dim[r][f];
      const double b = xj[d];
      const float ell = p[s.param_idx[r][f]];
      float t0 = 0.f, t1 = 0.f;
      if (kind == LVAE_RBF) {
#pragma unroll
        for (int k = 0; k < kTK; ++k) {
          const float df = float(sx1[(ii0 + 4 * k) * kMaxQ + d] - b);
          t0 += gp[k] * df * df;
        }
        const float v = wave_sum(sc * t0 / (ell * ell * ell));
        if (lane == 0) wrow[MC + (r * MF + f) * 2] = v;
      } else {
        const float per = p[s.param_idx[r][f] + 1], w = float(M_PI) / per;
#pragma unroll
        for (int k = 0; k < kTK; ++k) {
          const float ad = float(fabs(sx1[(ii0 + 4 * k) * kMaxQ + d] - b));
          const float u = w * ad, sn = sinf(u);
          t0 += gp[k] * sn * sn;
          t1 += gp[k] * ad * sinf(2.f * u);
        }
        const float v0 = wave_sum(sc * 4.f * t0 / (ell * ell * ell));
        const float v1 = wave_sum(sc * 2.f * float(M_PI) * t1 / (ell * ell * per * per));
        if (lane == 0) {
          wrow[MC + (r * MF + f) * 2] = v0;
          wrow[MC + (r * MF + f) * 2 + 1] = v1;
        }
      }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// Regime B: lower-triangular tiles of the padded [np, np] covariance, f32 out, + noise on the
// diagonal, identity on the padding rows/cols (keeps log|K| and the leading block of K^-1).
// Tile t of the lower triangle -> (I, J), I >= J.
// ------------------------------------------------------------------------------------------
__device__ inline void tri_index(int t, int& I, int& J) {
  int r = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
  while ((r + 1) * (r + 2) / 2 <= t) ++r;
  while (r * (r + 1) / 2 > t) --r;
  I = r;
  J = t - r * (r + 1) / 2;
}

template <int MC, int MF>
__global__ __launch_bounds__(256) void gram_sq_fill_kernel(DevSpec s, const double* __restrict__ x, int ldx,
                                                           int n, int np_, int qs,
                                                           const double* __restrict__ params,
                                                           const double* __restrict__ noise,
                                                           float* __restrict__ K) {
  __shared__ double sx1[kGT * kMaxQ];
  __shared__ double sx2[kGT * kMaxQ];
  __shared__ float sp[64];
  int I, J;
  tri_index(blockIdx.x, I, J);
  const int l = blockIdx.y, tid = threadIdx.x;
  const int i0 = I * kGT, j0 = J * kGT;
  if (tid < s.n_params) sp[tid] = float(params[(int64_t)l * s.n_params + tid]);
  for (int e = tid; e < kGT * qs; e += 256) {
    const int r = e / qs, q = e % qs;
    sx1[r * kMaxQ + q] = (i0 + r < n) ? x[(int64_t)(i0 + r) * ldx + q] : 0.0;
    sx2[r * kMaxQ + q] = (j0 + r < n) ? x[(int64_t)(j0 + r) * ldx + q] : 0.0;
  }
  __syncthreads();
  const float nz = float(noise[l]);
  const int jj = tid & 63, j = j0 + jj, w = tid >> 6;
  float v[kTK];
  tile_kernel_f32<MC, MF>(s, sx1, w, &sx2[jj * kMaxQ], sp, v);
  float* o = K + (int64_t)l * np_ * np_;
#pragma unroll
  for (int k = 0; k < kTK; ++k) {
    const int i = i0 + w + 4 * k;
    float e = v[k];
    if (i == j) e += nz;
    if (i >= n || j >= n) e = (i == j) ? 1.0f : 0.0f;
    o[(int64_t)i * np_ + j] = e;
  }
}

// Fused adjoint for the exact KL: per lower 64x64 tile, G = 1/2 (Kinv - S - a a^T) is formed on the
// fly from the symmetric K^-1 (f32), S = K^-1 V K^-1 (f32, lower tiles) and a = K^-1 mu (f64);
// per-slot partial sums of sum_ij w_ij G_ij dK_ij/dtheta go to part[l][tile][slot]
// (w = 2 strictly below the diagonal, 1 on it).  Slot NS-1 holds sum_i G_ii (noise).
template <int MC, int MF>
__global__ __launch_bounds__(256) void kl_gram_bwd_tiles(DevSpec s, const double* __restrict__ x, int ldx, int n,
                                                         int np_, int qs, const double* __restrict__ params,
                                                         const float* __restrict__ Kinv,
                                                         const float* __restrict__ S,
                                                         const double* __restrict__ alpha,
                                                         double* __restrict__ part, int ntiles) {
  constexpr int NS = MC + MC * MF * 2 + 1;
  __shared__ double sx1[kGT * kMaxQ];
  __shared__ double sx2[kGT * kMaxQ];
  __shared__ float sp[64];
  __shared__ double sa1[kGT], sa2[kGT];
  int I, J;
  tri_index(blockIdx.x, I, J);
  const int l = blockIdx.y, tid = threadIdx.x;
  const int i0 = I * kGT, j0 = J * kGT;
  if (tid < s.n_params) sp[tid] = float(params[(int64_t)l * s.n_params + tid]);
  for (int e = tid; e < kGT * qs; e += 256) {
    const int r = e / qs, q = e % qs;
    sx1[r * kMaxQ + q] = (i0 + r < n) ? x[(int64_t)(i0 + r) * ldx + q] : 0.0;
    sx2[r * kMaxQ + q] = (j0 + r < n) ? x[(int64_t)(j0 + r) * ldx + q] : 0.0;
  }
  if (tid < kGT) sa1[tid] = alpha[(int64_t)l * np_ + i0 + tid];
  else if (tid < 2 * kGT) sa2[tid - kGT] = alpha[(int64_t)l * np_ + j0 + tid - kGT];
  __shared__ double wred[4][NS];
  for (int e = tid; e < 4 * NS; e += 256) (&wred[0][0])[e] = 0.0;
  __syncthreads();
  float dd = 0.f;
  const int jj = tid & 63, j = j0 + jj, wv = tid >> 6;
  const float* ki = Kinv + (int64_t)l * np_ * np_;
  const float* si = S + (int64_t)l * np_ * np_;
  float g[kTK];
#pragma unroll
  for (int k = 0; k < kTK; ++k) {
    const int ii = wv + 4 * k, i = i0 + ii;
    const int64_t o = (int64_t)i * np_ + j;
    float gv = 0.5f * (ki[o] - si[o] - float(sa1[ii] * sa2[jj]));
    const bool in = i < n && j < n && j <= i;
    if (i == j && in) dd += gv;
    g[k] = in ? ((i == j) ? gv : 2.f * gv) : 0.f;
  }
  // per-slot wave sums land in wred[wave][slot] (unused slots stay 0) -> 4-wave sum per tile
  const int lane = tid & 63;
  tile_kernel_grad_f32<MC, MF>(s, sx1, wv, &sx2[jj * kMaxQ], sp, g, wred[wv], lane);
  {
    const float v = wave_sum(dd);
    if (lane == 0) wred[wv][NS - 1] = v;
  }
  __syncthreads();
  for (int sl = tid; sl < NS; sl += 256)
    part[((int64_t)l * NS + sl) * ntiles + blockIdx.x] = wred[0][sl] + wred[1][sl] + wred[2][sl] + wred[3][sl];
}

// Reduce the tile partials: dparams[l, p(slot)] = gkl[l] * sum over tiles, dnoise[l] (slot NS-1).
// Partials are laid out [l][slot][tile] (coalesced sums); one workgroup per (slot, l).  Every
// parameter has exactly one slot (slot_param is injective), so the writes never collide.
template <int MC, int MF>
__global__ __launch_bounds__(256) void kl_gram_bwd_reduce(DevSpec s, const double* __restrict__ part, int ntiles,
                                                          const double* __restrict__ gkl,
                                                          double* __restrict__ dparams,
                                                          double* __restrict__ dnoise) {
  constexpr int NS = MC + MC * MF * 2 + 1;
  __shared__ double red[4];
  const int slot = blockIdx.x, l = blockIdx.y, tid = threadIdx.x;
  const int pi = slot == NS - 1 ? -2 : slot_param<MC, MF>(s, slot);
  if (pi == -1) return;  // an unused slot (uniform over the workgroup)
  const double* p = part + ((int64_t)l * NS + slot) * ntiles;
  double v = 0.0;
  for (int t = tid; t < ntiles; t += 256) v += p[t];
  v = block_sum<256>(v, red);
  if (tid == 0) {
    if (pi == -2) {
      if (dnoise) dnoise[l] = gkl[l] * v;
    } else {
      dparams[(int64_t)l * s.n_params + pi] = gkl[l] * v;
    }
  }
}

// ------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------
static int spec_qs(const lvae_kernel_spec* s) {
  int q = 0;
  for (int r = 0; r < s->n_comp; ++r)
    for (int f = 0; f < s->n_fac[r]; ++f) q = s->dim[r][f] + 1 > q ? s->dim[r][f] + 1 : q;
  return q;
}

template <typename T>
static int gram_launch(const lvae_kernel_spec* spec, lvae_xview x1, lvae_xview x2, int nb, int L, int n1, int n2,
                       const double* params, const double* diag, T* out, int64_t osb, int64_t osl, int64_t ldo,
                       void* stream) {
  const int bucket = spec_bucket(spec);
  if (!bucket) return -1;
  const int qs = spec_qs(spec);
  if (qs > kMaxQ) return -1;
  if (nb < 1 || L < 1 || n1 < 0 || n2 < 0) return -4;
  if (n1 == 0 || n2 == 0) return 0;
  const DevSpec ds = to_dev(spec);
  dim3 grid(cdiv(n2, kGT), cdiv(n1, kGT), nb * L), block(256);
  hipStream_t st = (hipStream_t)stream;
  if (bucket == 1)
    gram_kernel<8, 2, T><<<grid, block, 0, st>>>(ds, x1, x2, L, n1, n2, qs, params, diag, out, osb, osl, ldo);
  else
    gram_kernel<16, 4, T><<<grid, block, 0, st>>>(ds, x1, x2, L, n1, n2, qs, params, diag, out, osb, osl, ldo);
  LVAE_CHECK_LAUNCH();
  return 0;
}

int kl_gram_fill(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int np_, int L,
                 const double* params, const double* noise, float* K, hipStream_t st) {
  const int bucket = spec_bucket(spec);
  const int qs = spec_qs(spec);
  if (!bucket || qs > kMaxQ || qs > ldx) return -1;
  const DevSpec ds = to_dev(spec);
  const int nt = np_ / kGT;
  dim3 grid(nt * (nt + 1) / 2, L);
  if (bucket == 1)
    gram_sq_fill_kernel<8, 2><<<grid, 256, 0, st>>>(ds, x, ldx, n, np_, qs, params, noise, K);
  else
    gram_sq_fill_kernel<16, 4><<<grid, 256, 0, st>>>(ds, x, ldx, n, np_, qs, params, noise, K);
  LVAE_CHECK_LAUNCH();
  return 0;
}

size_t kl_gram_bwd_partials_bytes(int np_, int L) {
  const int nt = np_ / kGT;
  return (size_t)L * (nt * (nt + 1) / 2) * (16 + 16 * 4 * 2 + 1) * sizeof(double);
}

int kl_gram_bwd(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int np_, int L,
                const double* params, const float* Kinv, const float* S, const double* alpha, const double* gkl,
                double* part, double* dparams, double* dnoise, hipStream_t st) {
  const int bucket = spec_bucket(spec);
  const int qs = spec_qs(spec);
  if (!bucket || qs > kMaxQ) return -1;
  const DevSpec ds = to_dev(spec);
  const int nt = np_ / kGT, ntiles = nt * (nt + 1) / 2;
  dim3 grid(ntiles, L);
  if (bucket == 1) {
    kl_gram_bwd_tiles<8, 2><<<grid, 256, 0, st>>>(ds, x, ldx, n, np_, qs, params, Kinv, S, alpha, part, ntiles);
    kl_gram_bwd_reduce<8, 2><<<dim3(8 + 8 * 2 * 2 + 1, L), 256, 0, st>>>(ds, part, ntiles, gkl, dparams, dnoise);
  } else {
    kl_gram_bwd_tiles<16, 4><<<grid, 256, 0, st>>>(ds, x, ldx, n, np_, qs, params, Kinv, S, alpha, part, ntiles);
    kl_gram_bwd_reduce<16, 4><<<dim3(16 + 16 * 4 * 2 + 1, L), 256, 0, st>>>(ds, part, ntiles, gkl, dparams, dnoise);
  }
  LVAE_CHECK_LAUNCH();
  return 0;
}

// Adjoints of up to kGBMaxJobs Grams in two launches (see gram_bwd_part_kernel); `jobs` hold
// host-side descriptors whose .spec indexes specs[0..1].  part: gram_bwd_part_bytes(...) bytes.
size_t gram_bwd_part_bytes(const GramBwdJob* jobs, int njobs, int L) {
  int64_t chunks = 0;
  for (int q = 0; q < njobs; ++q) chunks += cdiv((int64_t)jobs[q].nb * jobs[q].n1 * jobs[q].n2, kGBChunk);
  return (size_t)L * (size_t)(chunks > 0 ? chunks : 1) * (16 + 16 * 4 * 2 + 1) * sizeof(double);
}

int gram_bwd_multi_f64(const lvae_kernel_spec* const* specs, const GramBwdJob* jobs, int njobs, int L, double* part,
                       hipStream_t st) {
  if (njobs < 1 || njobs > kGBMaxJobs || L < 1) return -4;
  GramBwdJobs J;
  int bucket = 1;
  for (int q = 0; q < 2; ++q) {
    if (!specs[q]) {
      J.s[q] = J.s[0];
      continue;
    }
    const int bk = spec_bucket(specs[q]);
    if (!bk) return -1;
    bucket = bk > bucket ? bk : bucket;
    J.s[q] = to_dev(specs[q]);
  }
  int chunks = 0;
  for (int q = 0; q < njobs; ++q) {
    J.j[q] = jobs[q];
    J.j[q].n_params = specs[jobs[q].spec]->n_params;
    J.j[q].chunk0 = chunks;
    J.j[q].nchunks = cdiv((int64_t)jobs[q].nb * jobs[q].n1 * jobs[q].n2, kGBChunk);
    chunks += J.j[q].nchunks;
  }
  J.njobs = njobs;
  J.total_chunks = chunks;
  if (chunks == 0) return 0;
  if (bucket == 1) {
    gram_bwd_part_kernel<8, 2><<<dim3(chunks, L), 256, 0, st>>>(J, L, part);
    gram_bwd_sum_kernel<8, 2><<<L, 256, 0, st>>>(J, part);
  } else {
    gram_bwd_part_kernel<16, 4><<<dim3(chunks, L), 256, 0, st>>>(J, L, part);
    gram_bwd_sum_kernel<16, 4><<<L, 256, 0, st>>>(J, part);
  }
  LVAE_CHECK_LAUNCH();
  return 0;
}

}  // namespace lvae

extern "C" {

int lvae_gram_f64(const lvae_kernel_spec* spec, lvae_xview x1, lvae_xview x2, int nb, int L, int n1, int n2,
                  const double* params, const double* diag, double* out, int64_t osb, int64_t osl, int64_t ldo,
                  void* stream) {
  return lvae::gram_launch<double>(spec, x1, x2, nb, L, n1, n2, params, diag, out, osb, osl, ldo, stream);
}

int lvae_gram_f32(const lvae_kernel_spec* spec, lvae_xview x1, lvae_xview x2, int nb, int L, int n1, int n2,
                  const double* params, const double* diag, float* out, int64_t osb, int64_t osl, int64_t ldo,
                  void* stream) {
  return lvae::gram_launch<float>(spec, x1, x2, nb, L, n1, n2, params, diag, out, osb, osl, ldo, stream);
}

size_t lvae_gram_bwd_workspace_size(int nb, int L, int n1, int n2) {
  lvae::GramBwdJob j{};
  j.nb = nb, j.n1 = n1, j.n2 = n2;
  return lvae::gram_bwd_part_bytes(&j, 1, L);
}

int lvae_gram_bwd_f64(const lvae_kernel_spec* spec, lvae_xview x1, lvae_xview x2, int nb, int L, int n1, int n2,
                      const double* params, const double* G, int64_t gsb, int64_t gsl, int64_t ldg, double* dparams,
                      double* ddiag, void* workspace, void* stream) {
  if (!spec) return -1;
  if (nb < 1 || L < 1 || n1 < 0 || n2 < 0) return -4;
  if (!params) return -8;
  if (!G) return -9;
  if (!dparams) return -13;
  if (!workspace) return -15;
  lvae::GramBwdJob j{};
  j.spec = 0, j.x1 = x1, j.x2 = x2, j.nb = nb, j.n1 = n1, j.n2 = n2, j.params = params, j.G = G;
  j.gsb = gsb, j.gsl = gsl, j.ldg = ldg, j.dparams = dparams, j.ddiag = ddiag;
  const lvae_kernel_spec* specs[2] = {spec, nullptr};
  return lvae::gram_bwd_multi_f64(specs, &j, 1, L, (double*)workspace, (hipStream_t)stream);
}

}  // extern "C"
