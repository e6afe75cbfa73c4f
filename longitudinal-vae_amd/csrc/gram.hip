// gram.hip -- additive-kernel Gram assembly and its adjoint (GP_model.py:31-144; kernel_gen.py:9-310).
//
// Forward: one 256-thread workgroup per 64x64 output tile of one (batch, latent-dim) slice; the two
// covariate row blocks are staged in LDS (coalesced fp64 reads of the [n, Q] index arrays), each
// thread produces 16 elements of one column (consecutive lanes -> consecutive columns, so the
// stores are coalesced).  The Gram is HBM-write-bound: per element 4 B (f32) / 8 B (f64) out.
#include "gram_bwd.hpp"
#include "gram_tab.hpp"

namespace lvae {

constexpr int kGT = 64;     // Gram tile edge
constexpr int kMaxQ = 32;   // staged covariate columns

// The RBF / periodic factor of an integer distance m < kGTab, evaluated once per workgroup into an LDS
// table with kernel_eval's own expression (so a table read equals the direct evaluation bit for bit): the
// covariates of the reference's data (time points, ages) are integer-coded, and the Hensman Grams are
// small tiles where the exp / sin per element and component dominated.
constexpr int kGTab = 64;
template <int MC, int MF, typename T>
__device__ inline T factor_at(const DevSpec& s, int r, int f, const T* __restrict__ p, T ad) {
  const T ell = p[s.param_idx[r][f]];
  if (s.kind[r][f] == LVAE_RBF) return exp(-(ad * ad) / (T(2) * ell * ell));
  const T per = p[s.param_idx[r][f] + 1];
  const T sn = sin(T(M_PI) * ad / per);
  return exp(T(-2) * sn * sn / (ell * ell));
}

template <int MC, int MF, typename T>
__device__ inline T kernel_eval_tab(const DevSpec& s, const double* __restrict__ xi, const double* __restrict__ xj,
                                    const T* __restrict__ p, const T* __restrict__ tab) {
  T sum = T(0);
#pragma unroll
  for (int r = 0; r < MC; ++r) {
    if (r < s.n_comp) {
      T prod = p[s.scale_idx[r]];
#pragma unroll
      for (int f = 0; f < MF; ++f) {
        if (f < s.n_fac[r]) {
          const int d = s.dim[r][f];
          const double a = xi[d], b = xj[d];
          const int k = s.kind[r][f];
          if (k == LVAE_CAT) {
            prod = (a - b == 0.0) ? prod : T(0);
          } else if (k == LVAE_BIN) {
            prod = (a + b == 2.0) ? prod : T(0);
          } else if (k == LVAE_RBF || k == LVAE_PER) {
            const double ad = fabs(a - b);
            prod *= (ad < (double)kGTab && ad == floor(ad)) ? tab[(r * MF + f) * kGTab + (int)ad]
                                                            : factor_at<MC, MF, T>(s, r, f, p, T(ad));
          } else {
            prod *= T(a * b);  // LVAE_LIN
          }
        }
      }
      sum += prod;
    }
  }
  return sum;
}

// one 64 x 64 output block (bx, by) of Gram bz = b * L + l
template <int MC, int MF, typename T>
__device__ __attribute__((always_inline)) inline void gram_block(const DevSpec& s, const lvae_xview& x1,
                                                                 const lvae_xview& x2, int L, int n1, int n2, int qs,
                                                                 const double* __restrict__ params,
                                                                 const double* __restrict__ diag, T* __restrict__ out,
                                                                 int64_t osb, int64_t osl, int64_t ldo, int bx, int by,
                                                                 int bz) {
  __shared__ double sx1[kGT * kMaxQ];
  __shared__ double sx2[kGT * kMaxQ];
  __shared__ T sp[64];
  __shared__ T tab[MC * MF * kGTab];
  const int bl = bz, b = bl / L, l = bl % L;
  const int i0 = by * kGT, j0 = bx * kGT;
  const int tid = threadIdx.x;
  if (tid < s.n_params) sp[tid] = T(params[(int64_t)l * s.n_params + tid]);
  __syncthreads();
  for (int e = tid; e < MC * MF * kGTab; e += 256) {
    const int r = e / (MF * kGTab), f = (e / kGTab) % MF, m = e % kGTab;
    T v = T(0);
    if (r < s.n_comp && f < s.n_fac[r] && (s.kind[r][f] == LVAE_RBF || s.kind[r][f] == LVAE_PER))
      v = factor_at<MC, MF, T>(s, r, f, sp, T(m));
    tab[e] = v;
  }
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
    T v = kernel_eval_tab<MC, MF, T>(s, &sx1[ii * kMaxQ], &sx2[jj * kMaxQ], sp, tab);
    if (i == j) v += dg;
    o[(int64_t)i * ldo + j] = v;
  }
}

template <int MC, int MF, typename T>
__global__ __launch_bounds__(256) void gram_kernel(DevSpec s, lvae_xview x1, lvae_xview x2, int L, int n1, int n2,
                                                   int qs, const double* __restrict__ params,
                                                   const double* __restrict__ diag, T* __restrict__ out,
                                                   int64_t osb, int64_t osl, int64_t ldo) {
  gram_block<MC, MF, T>(s, x1, x2, L, n1, n2, qs, params, diag, out, osb, osl, ldo, blockIdx.x, blockIdx.y,
                        blockIdx.z);
}

// several fp64 Grams in one launch (the Hensman forward's four: K0xz, K0zz, K0_p with spec0, B_p with
// spec1): a 1-D grid over every job's blocks, block r of job q at (r % gx, r / gx % gy, r / (gx gy))
constexpr int kGFMaxJobs = 4;
struct GramFwdJobs {
  DevSpec s[2];
  int qs[2];
  GramFwdJob j[kGFMaxJobs];
  int njobs;
};

template <int MC, int MF>
__global__ __launch_bounds__(256) void gram_multi_kernel(GramFwdJobs J, int L) {
  int q = 0;
  while (q + 1 < J.njobs && (int)blockIdx.x >= J.j[q + 1].blk0) ++q;  // (uniform)
  const GramFwdJob& jb = J.j[q];
  const int r = blockIdx.x - jb.blk0;
  gram_block<MC, MF, double>(J.s[jb.spec], jb.x1, jb.x2, L, jb.n1, jb.n2, J.qs[jb.spec], jb.params, jb.diag, jb.out,
                             jb.osb, jb.osl, jb.ldo, r % jb.gx, (r / jb.gx) % jb.gy, r / (jb.gx * jb.gy));
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

// kernel_grad_acc with the factors of integer distances m < kGTab read from per-workgroup tables of phi(m),
// and for periodic factors sin(u) and sin(2u) (u = pi m / p), each with kernel_grad_acc's own expression:
// bit-identical to it, without the exp / sin per element and component
template <int MC, int MF>
__device__ inline void kernel_grad_acc_tab(const DevSpec& s, const double* __restrict__ xi,
                                           const double* __restrict__ xj, const double* __restrict__ p, double g,
                                           double (&acc_s)[MC], double (&acc_f)[MC][MF][2],
                                           const double* __restrict__ tphi, const double* __restrict__ tsn,
                                           const double* __restrict__ ts2) {
#pragma unroll
  for (int r = 0; r < MC; ++r) {
    if (r < s.n_comp) {
      double prod = 1.0;
      double dlog[MF][2];
#pragma unroll
      for (int f = 0; f < MF; ++f) {
        dlog[f][0] = 0.0;
        dlog[f][1] = 0.0;
        if (f >= s.n_fac[r]) continue;
        const int d = s.dim[r][f];
        const double a = xi[d], b = xj[d];
        const int k = s.kind[r][f];
        if (k == LVAE_CAT) {
          prod = (a - b == 0.0) ? prod : 0.0;
        } else if (k == LVAE_BIN) {
          prod = (a + b == 2.0) ? prod : 0.0;
        } else if (k == LVAE_RBF || k == LVAE_PER) {
          const double ad = fabs(a - b);
          const bool hit = ad < (double)kGTab && ad == floor(ad);
          const int ti = (r * MF + f) * kGTab + (hit ? (int)ad : 0);
          const double ell = p[s.param_idx[r][f]];
          if (k == LVAE_RBF) {
            const double diff = a - b, d2 = diff * diff;
            prod *= hit ? tphi[ti] : exp(-d2 / (2.0 * ell * ell));
            dlog[f][0] = d2 / (ell * ell * ell);
          } else {
            const double per = p[s.param_idx[r][f] + 1];
            const double u = M_PI * ad / per;
            const double sn = hit ? tsn[ti] : sin(u);
            prod *= hit ? tphi[ti] : exp(-2.0 * sn * sn / (ell * ell));
            dlog[f][0] = 4.0 * sn * sn / (ell * ell * ell);
            dlog[f][1] = 2.0 * M_PI * ad * (hit ? ts2[ti] : sin(2.0 * u)) / (ell * ell * per * per);
          }
        } else {
          prod *= a * b;  // LVAE_LIN
        }
      }
      const double gp = g * prod;
      acc_s[r] += gp;
      const double gc = gp * p[s.scale_idx[r]];
#pragma unroll
      for (int f = 0; f < MF; ++f) {
        acc_f[r][f][0] += gc * dlog[f][0];
        acc_f[r][f][1] += gc * dlog[f][1];
      }
    }
  }
}

template <int MC, int MF>
__global__ __launch_bounds__(256) void gram_bwd_part_kernel(GramBwdJobs J, int L, double* __restrict__ part) {
  constexpr int NS = MC + MC * MF * 2 + 1;
  constexpr bool kTab = MC * MF <= 16;  // (the tables: 3 x 8 KB at the small bucket)
  constexpr int NT = kTab ? MC * MF * kGTab : 1;
  __shared__ double sp[64];
  __shared__ double wred[4][NS];
  __shared__ double tphi[NT], tsn[NT], ts2[NT];
  const int c = blockIdx.x, l = blockIdx.y, tid = threadIdx.x;
  int jb = 0;
  while (jb + 1 < J.njobs && c >= J.j[jb + 1].chunk0) ++jb;
  const GramBwdJob& job = J.j[jb];
  const DevSpec& s = J.s[job.spec];
  if (tid < job.n_params) sp[tid] = job.params[(int64_t)l * job.n_params + tid];
  __syncthreads();
  if (kTab) {
    for (int e = tid; e < NT; e += 256) {
      const int r = e / (MF * kGTab), f = (e / kGTab) % MF, m = e % kGTab;
      double phi = 0.0, sn = 0.0, s2 = 0.0;
      if (r < s.n_comp && f < s.n_fac[r]) {
        const double ell = sp[s.param_idx[r][f]], ad = (double)m;
        if (s.kind[r][f] == LVAE_RBF) {
          phi = exp(-(ad * ad) / (2.0 * ell * ell));
        } else if (s.kind[r][f] == LVAE_PER) {
          const double per = sp[s.param_idx[r][f] + 1], u = M_PI * ad / per;
          sn = sin(u);
          phi = exp(-2.0 * sn * sn / (ell * ell));
          s2 = sin(2.0 * u);
        }
      }
      tphi[e] = phi;
      tsn[e] = sn;
      ts2[e] = s2;
    }
    __syncthreads();
  }
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
    if (kTab)
      kernel_grad_acc_tab<MC, MF>(s, xi, xj, sp, g, acc_s, acc_f, tphi, tsn, ts2);
    else
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
// Regime B Gram tiles, 4 x 4 micro-tiles.  A 256-thread workgroup owns a 64 x 64 tile; thread
// (tr, tc) = (tid >> 4, tid & 15) owns rows 4 tr + a and columns 4 tc + c (a, c < 4): per factor
// it reads 4 row and 4 column covariates (fp64, LDS) for 16 elements and the tile rows go out /
// come in as float4 (16 B per lane, 256 contiguous bytes per row and 16 lanes).  The (uniform)
// spec is walked once per 16 elements.  Category / binary tests and covariate differences stay in
// fp64 (exact 0/1 and exact differences, as the reference's double arithmetic); factor values,
// products and sums are fp32 (the covariance is fp32); RBF / periodic use the native exp2.
// ------------------------------------------------------------------------------------------
typedef float g_f32x4 __attribute__((ext_vector_type(4)));

__device__ inline void tri_index(int t, int& I, int& J) {
  int r = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
  while ((r + 1) * (r + 2) / 2 <= t) ++r;
  while (r * (r + 1) / 2 > t) --r;
  I = r;
  J = t - r * (r + 1) / 2;
}

// stage the covariates of rows [i0, i0 + 64) and [j0, j0 + 64) (zero beyond n) into LDS.  Layout
// [dim][slot]: row r of the tile sits at slot (r & 3) * 16 + (r >> 2), so the 16 lanes that read
// rows 4 tc + c (c fixed) touch 16 consecutive doubles -- conflict-free ds_read_b64 (a row-major
// [row][dim] image puts those 16 reads on one bank pair: 16-way conflicts).
constexpr int kMaxQB = 16;  // covariate columns the Regime B kernels stage (spec dims < 16)
__device__ inline int cov_slot(int r) { return (r & 3) * 16 + (r >> 2); }
template <typename CT>
__device__ inline void stage_cov(const double* __restrict__ x, int ldx, int n, int qs, int i0, int j0,
                                 CT* __restrict__ sx1, CT* __restrict__ sx2) {
  for (int e = threadIdx.x; e < kGT * qs; e += 256) {
    const int r = e / qs, q = e % qs;
    sx1[q * kGT + cov_slot(r)] = CT((i0 + r < n) ? x[(int64_t)(i0 + r) * ldx + q] : 0.0);
    sx2[q * kGT + cov_slot(r)] = CT((j0 + r < n) ? x[(int64_t)(j0 + r) * ldx + q] : 0.0);
  }
}

// Integer-coded covariates (the common case: subject / time / class indices) take an fp32 path in the
// Regime B Gram kernels: covariates staged as fp32, category / binary tests and differences in fp32 --
// exact, and bitwise the same Gram, when every covariate is an integer of magnitude < 2^22 (the
// fp64 path rounds the exact fp64 difference to fp32 as well).  One workgroup, written by the factor for
// its kernels: flag 0 = not integer-coded (fp64 covariates), 1 = integer-coded, 2 = integer-coded and
// every dim of tabmask spans < kTabD values (the table path, gram_tab_*; tab_ok: the spec allows it).
__global__ __launch_bounds__(1024) void cov_int_check_kernel(const double* __restrict__ x, int ldx, int n, int qs,
                                                             int tab_ok, int tabmask, int* __restrict__ flag) {
  __shared__ int bad, wide;
  __shared__ int lo[kMaxQB], hi[kMaxQB];
  if (threadIdx.x == 0) bad = wide = 0;
  if (threadIdx.x < kMaxQB) {
    lo[threadIdx.x] = INT_MAX;
    hi[threadIdx.x] = INT_MIN;
  }
  __syncthreads();
  int b = 0;
  for (int q = 0; q < qs; ++q) {
    int mn = INT_MAX, mx = INT_MIN;
    for (int r = threadIdx.x; r < n; r += 1024) {
      const double v = x[(int64_t)r * ldx + q];
      const bool ok = v == rint(v) && fabs(v) < 4194304.0;
      b |= !ok;
      if (ok) {
        mn = min(mn, (int)v);
        mx = max(mx, (int)v);
      }
    }
    if ((tabmask >> q) & 1) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        mn = min(mn, __shfl_xor(mn, o, 64));
        mx = max(mx, __shfl_xor(mx, o, 64));
      }
      if ((threadIdx.x & 63) == 0) {
        atomicMin(&lo[q], mn);
        atomicMax(&hi[q], mx);
      }
    }
  }
  if (__any(b) && (threadIdx.x & 63) == 0) atomicOr(&bad, 1);
  __syncthreads();
  if (threadIdx.x < qs && ((tabmask >> threadIdx.x) & 1) && hi[threadIdx.x] - lo[threadIdx.x] >= kTabD)
    atomicOr(&wide, 1);
  __syncthreads();
  if (threadIdx.x == 0) *flag = bad ? 0 : (tab_ok && !wide ? 2 : 1);
}


// factor (kind, dim d, params pf) on the thread's 4 x 4 micro-tile: v[a][c] *= phi(x_i, x_j)
template <typename CT>
__device__ inline void apply_factor(int kind, int d, const float* __restrict__ pf, const CT* __restrict__ sx1,
                                    const CT* __restrict__ sx2, int tr, int tc, float (&v)[4][4]) {
  CT xr[4], xc[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) xr[a] = sx1[d * kGT + a * 16 + tr];
#pragma unroll
  for (int c = 0; c < 4; ++c) xc[c] = sx2[d * kGT + c * 16 + tc];
  if (kind == LVAE_CAT) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) v[a][c] = (xr[a] == xc[c]) ? v[a][c] : 0.f;
  } else if (kind == LVAE_BIN) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) v[a][c] = (xr[a] + xc[c] == CT(2)) ? v[a][c] : 0.f;
  } else if (kind == LVAE_RBF) {
    const float ell = pf[0], cf = -0.5f * kLog2e / (ell * ell);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float df = float(xr[a] - xc[c]);
        v[a][c] *= __builtin_amdgcn_exp2f(cf * df * df);
      }
  } else if (kind == LVAE_PER) {
    const float ell = pf[0], cf = -2.f * kLog2e / (ell * ell);
    const double ip = 1.0 / (double)pf[1];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float sn = per_sin(fabs(double(xr[a]) - double(xc[c])) * ip);
        v[a][c] *= __builtin_amdgcn_exp2f(cf * sn * sn);
      }
  } else {  // LVAE_LIN
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) v[a][c] *= float(double(xr[a]) * double(xc[c]));
  }
}

// component r's factors on the micro-tile, Cat / Bin gates first: when they leave the whole WAVE at zero
// (e.g. Cat(subject) on a tile pair of different subjects) the parametrised factors (exp / sin) are
// skipped and false returned (v is then 0: the component adds nothing; wave-uniform, no divergence)
template <typename CT>
__device__ inline bool apply_factors_gated(const DevSpec& s, int r, const float* __restrict__ sp,
                                           const CT* __restrict__ sx1, const CT* __restrict__ sx2, int tr,
                                           int tc, float (&v)[4][4]) {
  bool gated = false;
#pragma unroll 1
  for (int f = 0; f < s.n_fac[r]; ++f) {
    const int kind = s.kind[r][f];
    if (kind != LVAE_CAT && kind != LVAE_BIN) continue;
    apply_factor(kind, s.dim[r][f], sp, sx1, sx2, tr, tc, v);
    gated = true;
  }
  if (gated) {
    bool any = false;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) any |= v[a][c] != 0.f;
    if (!__any(any)) return false;
  }
#pragma unroll 1
  for (int f = 0; f < s.n_fac[r]; ++f) {
    const int kind = s.kind[r][f];
    if (kind == LVAE_CAT || kind == LVAE_BIN) continue;
    const int pi = s.param_idx[r][f];
    apply_factor(kind, s.dim[r][f], sp + (pi < 0 ? 0 : pi), sx1, sx2, tr, tc, v);
  }
  return true;
}

// the adjoint's per-factor sums over the micro-tile: u0 = sum v d^2 (RBF) or sum v sin^2 u (PER),
// u1 = sum v |d| sin 2u (PER); the ingredients are recomputed so only v stays live
template <typename CT>
__device__ inline void factor_sums(int kind, int d, const float* __restrict__ pf, const CT* __restrict__ sx1,
                                   const CT* __restrict__ sx2, int tr, int tc, const float (&v)[4][4], float& u0,
                                   float& u1) {
  CT xr[4], xc[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) xr[a] = sx1[d * kGT + a * 16 + tr];
#pragma unroll
  for (int c = 0; c < 4; ++c) xc[c] = sx2[d * kGT + c * 16 + tc];
  u0 = u1 = 0.f;
  if (kind == LVAE_RBF) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float df = float(xr[a] - xc[c]);
        u0 += v[a][c] * df * df;
      }
  } else {  // LVAE_PER
    const double ip = 1.0 / (double)pf[1];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const double ad = fabs(double(xr[a]) - double(xc[c])), t = ad * ip;
        const float sn = per_sin(t);
        u0 += v[a][c] * sn * sn;
        u1 += v[a][c] * float(ad) * per_sin2(t);
      }
  }
}

// covariate prefetch: each thread carries up to kPre (row, dim) values of the next tile's two
// row blocks in registers while the current tile is evaluated
constexpr int kPre = (kGT * kMaxQB + 255) / 256;
struct CovPrefetch {
  double a[kPre], b[kPre];
  __device__ inline void load(const double* __restrict__ x, int ldx, int n, int qs, int i0, int j0) {
#pragma unroll
    for (int u = 0; u < kPre; ++u) {
      const int e = threadIdx.x + 256 * u, r = e / qs, q = e % qs;
      const bool ok = e < kGT * qs;
      a[u] = (ok && i0 + r < n) ? x[(int64_t)(i0 + r) * ldx + q] : 0.0;
      b[u] = (ok && j0 + r < n) ? x[(int64_t)(j0 + r) * ldx + q] : 0.0;
    }
  }
  template <typename CT>
  __device__ inline void store(int qs, CT* __restrict__ sx1, CT* __restrict__ sx2) const {
#pragma unroll
    for (int u = 0; u < kPre; ++u) {
      const int e = threadIdx.x + 256 * u, r = e / qs, q = e % qs;
      if (e < kGT * qs) {
        sx1[q * kGT + cov_slot(r)] = CT(a[u]);
        sx2[q * kGT + cov_slot(r)] = CT(b[u]);
      }
    }
  }
};

// the same for integer-coded covariates (flag >= 1: exact in fp32), half the registers
struct CovPrefetchF {
  float a[kPre], b[kPre];
  __device__ inline void load(const double* __restrict__ x, int ldx, int n, int qs, int i0, int j0) {
#pragma unroll
    for (int u = 0; u < kPre; ++u) {
      const int e = threadIdx.x + 256 * u, r = e / qs, q = e % qs;
      const bool ok = e < kGT * qs;
      a[u] = (ok && i0 + r < n) ? float(x[(int64_t)(i0 + r) * ldx + q]) : 0.f;
      b[u] = (ok && j0 + r < n) ? float(x[(int64_t)(j0 + r) * ldx + q]) : 0.f;
    }
  }
  __device__ inline void store(int qs, float* __restrict__ sx1, float* __restrict__ sx2) const {
#pragma unroll
    for (int u = 0; u < kPre; ++u) {
      const int e = threadIdx.x + 256 * u, r = e / qs, q = e % qs;
      if (e < kGT * qs) {
        sx1[q * kGT + cov_slot(r)] = a[u];
        sx2[q * kGT + cov_slot(r)] = b[u];
      }
    }
  }
};

// Lower 64-tiles of the padded [np, np] covariance, f32 out, + noise on the diagonal, identity on
// the padding rows / cols (keeps log|K| and the leading block of K^-1).  Grid (G, L): workgroup g
// of dim l fills the tiles t = g, g + G, ... (t -> (I, J), I >= J), prefetching the next tile's
// covariates under the current tile's arithmetic.  HBM-write-bound: 4 B per element.
// CT: the covariates' type in LDS; both instantiations are launched and the one that does not match the
// factor's covariate flag (cov_int_check_kernel: float for integer covariates) exits at once.
template <int MC, int MF, typename CT>
__global__ __launch_bounds__(256) void gram_sq_fill_kernel(DevSpec s, const double* __restrict__ x, int ldx,
                                                           int n, int np_, int qs,
                                                           const double* __restrict__ params,
                                                           const double* __restrict__ noise,
                                                           float* __restrict__ K, int ntiles,
                                                           const int* __restrict__ covflag) {
  if (*covflag != (sizeof(CT) == 4 ? 1 : 0)) return;  // (uniform, before any barrier)
  __shared__ CT sx1[kGT * kMaxQB];
  __shared__ CT sx2[kGT * kMaxQB];
  __shared__ float sp[64];
  const int G = gridDim.x, l = blockIdx.y, tid = threadIdx.x, tr = tid >> 4, tc = tid & 15;
  if (tid < s.n_params) sp[tid] = float(params[(int64_t)l * s.n_params + tid]);
  const float nz = float(noise[l]);
  float* o = K + (int64_t)l * np_ * np_;
  int t = blockIdx.x, I, J;
  if (t >= ntiles) return;
  tri_index(t, I, J);
  CovPrefetch pf;
  pf.load(x, ldx, n, qs, I * kGT, J * kGT);
  pf.store(qs, sx1, sx2);
  __syncthreads();
  for (; t < ntiles; t += G) {
    const int i0 = I * kGT, j0 = J * kGT;
    int In = 0, Jn = 0;
    const bool more = t + G < ntiles;
    if (more) {
      tri_index(t + G, In, Jn);
      pf.load(x, ldx, n, qs, In * kGT, Jn * kGT);
    }
    float out[4][4] = {};
#pragma unroll 1
    for (int r = 0; r < s.n_comp; ++r) {  // (rolled: the spec is uniform; keeps the live set small)
      float v[4][4];
      const float sc = sp[s.scale_idx[r]];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c) v[a][c] = sc;
      if (!apply_factors_gated(s, r, sp, sx1, sx2, tr, tc, v)) continue;
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c) out[a][c] += v[a][c];
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int i = i0 + 4 * tr + a;
      g_f32x4 w;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int j = j0 + 4 * tc + c;
        float e = out[a][c];
        if (i == j) e += nz;
        if (i >= n || j >= n) e = (i == j) ? 1.0f : 0.0f;
        w[c] = e;
      }
      *reinterpret_cast<g_f32x4*>(o + (int64_t)i * np_ + j0 + 4 * tc) = w;
    }
    if (more) {
      __syncthreads();  // every reader of this tile's covariates is done
      pf.store(qs, sx1, sx2);
      __syncthreads();
      I = In, J = Jn;
    }
  }
}

// Fused adjoint for the exact KL: G = 1/2 (Kinv - S - a a^T) formed on the fly from the symmetric
// K^-1 (f32), S = K^-1 V K^-1 (f32, lower tiles) and a = K^-1 mu (f64), contracted with dK/dtheta.
// Grid (G, L): workgroup g of dim l loops over the lower 64-tiles t = g, g + G, ...; every thread
// keeps fp32 sums per PARAMETER (one slot per parameter -- each has exactly one -- plus the noise
// slot kNoiseSlot) in its private LDS column over 4 tiles (64 elements), then folds the wave sums
// into fp64 LDS accumulators; one partial per (dim, slot, workgroup) -> part[l][slot][g].  Raw sums
// (kl_gram_bwd_reduce applies the per-parameter constants):
//   scale s_r           sum w g prod_r                              (d k / d s_r = prod_r)
//   RBF lengthscale     sum w g k_r d^2                              x 1 / l^3
//   PER l / period      sum w g k_r sin^2 u,  sum w g k_r |d| sin 2u  x 4 / l^3,  2 pi / (l^2 p^2)
//   noise               sum_i G_ii
// with k_r = s_r prod_r and w = 2 strictly below the diagonal, 1 on it.
constexpr int kNoiseSlot = 64;
constexpr int kBwdSlots = 65;

template <int MC, int MF, typename CT>
__global__ __launch_bounds__(256) void kl_gram_bwd_tiles(DevSpec s, const double* __restrict__ x, int ldx, int n,
                                                         int np_, int qs, const double* __restrict__ params,
                                                         const float* __restrict__ Kinv,
                                                         const float* __restrict__ S,
                                                         const float* __restrict__ Sx, int nsplit,
                                                         const double* __restrict__ alpha,
                                                         double* __restrict__ part, int ntiles,
                                                         const int* __restrict__ covflag) {
  if (*covflag != (sizeof(CT) == 4 ? 1 : 0)) return;  // (uniform, before any barrier)
  __shared__ CT sx1[kGT * kMaxQB];
  __shared__ CT sx2[kGT * kMaxQB];
  __shared__ float sp[64];
  __shared__ float sa1[kGT], sa2[kGT];
  __shared__ double wred[4][kBwdSlots];
  // per-thread fp32 sums (thread-private columns: no races): slots 0..n_params-1, then the noise
  // at row n_params (dynamic LDS: (n_params + 1) x 256 floats)
  extern __shared__ float tacc_dyn[];
  const int G = gridDim.x, g0 = blockIdx.x, l = blockIdx.y, tid = threadIdx.x, tr = tid >> 4, tc = tid & 15;
  const int lane = tid & 63, wv = tid >> 6, np_s = s.n_params;
  auto tacc = [&](int q) -> float& { return tacc_dyn[(q == kNoiseSlot ? np_s : q) * 256 + tid]; };
  if (tid < np_s) sp[tid] = float(params[(int64_t)l * np_s + tid]);
  for (int e = tid; e < 4 * kBwdSlots; e += 256) (&wred[0][0])[e] = 0.0;
  for (int q = 0; q < np_s; ++q) tacc(q) = 0.f;
  tacc(kNoiseSlot) = 0.f;
  const float* ki = Kinv + (int64_t)l * np_ * np_;
  const float* si = S + (int64_t)l * np_ * np_;
  float dd = 0.f;
  int since_flush = 0;
  for (int t = g0; t < ntiles; t += G) {
    int I, J;
    tri_index(t, I, J);
    const int i0 = I * kGT, j0 = J * kGT;
    // this tile's K^-1 / S rows first: their latency overlaps the covariate staging and barriers
    g_f32x4 kv4[4], sv4[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int64_t o = (int64_t)(i0 + 4 * tr + a) * np_ + j0 + 4 * tc;
      kv4[a] = __builtin_nontemporal_load(reinterpret_cast<const g_f32x4*>(ki + o));
      sv4[a] = __builtin_nontemporal_load(reinterpret_cast<const g_f32x4*>(si + o));
    }
    for (int q = 1; q < nsplit; ++q) {  // K-split partials of S (syrk_x3_splits)
      const float* sq = Sx + (int64_t)(q - 1) * gridDim.y * np_ * np_ + (int64_t)l * np_ * np_;
#pragma unroll
      for (int a = 0; a < 4; ++a)
        sv4[a] += __builtin_nontemporal_load(
            reinterpret_cast<const g_f32x4*>(sq + (int64_t)(i0 + 4 * tr + a) * np_ + j0 + 4 * tc));
    }
    __syncthreads();  // previous tile's LDS readers done
    stage_cov(x, ldx, n, qs, i0, j0, sx1, sx2);
    if (tid < kGT) sa1[tid] = float(alpha[(int64_t)l * np_ + i0 + tid]);
    else if (tid < 2 * kGT) sa2[tid - kGT] = float(alpha[(int64_t)l * np_ + j0 + tid - kGT]);
    __syncthreads();
    float g[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int i = i0 + 4 * tr + a;
      const g_f32x4 kv = kv4[a], sv = sv4[a];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int j = j0 + 4 * tc + c;
        const float gv = 0.5f * (kv[c] - sv[c] - sa1[4 * tr + a] * sa2[4 * tc + c]);
        const bool in = i < n && j < n && j <= i;
        if (in && i == j) dd += gv;
        g[a][c] = in ? ((i == j) ? gv : 2.f * gv) : 0.f;
      }
    }
#pragma unroll 1
    for (int r = 0; r < s.n_comp; ++r) {
      float v[4][4];
      const float sc = sp[s.scale_idx[r]];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c) v[a][c] = g[a][c];
      if (!apply_factors_gated(s, r, sp, sx1, sx2, tr, tc, v)) continue;  // (every sum below is 0)
      // v = g prod_r: the scale's slot; g k_r = sc v for the parametrised factors
      float ssum = 0.f;
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c) ssum += v[a][c];
      tacc(s.scale_idx[r]) += ssum;
#pragma unroll 1
      for (int f = 0; f < s.n_fac[r]; ++f) {
        const int kind = s.kind[r][f];
        if (kind == LVAE_RBF || kind == LVAE_PER) {
          const int pi = s.param_idx[r][f];
          float u0, u1;
          factor_sums(kind, s.dim[r][f], sp + pi, sx1, sx2, tr, tc, v, u0, u1);
          tacc(pi) += sc * u0;
          if (kind == LVAE_PER) tacc(pi + 1) += sc * u1;
        }
      }
    }
    if (++since_flush == 4 || t + G >= ntiles) {  // fold the fp32 sums into the fp64 wave slots
      since_flush = 0;
      tacc(kNoiseSlot) += dd;
      dd = 0.f;
      for (int q = 0; q < kBwdSlots; ++q) {
        if (q >= np_s && q != kNoiseSlot) continue;  // (uniform)
        const float w = wave_sum(tacc(q));
        if (lane == 0) wred[wv][q] += (double)w;
        tacc(q) = 0.f;
      }
    }
  }
  __syncthreads();
  for (int sl = tid; sl < kBwdSlots; sl += 256)
    part[((int64_t)l * kBwdSlots + sl) * G + g0] = wred[0][sl] + wred[1][sl] + wred[2][sl] + wred[3][sl];
}

// ------------------------------------------------------------------------------------------
// Table path of the Regime B Gram fill and adjoint (covariate flag 2: integer-coded covariates whose
// continuous dims each span < kTabD values).  Every component is gates (Cat / Bin tests) times at most
// one RBF / periodic factor of |x_i[d] - x_j[d]|, so with B distinct gates and the components grouped by
// the dim of their continuous factor, an element of K is
//   K_ij = sum_g T_g[bits_ij][|x_i[d_g] - x_j[d_g]|],   T_g[b][m] = sum_{r in g, gates_r in b} s_r phi_r(m)
// (bits_ij: which of the B gates pass; components with no continuous factor join group 0 as
// d-independent terms), and each raw adjoint sum is  sum_ij w g_ij D_p[bits_ij][|d_ij|]  with D_p the
// same derivative factors as kl_gram_bwd_tiles'.  The tables (fp32, from the same fp32 formulas as the
// direct path) are built per workgroup into LDS; per element the work drops to the B gate tests, one
// difference + table read per group and, in the adjoint, one FMA per parameter.
// ------------------------------------------------------------------------------------------
#ifndef LVAE_TAB_WPE
#define LVAE_TAB_WPE 3  // the table adjoint's waves per SIMD (register cap)
#endif
// the micro-tile's gate bits as table row offsets: bits[a][c] = (sum_b pass_b << b) * kTabR
__device__ inline void tab_bits(const GramTab& t, const float* __restrict__ sx1, const float* __restrict__ sx2,
                                int tr, int tc, int (&bits)[4][4]) {
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) bits[a][c] = 0;
#pragma unroll 1
  for (int b = 0; b < t.nbits; ++b) {
    const int d = t.bdim[b], bit = kTabR << b;
    float xr[4], xc[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) xr[a] = sx1[d * kGT + a * 16 + tr];
#pragma unroll
    for (int c = 0; c < 4; ++c) xc[c] = sx2[d * kGT + c * 16 + tc];
    if (t.bkind[b] == LVAE_CAT) {
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c) bits[a][c] += (xr[a] == xc[c]) ? bit : 0;
    } else {
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c) bits[a][c] += (xr[a] + xc[c] == 2.f) ? bit : 0;
    }
  }
}

// group g's table index per element: bits + |x_i[d_g] - x_j[d_g]| (< kTabD by the covariate flag)
__device__ inline void tab_index(const GramTab& t, int g, const float* __restrict__ sx1,
                                 const float* __restrict__ sx2, int tr, int tc, const int (&bits)[4][4],
                                 int (&idx)[4][4]) {
  const int d = t.gdim[g];
  if (d < 0) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) idx[a][c] = bits[a][c];
    return;
  }
  float xr[4], xc[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) xr[a] = sx1[d * kGT + a * 16 + tr];
#pragma unroll
  for (int c = 0; c < 4; ++c) xc[c] = sx2[d * kGT + c * 16 + tc];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) idx[a][c] = bits[a][c] + (int)fabsf(xr[a] - xc[c]);
}

// gram_sq_fill_kernel's table twin (flag 2)
__global__ __launch_bounds__(256) void gram_sq_fill_tab_kernel(GramTab tb, const double* __restrict__ x, int ldx,
                                                               int n, int np_, int qs,
                                                               const double* __restrict__ params,
                                                               const double* __restrict__ noise,
                                                               float* __restrict__ K, int ntiles,
                                                               const int* __restrict__ covflag) {
  if (*covflag != 2) return;  // (uniform, before any barrier)
  __shared__ float sx1[kGT * kMaxQB];
  __shared__ float sx2[kGT * kMaxQB];
  __shared__ float sp[64];
  extern __shared__ float tab[];  // ng 2^B kTabR floats
  const int G = gridDim.x, l = blockIdx.y, tid = threadIdx.x, tr = tid >> 4, tc = tid & 15;
  if (tid < tb.n_params) sp[tid] = float(params[(int64_t)l * tb.n_params + tid]);
  const float nz = float(noise[l]);
  float* o = K + (int64_t)l * np_ * np_;
  int t = blockIdx.x, I, J;
  if (t >= ntiles) return;
  tri_index(t, I, J);
  CovPrefetchF pf;
  pf.load(x, ldx, n, qs, I * kGT, J * kGT);
  pf.store(qs, sx1, sx2);
  __syncthreads();
  tab_build_fill(tb, sp, tab);
  __syncthreads();
  const int tstride = (1 << tb.nbits) * kTabR;
  for (; t < ntiles; t += G) {
    const int i0 = I * kGT, j0 = J * kGT;
    int In = 0, Jn = 0;
    const bool more = t + G < ntiles;
    if (more) {
      tri_index(t + G, In, Jn);
      pf.load(x, ldx, n, qs, In * kGT, Jn * kGT);
    }
    int bits[4][4];
    tab_bits(tb, sx1, sx2, tr, tc, bits);
    float out[4][4] = {};
#pragma unroll 1
    for (int g = 0; g < tb.ng; ++g) {
      int idx[4][4];
      tab_index(tb, g, sx1, sx2, tr, tc, bits, idx);
      const float* tg = tab + g * tstride;
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c) out[a][c] += tg[idx[a][c]];
    }
    if (I != J && i0 + kGT <= n) {  // (uniform) an interior tile below the diagonal: no noise, no padding
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const g_f32x4 w = {out[a][0], out[a][1], out[a][2], out[a][3]};
        *reinterpret_cast<g_f32x4*>(o + (int64_t)(i0 + 4 * tr + a) * np_ + j0 + 4 * tc) = w;
      }
    } else {
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const int i = i0 + 4 * tr + a;
        g_f32x4 w;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int j = j0 + 4 * tc + c;
          float e = out[a][c];
          if (i == j) e += nz;
          if (i >= n || j >= n) e = (i == j) ? 1.0f : 0.0f;
          w[c] = e;
        }
        *reinterpret_cast<g_f32x4*>(o + (int64_t)i * np_ + j0 + 4 * tc) = w;
      }
    }
    if (more) {
      __syncthreads();  // every reader of this tile's covariates is done
      pf.store(qs, sx1, sx2);
      __syncthreads();
      I = In, J = Jn;
    }
  }
}

// kl_gram_bwd_tiles' table twin (flag 2): the same G, weights, slots and partials
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LVAE_TAB_WPE))) void kl_gram_bwd_tab_kernel(GramTab tb, const double* __restrict__ x, int ldx,
                                                              int n, int np_, int qs,
                                                              const double* __restrict__ params,
                                                              const float* __restrict__ Kinv,
                                                              const float* __restrict__ S,
                                                              const float* __restrict__ Sx, int nsplit,
                                                              const double* __restrict__ alpha,
                                                              double* __restrict__ part, int ntiles,
                                                              const int* __restrict__ covflag,
                                                              const int* __restrict__ hbon) {
  if (*covflag != 2 || (hbon && *hbon)) return;  // (uniform, before any barrier; hbon: kl_hyper.hip's path)
  __shared__ float sx1[2][kGT * kMaxQB];  // (two buffers: this tile's and the next one's)
  __shared__ float sx2[2][kGT * kMaxQB];
  __shared__ float sp[64];
  __shared__ float sa1[2][kGT], sa2[2][kGT];
  __shared__ double wred[4][kBwdSlots];
  extern __shared__ float tdyn[];  // [(n_params + 1) x 256] per-thread sums, then the tables
  const int G = gridDim.x, g0 = blockIdx.x, l = blockIdx.y, tid = threadIdx.x, tr = tid >> 4, tc = tid & 15;
  const int lane = tid & 63, wv = tid >> 6, np_s = tb.n_params;
  float* tab = tdyn + (np_s + 1) * 256;
  auto tacc = [&](int q) -> float& { return tdyn[(q == kNoiseSlot ? np_s : q) * 256 + tid]; };
  if (tid < np_s) sp[tid] = float(params[(int64_t)l * np_s + tid]);
  for (int e = tid; e < 4 * kBwdSlots; e += 256) (&wred[0][0])[e] = 0.0;
  for (int q = 0; q < np_s; ++q) tacc(q) = 0.f;
  tacc(kNoiseSlot) = 0.f;
  __syncthreads();
  tab_build_bwd(tb, sp, tab);
  const int tstride = (1 << tb.nbits) * kTabR;
  const float* ki = Kinv + (int64_t)l * np_ * np_;
  const float* si = S + (int64_t)l * np_ * np_;
  const double* al = alpha + (int64_t)l * np_;
  auto load_ks = [&](int i0, int j0, g_f32x4 (&kv4)[4], g_f32x4 (&sv4)[4]) {
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int64_t o = (int64_t)(i0 + 4 * tr + a) * np_ + j0 + 4 * tc;
      kv4[a] = __builtin_nontemporal_load(reinterpret_cast<const g_f32x4*>(ki + o));
      sv4[a] = __builtin_nontemporal_load(reinterpret_cast<const g_f32x4*>(si + o));
    }
    for (int q = 1; q < nsplit; ++q) {  // K-split partials of S (syrk_x3_splits)
      const float* sq = Sx + (int64_t)(q - 1) * gridDim.y * np_ * np_ + (int64_t)l * np_ * np_;
#pragma unroll
      for (int a = 0; a < 4; ++a)
        sv4[a] += __builtin_nontemporal_load(
            reinterpret_cast<const g_f32x4*>(sq + (int64_t)(i0 + 4 * tr + a) * np_ + j0 + 4 * tc));
    }
  };
  float dd = 0.f;
  int since_flush = 0;
  int t = g0, I = 0, J = 0, In = 0, Jn = 0;
  g_f32x4 kv4[4], sv4[4];
  CovPrefetchF pf;
  double an = 0.0;
  // software pipeline: tile t's K^-1 / S rows are loaded into registers during tile t - G and its
  // covariates / alpha entries during tile t - 2G (stored to the other LDS buffer at the end of tile
  // t - G), so that no tile waits for a global round trip and one barrier per tile suffices
  if (t < ntiles) {
    tri_index(t, I, J);
    load_ks(I * kGT, J * kGT, kv4, sv4);
    pf.load(x, ldx, n, qs, I * kGT, J * kGT);
    if (tid < 2 * kGT) an = al[(tid < kGT ? I : J) * kGT + (tid & (kGT - 1))];
    pf.store(qs, sx1[0], sx2[0]);
    if (tid < kGT) sa1[0][tid] = float(an);
    else if (tid < 2 * kGT) sa2[0][tid - kGT] = float(an);
    if (t + G < ntiles) {
      tri_index(t + G, In, Jn);
      pf.load(x, ldx, n, qs, In * kGT, Jn * kGT);
      if (tid < 2 * kGT) an = al[(tid < kGT ? In : Jn) * kGT + (tid & (kGT - 1))];
    }
  }
  __syncthreads();  // the tables and the first tile's LDS
  for (int b = 0; t < ntiles; t += G, b ^= 1) {
    const int i0 = I * kGT, j0 = J * kGT;
    const bool more = t + G < ntiles;
    const float* __restrict__ cx1 = sx1[b];
    const float* __restrict__ cx2 = sx2[b];
    float g[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int i = i0 + 4 * tr + a;
      const g_f32x4 kv = kv4[a], sv = sv4[a];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int j = j0 + 4 * tc + c;
        const float gv = 0.5f * (kv[c] - sv[c] - sa1[b][4 * tr + a] * sa2[b][4 * tc + c]);
        const bool in = i < n && j < n && j <= i;
        if (in && i == j) dd += gv;
        g[a][c] = in ? ((i == j) ? gv : 2.f * gv) : 0.f;
      }
    }
    if (more) load_ks(In * kGT, Jn * kGT, kv4, sv4);  // (in flight under this tile's tables)
#pragma unroll 1
    for (int gi = 0; gi < tb.ng; ++gi) {
      int idx[4][4];  // (the gate bits recomputed per group: fewer live registers)
      tab_bits(tb, cx1, cx2, tr, tc, idx);
      tab_index(tb, gi, cx1, cx2, tr, tc, idx, idx);
#pragma unroll 1
      for (int k = tb.pbeg[gi]; k < tb.pbeg[gi + 1]; ++k) {
        const float* tk = tab + k * tstride;
        float acc = 0.f;
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int c = 0; c < 4; ++c) acc += g[a][c] * tk[idx[a][c]];
        tacc(tb.porder[k]) += acc;
      }
    }
    if (++since_flush == 4 || t + G >= ntiles) {  // fold the fp32 sums into the fp64 wave slots
      since_flush = 0;
      tacc(kNoiseSlot) += dd;
      dd = 0.f;
      for (int q = 0; q < kBwdSlots; ++q) {
        if (q >= np_s && q != kNoiseSlot) continue;  // (uniform)
        const float w = wave_sum(tacc(q));
        if (lane == 0) wred[wv][q] += (double)w;
        tacc(q) = 0.f;
      }
    }
    if (more) {
      // tile t + G's covariates (loaded during the previous tile) to the other buffer, whose last
      // readers finished before the previous barrier; then tile t + 2G's go in flight
      pf.store(qs, sx1[b ^ 1], sx2[b ^ 1]);
      if (tid < kGT) sa1[b ^ 1][tid] = float(an);
      else if (tid < 2 * kGT) sa2[b ^ 1][tid - kGT] = float(an);
      int I2 = 0, J2 = 0;
      if (t + 2 * G < ntiles) {
        tri_index(t + 2 * G, I2, J2);
        pf.load(x, ldx, n, qs, I2 * kGT, J2 * kGT);
        if (tid < 2 * kGT) an = al[(tid < kGT ? I2 : J2) * kGT + (tid & (kGT - 1))];
      }
      __syncthreads();  // buffer b ^ 1 written; every reader of buffer b done
      I = In, J = Jn, In = I2, Jn = J2;
    }
  }
  __syncthreads();
  for (int sl = tid; sl < kBwdSlots; sl += 256)
    part[((int64_t)l * kBwdSlots + sl) * G + g0] = wred[0][sl] + wred[1][sl] + wred[2][sl] + wred[3][sl];
}

// ------------------------------------------------------------------------------------------
// The table path's adjoint as a HISTOGRAM (r5): every raw adjoint sum is  sum_ij g_ij D_p[bits_ij][d_ij,g]
// with D_p a function of (the pair's gate bits, its distance in the dim of p's group) only, so
//     raw_p = sum_{b, d} H_g[b][d] D_p[b][d],      H_g[b][d] = sum of g_ij over the pairs in bin (b, d) of group g
// -- per element ONE histogram add per group instead of one table read + FMA per parameter.  The bins are
// int64 fixed point (LDS atomics, ds_add_u64): g_ij is converted to q = round(g 2^(SHIFT - E)) straight from
// its float bits, with E a per-dim bound on |g| (2^E > 2 (max diag K^-1 + max v max diag K^-1 tr K^-1 +
// max alpha^2): |K^-1_ij|, |S_ij| <= their diagonals' max, S_ii <= max v (K^-2)_ii <= max v tr K^-1 (K^-1)_ii)
// and SHIFT = 62 - the bits a bin's count can take over the workgroup's tiles: integer adds are exact and
// associative, so the sums are DETERMINISTIC (no order dependence) and every element keeps 2^-SHIFT of the
// bound (~2^-44).  After the tiles: raw_p = 2^(E - SHIFT) sum_bins (double) H D_p in a fixed order, into the
// same per-workgroup slots kl_gram_bwd_reduce reads.  The diagonal's sum (d/d noise) stays an fp32 / fp64 sum.
// Measured (r5, scripts/gpu_r5b.sh, the exact-KL fwd + bwd alone at the headline, rocprofv3, same box): 813-845 us
// against the table kernel's 519-524 us -- bit-reproducible and within 4e-6 of it, but the 64-bit LDS atomics
// serialise on the bins the lanes of one instruction share (~16-30 distinct (bits, d) per 64 elements of a tile
// row band), which costs more than the per-parameter table reads they replace.  Opt-in: LVAE_GRAM_HIST=1.
// ------------------------------------------------------------------------------------------
__device__ inline long long fx_q(float g, int sbias) {
  const unsigned u = __float_as_uint(g);
  const int e = (int)((u >> 23) & 0xffu);
  const long long m = (long long)((u & 0x7fffffu) | 0x800000u);
  const int sh = e + sbias;
  long long q;
  if (sh >= 0) {
    q = m << (sh < 39 ? sh : 39);  // (sh <= SHIFT - 24 <= 38 when |g| < 2^E: the clamp never binds)
  } else {
    const int r = -sh;
    q = r < 25 ? ((m + (1ll << (r - 1))) >> r) : 0ll;  // round to nearest (ties up); below 2^-25 of the grid: 0
  }
  q = e == 0 ? 0ll : q;  // zero / subnormal (|g| < 2^-126: below any grid)
  return (u >> 31) ? -q : q;
}

#ifndef LVAE_HIST_WPE
#define LVAE_HIST_WPE 2  // the histogram adjoint's waves per SIMD (register cap)
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LVAE_HIST_WPE))) void kl_gram_bwd_hist_kernel(
    GramTab tb, const double* __restrict__ x, int ldx, int n, int np_, int qs, const double* __restrict__ params,
    const float* __restrict__ Kinv, const float* __restrict__ S, const float* __restrict__ Sx, int nsplit,
    const double* __restrict__ alpha, const double* __restrict__ kdiag, const float* __restrict__ vv, int shift,
    double* __restrict__ part, int ntiles, const int* __restrict__ covflag, const int* __restrict__ hbon) {
  if (*covflag != 2 || (hbon && *hbon)) return;  // (uniform, before any barrier)
  __shared__ float sx1[2][kGT * kMaxQB];  // (two buffers: this tile's and the next one's)
  __shared__ float sx2[2][kGT * kMaxQB];
  __shared__ float sp[64];
  __shared__ float sa1[2][kGT], sa2[2][kGT];
  __shared__ double wred[4][kBwdSlots];
  __shared__ double bred[4][4];
  extern __shared__ double hdyn[];  // [ng 2^B kTabR] int64 bins, then the fp32 derivative tables
  const int G = gridDim.x, g0 = blockIdx.x, l = blockIdx.y, tid = threadIdx.x, tr = tid >> 4, tc = tid & 15;
  const int lane = tid & 63, wv = tid >> 6, np_s = tb.n_params;
  const int tstride = (1 << tb.nbits) * kTabR, nbins = tb.ng * tstride;
  unsigned long long* H = reinterpret_cast<unsigned long long*>(hdyn);
  float* tab = reinterpret_cast<float*>(hdyn + nbins);
  if (tid < np_s) sp[tid] = float(params[(int64_t)l * np_s + tid]);
  for (int e = tid; e < 4 * kBwdSlots; e += 256) (&wred[0][0])[e] = 0.0;
  for (int e = tid; e < nbins; e += 256) H[e] = 0ull;
  // the bound on |g| of this dim (every workgroup of the dim computes the same value: no extra launch)
  int sbias;
  {
    const double* kd = kdiag + (int64_t)l * np_;
    const float* vl = vv + (int64_t)l * np_;
    const double* al = alpha + (int64_t)l * np_;
    double kmx = 0.0, ksum = 0.0, vmx = 0.0, amx = 0.0;
    for (int i = tid; i < n; i += 256) {
      const double k = kd[i], a = al[i];
      kmx = fmax(kmx, fabs(k));
      ksum += fabs(k);
      vmx = fmax(vmx, (double)vl[i]);
      amx = fmax(amx, a * a);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      kmx = fmax(kmx, __shfl_xor(kmx, o, 64));
      ksum += __shfl_xor(ksum, o, 64);
      vmx = fmax(vmx, __shfl_xor(vmx, o, 64));
      amx = fmax(amx, __shfl_xor(amx, o, 64));
    }
    if (lane == 0) {
      bred[wv][0] = kmx;
      bred[wv][1] = ksum;
      bred[wv][2] = vmx;
      bred[wv][3] = amx;
    }
    __syncthreads();
    kmx = fmax(fmax(bred[0][0], bred[1][0]), fmax(bred[2][0], bred[3][0]));
    ksum = (bred[0][1] + bred[1][1]) + (bred[2][1] + bred[3][1]);
    vmx = fmax(fmax(bred[0][2], bred[1][2]), fmax(bred[2][2], bred[3][2]));
    amx = fmax(fmax(bred[0][3], bred[1][3]), fmax(bred[2][3], bred[3][3]));
    const double gb = 2.0 * (kmx + vmx * kmx * ksum + amx);
    int E = 0;
    if (gb > 0.0 && gb < 1e300) (void)frexp(gb, &E);  // gb < 2^E
    sbias = shift - E - 150;
  }
  tab_build_bwd(tb, sp, tab);
  const float* ki = Kinv + (int64_t)l * np_ * np_;
  const float* si = S + (int64_t)l * np_ * np_;
  const double* al = alpha + (int64_t)l * np_;
  auto load_ks = [&](int i0, int j0, g_f32x4 (&kv4)[4], g_f32x4 (&sv4)[4]) {
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int64_t o = (int64_t)(i0 + 4 * tr + a) * np_ + j0 + 4 * tc;
      kv4[a] = __builtin_nontemporal_load(reinterpret_cast<const g_f32x4*>(ki + o));
      sv4[a] = __builtin_nontemporal_load(reinterpret_cast<const g_f32x4*>(si + o));
    }
    for (int q = 1; q < nsplit; ++q) {  // K-split partials of S (syrk_x3_splits)
      const float* sq = Sx + (int64_t)(q - 1) * gridDim.y * np_ * np_ + (int64_t)l * np_ * np_;
#pragma unroll
      for (int a = 0; a < 4; ++a)
        sv4[a] += __builtin_nontemporal_load(
            reinterpret_cast<const g_f32x4*>(sq + (int64_t)(i0 + 4 * tr + a) * np_ + j0 + 4 * tc));
    }
  };
  float dd = 0.f;
  double dsum = 0.0;
  int since_flush = 0;
  int t = g0, I = 0, J = 0, In = 0, Jn = 0;
  g_f32x4 kv4[4], sv4[4];
  CovPrefetchF pf;
  double an = 0.0;
  // software pipeline as kl_gram_bwd_tab_kernel: K^-1 / S one tile ahead in registers, the covariates and
  // alpha entries two tiles ahead (the other LDS buffer), one barrier per tile
  if (t < ntiles) {
    tri_index(t, I, J);
    load_ks(I * kGT, J * kGT, kv4, sv4);
    pf.load(x, ldx, n, qs, I * kGT, J * kGT);
    if (tid < 2 * kGT) an = al[(tid < kGT ? I : J) * kGT + (tid & (kGT - 1))];
    pf.store(qs, sx1[0], sx2[0]);
    if (tid < kGT) sa1[0][tid] = float(an);
    else if (tid < 2 * kGT) sa2[0][tid - kGT] = float(an);
    if (t + G < ntiles) {
      tri_index(t + G, In, Jn);
      pf.load(x, ldx, n, qs, In * kGT, Jn * kGT);
      if (tid < 2 * kGT) an = al[(tid < kGT ? In : Jn) * kGT + (tid & (kGT - 1))];
    }
  }
  __syncthreads();  // the bins, the tables and the first tile's LDS
  for (int b = 0; t < ntiles; t += G, b ^= 1) {
    const int i0 = I * kGT, j0 = J * kGT;
    const bool more = t + G < ntiles;
    const float* __restrict__ cx1 = sx1[b];
    const float* __restrict__ cx2 = sx2[b];
    long long q[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int i = i0 + 4 * tr + a;
      const g_f32x4 kv = kv4[a], sv = sv4[a];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int j = j0 + 4 * tc + c;
        const float gv = 0.5f * (kv[c] - sv[c] - sa1[b][4 * tr + a] * sa2[b][4 * tc + c]);
        const bool in = i < n && j < n && j <= i;
        if (in && i == j) dd += gv;
        q[a][c] = fx_q(in ? ((i == j) ? gv : 2.f * gv) : 0.f, sbias);
      }
    }
    if (more) load_ks(In * kGT, Jn * kGT, kv4, sv4);  // (in flight under this tile's bins)
    int bits[4][4];
    tab_bits(tb, cx1, cx2, tr, tc, bits);
#pragma unroll 1
    for (int gi = 0; gi < tb.ng; ++gi) {
      int idx[4][4];
      tab_index(tb, gi, cx1, cx2, tr, tc, bits, idx);
      unsigned long long* hg = H + gi * tstride;
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (q[a][c] != 0) atomicAdd(hg + idx[a][c], (unsigned long long)q[a][c]);
    }
    if (++since_flush == 8 || t + G >= ntiles) {  // the diagonal's fp32 sums into fp64
      since_flush = 0;
      dsum += (double)dd;
      dd = 0.f;
    }
    if (more) {
      pf.store(qs, sx1[b ^ 1], sx2[b ^ 1]);
      if (tid < kGT) sa1[b ^ 1][tid] = float(an);
      else if (tid < 2 * kGT) sa2[b ^ 1][tid - kGT] = float(an);
      int I2 = 0, J2 = 0;
      if (t + 2 * G < ntiles) {
        tri_index(t + 2 * G, I2, J2);
        pf.load(x, ldx, n, qs, I2 * kGT, J2 * kGT);
        if (tid < 2 * kGT) an = al[(tid < kGT ? I2 : J2) * kGT + (tid & (kGT - 1))];
      }
      __syncthreads();  // buffer b ^ 1 written; every reader of buffer b done
      I = In, J = Jn, In = I2, Jn = J2;
    }
  }
  __syncthreads();  // every bin add done
  // raw_p = 2^(E - SHIFT) sum_bins H D_p: thread t takes bins t, t + 256, ... of p's group, then the waves'
  // sums in a fixed order
  const double unscale = ldexp(1.0, -(sbias + 150));  // 2^(E - SHIFT)
  for (int gi = 0; gi < tb.ng; ++gi) {
    const long long* hg = reinterpret_cast<const long long*>(H + gi * tstride);
    for (int k = tb.pbeg[gi]; k < tb.pbeg[gi + 1]; ++k) {
      const float* tk = tab + k * tstride;
      double acc = 0.0;
      for (int e = tid; e < tstride; e += 256) acc += (double)hg[e] * (double)tk[e];
      acc = wave_sum(acc);
      if (lane == 0) wred[wv][tb.porder[k]] = acc * unscale;
    }
  }
  {
    const double w = wave_sum(dsum);
    if (lane == 0) wred[wv][kNoiseSlot] = w;
  }
  __syncthreads();
  for (int sl = tid; sl < kBwdSlots; sl += 256)
    part[((int64_t)l * kBwdSlots + sl) * G + g0] = ((wred[0][sl] + wred[1][sl]) + wred[2][sl]) + wred[3][sl];
}

// fp64 residual of the exact-KL solve, r = mu - K alpha0 (K = Gram + noise I, alpha0 = K^-1 mu from the
// fp32 inverse), the matrix never materialised: every lower 64-tile's kernel values are evaluated in
// fp64 (fp64 exp / sin, covariate tests and differences exact, as the reference's double arithmetic)
// and contracted with alpha0 on both sides -- the row sums K_IJ a_J of block I and, off the diagonal,
// the column sums K_IJ^T a_I of block J -- each written once to part[l][other block][row], summed in a
// fixed order by kl_resid_reduce (deterministic).  Grid (G, L) over the tiles t = g, g + G, ...;
// diagonal tiles are evaluated whole.  Components whose Cat / Bin gates are zero on a whole wave skip
// their exp / sin factors.  Refining alpha = alpha0 + K^-1 r (kl_alpha_kernel) then makes K^-1 mu
// (and mu^T K^-1 mu) fp64-accurate up to cond(K)^2 x the inverse's error (elbo_functions.py:27-30).
// exp(x) for x <= 0 to ~1e-15 relative with a 64-entry table: 2^y = 2^m 2^(i/64) 2^f, y = x log2 e,
// f in [0, 1/64) by a degree-5 polynomial (truncation (f ln 2)^6 / 720 < 3e-15) -- about half the fp64
// instructions of the library exp.  tab[i] = 2^(i/64) in LDS.
__device__ inline double exp_nonpos64(double x, const double* __restrict__ tab) {
  constexpr double kLog2e = 1.4426950408889634074;
  constexpr double kLn2 = 0.69314718055994530942;
  const double y = fmax(x * kLog2e, -1100.0);
  const double k = floor(y * 64.0);
  const double f = (y - k * (1.0 / 64.0)) * kLn2;  // in [0, ln2 / 64)
  const int ki = (int)k;
  double p = 1.0 / 120.0;
  p = fma(p, f, 1.0 / 24.0);
  p = fma(p, f, 1.0 / 6.0);
  p = fma(p, f, 0.5);
  p = fma(p, f, 1.0);
  p = fma(p, f, 1.0);
  return ldexp(tab[ki & 63] * p, ki >> 6);
}

// Covariates are often integer-coded (time points, disease times): an RBF / periodic factor of an
// integer distance |d| < kIntTab is read from a per-(component, factor) table of its fp64 values (the
// same function of the same argument), and evaluated directly otherwise.
constexpr int kIntTab = 64;
__device__ inline double factor64_at(int kind, double ad, const double* __restrict__ pf,
                                     const double* __restrict__ tab) {
  if (kind == LVAE_RBF) return exp_nonpos64(-0.5 / (pf[0] * pf[0]) * ad * ad, tab);
  const double sn = sin(ad * (M_PI / pf[1]));
  return exp_nonpos64(-2.0 / (pf[0] * pf[0]) * sn * sn, tab);
}

__device__ inline void apply_factor64(int kind, int d, const double* __restrict__ pf, const double* __restrict__ sx1,
                                      const double* __restrict__ sx2, int tr, int tc, int hf, double (&v)[2][4],
                                      const double* __restrict__ tab, const double* __restrict__ itab) {
  double xr[2], xc[4];
#pragma unroll
  for (int a = 0; a < 2; ++a) xr[a] = sx1[d * kGT + (2 * hf + a) * 16 + tr];
#pragma unroll
  for (int c = 0; c < 4; ++c) xc[c] = sx2[d * kGT + c * 16 + tc];
  if (kind == LVAE_CAT) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) v[a][c] = (xr[a] == xc[c]) ? v[a][c] : 0.0;
  } else if (kind == LVAE_BIN) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) v[a][c] = (xr[a] + xc[c] == 2.0) ? v[a][c] : 0.0;
  } else if (kind == LVAE_RBF || kind == LVAE_PER) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const double ad = fabs(xr[a] - xc[c]);
        const bool hit = ad < (double)kIntTab && ad == floor(ad);
        v[a][c] *= hit ? itab[hit ? (int)ad : 0] : factor64_at(kind, ad, pf, tab);
      }
  } else {  // LVAE_LIN
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) v[a][c] *= xr[a] * xc[c];
  }
}

template <int MC, int MF>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void kl_resid_tiles(DevSpec s, const double* __restrict__ x, int ldx, int n, int np_,
                                                      int qs, const double* __restrict__ params,
                                                      const double* __restrict__ noise,
                                                      const double* __restrict__ alpha, double* __restrict__ part,
                                                      int ntiles, const int* __restrict__ skip) {
  if (skip && *skip) return;  // the binned path (kl_resid_bins.hip) took this call
  __shared__ double sx1[kGT * kMaxQB];
  __shared__ double sx2[kGT * kMaxQB];
  __shared__ double sp[64];
  __shared__ double sa1[kGT], sa2[kGT];
  __shared__ double cred[4][kGT];
  __shared__ double tab[64];
  __shared__ double itab[MC * MF * kIntTab];  // integer-distance tables, slot r * MF + f
  const int G = gridDim.x, l = blockIdx.y, tid = threadIdx.x, tr = tid >> 4, tc = tid & 15;
  if (tid < 64) tab[tid] = exp2((double)tid / 64.0);
  const int lane = tid & 63, wv = tid >> 6, nt = np_ / kGT;
  if (tid < s.n_params) sp[tid] = params[(int64_t)l * s.n_params + tid];
  __syncthreads();
  for (int e = tid; e < MC * MF * kIntTab; e += 256) {
    const int r = e / (MF * kIntTab), f = (e / kIntTab) % MF, m = e % kIntTab;
    double val = 0.0;
    if (r < s.n_comp && f < s.n_fac[r] && (s.kind[r][f] == LVAE_RBF || s.kind[r][f] == LVAE_PER))
      val = factor64_at(s.kind[r][f], (double)m, sp + s.param_idx[r][f], tab);
    itab[e] = val;
  }
  const double nz = noise[l];
  const double* al = alpha + (int64_t)l * np_;
  for (int t = blockIdx.x; t < ntiles; t += G) {
    int I, J;
    tri_index(t, I, J);
    const int i0 = I * kGT, j0 = J * kGT;
    __syncthreads();  // the previous tile's LDS readers are done
    stage_cov(x, ldx, n, qs, i0, j0, sx1, sx2);
    if (tid < kGT) sa1[tid] = al[i0 + tid];
    else if (tid < 2 * kGT) sa2[tid - kGT] = al[j0 + tid - kGT];
    __syncthreads();
    // the 4 x 4 micro-tile in two halves of 2 rows (fewer live fp64 registers): row sums of block I
    // (this tile's share, reduced over the 16 lanes tc of each row group) and the column sums of block
    // J accumulated over both halves
    double rs[4], cs[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 1
    for (int hf = 0; hf < 2; ++hf) {
      double k[2][4] = {};
#pragma unroll 1
      for (int r = 0; r < s.n_comp; ++r) {
        double v[2][4];
        const double sc = sp[s.scale_idx[r]];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int c = 0; c < 4; ++c) v[a][c] = sc;
        // gates first (cheap, exact), then the transcendental factors unless the gates zeroed the wave
#pragma unroll 1
        for (int f = 0; f < s.n_fac[r]; ++f) {
          const int kind = s.kind[r][f];
          if (kind != LVAE_CAT && kind != LVAE_BIN) continue;
          apply_factor64(kind, s.dim[r][f], sp, sx1, sx2, tr, tc, hf, v, tab, itab);
        }
        bool any = false;
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int c = 0; c < 4; ++c) any |= v[a][c] != 0.0;
        if (!__any(any)) continue;
#pragma unroll 1
        for (int f = 0; f < s.n_fac[r]; ++f) {
          const int kind = s.kind[r][f];
          if (kind == LVAE_CAT || kind == LVAE_BIN) continue;
          const int pi = s.param_idx[r][f];
          apply_factor64(kind, s.dim[r][f], sp + (pi < 0 ? 0 : pi), sx1, sx2, tr, tc, hf, v, tab,
                         itab + (r * MF + f) * kIntTab);
        }
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int c = 0; c < 4; ++c) k[a][c] += v[a][c];
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int i = i0 + 4 * tr + 2 * hf + a, j = j0 + 4 * tc + c;
          if (i >= n || j >= n) k[a][c] = 0.0;
          else if (i == j) k[a][c] += nz;
        }
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        double v = 0.0;
#pragma unroll
        for (int c = 0; c < 4; ++c) v += k[a][c] * sa2[4 * tc + c];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
        rs[2 * hf + a] = v;
      }
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int a = 0; a < 2; ++a) cs[c] += k[a][c] * sa1[4 * tr + 2 * hf + a];
    }
    if (tc == 0) {
      double* pr = part + ((int64_t)l * nt + J) * np_ + i0 + 4 * tr;
#pragma unroll
      for (int a = 0; a < 4; ++a) pr[a] = rs[a];
    }
    if (I != J) {  // (uniform) column sums of block J: over tr (4 per wave, then the 4 waves)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        cs[c] += __shfl_xor(cs[c], 16, 64);
        cs[c] += __shfl_xor(cs[c], 32, 64);
      }
      if (lane < 16) {
#pragma unroll
        for (int c = 0; c < 4; ++c) cred[wv][4 * tc + c] = cs[c];
      }
      __syncthreads();
      if (tid < kGT) part[((int64_t)l * nt + I) * np_ + j0 + tid] = cred[0][tid] + cred[1][tid] + cred[2][tid] + cred[3][tid];
    }
  }
}

// r[l][i] = mu[l][i] - sum_s part[l][s][i] (fixed order), 0 on the padding.  Grid (np / 256, L).
__global__ __launch_bounds__(256) void kl_resid_reduce(const double* __restrict__ part, const double* __restrict__ muc,
                                                       int n, int np_, double* __restrict__ res,
                                                       const int* __restrict__ skip) {
  const int i = blockIdx.x * 256 + threadIdx.x, l = blockIdx.y, nt = np_ / kGT;
  if (i >= np_ || (skip && *skip)) return;
  double acc = 0.0;
  for (int s = 0; s < nt; ++s) acc += part[((int64_t)l * nt + s) * np_ + i];
  res[(int64_t)l * np_ + i] = i < n ? muc[(int64_t)l * np_ + i] - acc : 0.0;
}

// per-parameter derivative constants of kl_gram_bwd_tiles' raw sums (host-built from the spec):
// type 0 scale (1), 1 RBF lengthscale (1 / l^3), 2 PER lengthscale (4 / l^3), 3 PER period
// (2 pi / (l^2 p^2), l at index ell[p])
struct BwdParamInfo {
  int8_t type[64];
  int8_t ell[64];
};

// dparams[l, p] = gkl[l] c_p sum_g part[l][p][g]; dnoise[l] from kNoiseSlot.  Grid (n_params + 1, L).
__global__ __launch_bounds__(256) void kl_gram_bwd_reduce(BwdParamInfo pinfo, int n_params,
                                                          const double* __restrict__ part, int G,
                                                          const double* __restrict__ params,
                                                          const double* __restrict__ gkl,
                                                          double* __restrict__ dparams,
                                                          double* __restrict__ dnoise) {
  __shared__ double red[4];
  const int b = blockIdx.x, l = blockIdx.y, tid = threadIdx.x;
  const int slot = b == n_params ? kNoiseSlot : b;
  const double* p = part + ((int64_t)l * kBwdSlots + slot) * G;
  double v = 0.0;
  for (int t = tid; t < G; t += 256) v += p[t];
  v = block_sum<256>(v, red);
  if (tid != 0) return;
  if (slot == kNoiseSlot) {
    if (dnoise) dnoise[l] = gkl[l] * v;
    return;
  }
  const double* pl = params + (int64_t)l * n_params;
  double c = 1.0;
  const int ty = pinfo.type[b];
  if (ty == 1) c = 1.0 / (pl[b] * pl[b] * pl[b]);
  else if (ty == 2) c = 4.0 / (pl[b] * pl[b] * pl[b]);
  else if (ty == 3) {
    const double ell = pl[pinfo.ell[b]];
    c = 2.0 * M_PI / (ell * ell * pl[b] * pl[b]);
  }
  dparams[(int64_t)l * n_params + b] = gkl[l] * c * v;
}

// ------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------
// LVAE_<name>=0 in the environment switches a fast path off (A/B runs)
static bool getenv_off(const char* name) {
  const char* v = getenv(name);
  return v && atoi(v) == 0;
}

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

// host: up to kGFMaxJobs fp64 Grams (descriptors as lvae_gram_f64's arguments; spec index into specs[0..1])
int gram_multi_f64(const lvae_kernel_spec* const* specs, const GramFwdJob* jobs, int njobs, int L, hipStream_t st) {
  if (njobs < 1 || njobs > kGFMaxJobs || L < 1) return -4;
  GramFwdJobs J{};
  int bucket = 0, blocks = 0;
  for (int k = 0; k < 2; ++k) {
    if (!specs[k]) continue;
    const int bk = spec_bucket(specs[k]);
    if (!bk || spec_qs(specs[k]) > kMaxQ) return -1;
    bucket = bk > bucket ? bk : bucket;
    J.s[k] = to_dev(specs[k]);
    J.qs[k] = spec_qs(specs[k]);
  }
  J.njobs = 0;
  for (int q = 0; q < njobs; ++q) {
    GramFwdJob jb = jobs[q];
    if (jb.spec < 0 || jb.spec > 1 || !specs[jb.spec]) return -1;
    if (jb.nb < 1 || jb.n1 < 0 || jb.n2 < 0) return -4;
    if (jb.n1 == 0 || jb.n2 == 0) continue;
    jb.gx = cdiv(jb.n2, kGT), jb.gy = cdiv(jb.n1, kGT), jb.blk0 = blocks;
    blocks += jb.gx * jb.gy * jb.nb * L;
    J.j[J.njobs++] = jb;
  }
  if (J.njobs == 0) return 0;
  if (bucket == 1)
    gram_multi_kernel<8, 2><<<blocks, 256, 0, st>>>(J, L);
  else
    gram_multi_kernel<16, 4><<<blocks, 256, 0, st>>>(J, L);
  LVAE_CHECK_LAUNCH();
  return 0;
}

int kl_gram_fill(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int np_, int L,
                 const double* params, const double* noise, float* K, int* covflag, hipStream_t st) {
  const int bucket = spec_bucket(spec);
  const int qs = spec_qs(spec);
  if (!bucket || qs > kMaxQB || qs > ldx) return -1;
  const DevSpec ds = to_dev(spec);
  const int nt = np_ / kGT, ntiles = nt * (nt + 1) / 2;
  int G = (2048 + L - 1) / L;  // ~8 resident workgroups per CU, 2 rounds
  G = G < ntiles ? G : ntiles;
  dim3 grid(G, L);
  GramTab tb;
  const bool tab_ok = gram_tab_build(spec, tb) && !getenv_off("LVAE_GRAM_TAB");
  int tabmask = 0;
  for (int g = 0; g < tb.ng && tab_ok; ++g)
    if (tb.gdim[g] >= 0) tabmask |= 1 << tb.gdim[g];
  cov_int_check_kernel<<<1, 1024, 0, st>>>(x, ldx, n, qs, tab_ok, tabmask, covflag);
  if (tab_ok)
    gram_sq_fill_tab_kernel<<<grid, 256, (size_t)tb.ng * (1 << tb.nbits) * kTabR * sizeof(float), st>>>(
        tb, x, ldx, n, np_, qs, params, noise, K, ntiles, covflag);
  if (bucket == 1) {
    gram_sq_fill_kernel<8, 2, float><<<grid, 256, 0, st>>>(ds, x, ldx, n, np_, qs, params, noise, K, ntiles, covflag);
    gram_sq_fill_kernel<8, 2, double><<<grid, 256, 0, st>>>(ds, x, ldx, n, np_, qs, params, noise, K, ntiles, covflag);
  } else {
    gram_sq_fill_kernel<16, 4, float><<<grid, 256, 0, st>>>(ds, x, ldx, n, np_, qs, params, noise, K, ntiles, covflag);
    gram_sq_fill_kernel<16, 4, double><<<grid, 256, 0, st>>>(ds, x, ldx, n, np_, qs, params, noise, K, ntiles, covflag);
  }
  LVAE_CHECK_LAUNCH();
  return 0;
}

int kl_resid_bins(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int np_, int L,
                  const double* params, const double* noise, const double* alpha0, const double* muc, double* res,
                  void* wsbuf, int** okflag, hipStream_t st);

size_t kl_resid_partials_bytes(int np_, int L) { return (size_t)L * (np_ / kGT) * np_ * sizeof(double); }

int kl_gram_resid(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int np_, int L,
                  const double* params, const double* noise, const double* alpha0, const double* muc, double* part,
                  double* res, void* rbws, hipStream_t st) {
  const int bucket = spec_bucket(spec);
  const int qs = spec_qs(spec);
  if (!bucket || qs > kMaxQB || qs > ldx || spec->n_params > 64) return -1;
  const DevSpec ds = to_dev(spec);
  const int nt = np_ / kGT, ntiles = nt * (nt + 1) / 2;
  // ~8 resident workgroups per CU in 2 rounds; one round of 2 per CU behind the binned path (when it
  // runs, these launches only read the flag and exit: fewer of them)
  int G = ((rbws ? 512 : 2048) + L - 1) / L;
  G = G < ntiles ? G : ntiles;
  // rbws (the binned residual's planned workspace, kl_resid_bins_plan): integer-coded covariates take
  // the binned O(N W) residual and the tiled kernels below exit at once (checked on the device: *skip)
  int* skip = nullptr;
  if (rbws)
    LVAE_TRY(kl_resid_bins(spec, x, ldx, n, np_, L, params, noise, alpha0, muc, res, rbws, &skip, st));
  if (bucket == 1)
    kl_resid_tiles<8, 2><<<dim3(G, L), 256, 0, st>>>(ds, x, ldx, n, np_, qs, params, noise, alpha0, part, ntiles, skip);
  else
    kl_resid_tiles<16, 4><<<dim3(G, L), 256, 0, st>>>(ds, x, ldx, n, np_, qs, params, noise, alpha0, part, ntiles, skip);
  kl_resid_reduce<<<dim3(cdiv(np_, 256), L), 256, 0, st>>>(part, muc, n, np_, res, skip);
  LVAE_CHECK_LAUNCH();
  return 0;
}

// workgroups per latent dim of the adjoint: ~1536 in all, each looping over ~ntiles / G tiles
static int kl_gram_bwd_groups(int np_, int L) {
  const int nt = np_ / kGT, ntiles = nt * (nt + 1) / 2;
  int G = (1536 + L - 1) / L;  // 2 full rounds of 256 CUs x 3 resident workgroups
  G = G < 8 ? 8 : G;
  return G < ntiles ? G : ntiles;
}

size_t kl_gram_bwd_partials_bytes(int np_, int L) {
  return (size_t)L * kl_gram_bwd_groups(np_, L) * kBwdSlots * sizeof(double);
}

int kl_hyper_bwd(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int np_, int L, const double* params,
                 const float* Kinv, const float* v, const double* alpha, const double* kdiag, void* wsbase, double* part,
                 int G, hipStream_t st);

int kl_gram_bwd(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int np_, int L,
                const double* params, const float* Kinv, const float* S, const float* Sx, int nsplit,
                const double* alpha, const double* kdiag, const float* v, const double* gkl, double* part,
                double* dparams, double* dnoise, const int* covflag, void* hbws, const int* hbon, hipStream_t st) {
  const int bucket = spec_bucket(spec);
  const int qs = spec_qs(spec);
  if (!bucket || qs > kMaxQB || spec->n_params > 64) return -1;
  const DevSpec ds = to_dev(spec);
  BwdParamInfo pinfo{};
  for (int r = 0; r < spec->n_comp; ++r)
    for (int f = 0; f < spec->n_fac[r]; ++f) {
      const int pi = spec->param_idx[r][f];
      if (spec->kind[r][f] == LVAE_RBF) pinfo.type[pi] = 1;
      if (spec->kind[r][f] == LVAE_PER) {
        pinfo.type[pi] = 2;
        pinfo.type[pi + 1] = 3;
        pinfo.ell[pi + 1] = (int8_t)pi;
      }
    }
  const int nt = np_ / kGT, ntiles = nt * (nt + 1) / 2, G = kl_gram_bwd_groups(np_, L);
  const size_t dyn = (size_t)(spec->n_params + 1) * 256 * sizeof(float);
  GramTab tb;
  if (gram_tab_build(spec, tb) && !getenv_off("LVAE_GRAM_TAB")) {  // (the same decision as kl_gram_fill's)
    const size_t tabb = (size_t)tb.pbeg[tb.ng] * (1 << tb.nbits) * kTabR * sizeof(float);
    const char* hv = getenv("LVAE_GRAM_HIST");
    if (hv && atoi(hv) == 1) {  // opt-in: measured slower (r5: 813-845 vs 519-524 us alone, gpurun_out/r5b)
      // the histogram adjoint: SHIFT = 62 - (bits of a bin's largest possible count, + 1)
      const int per = (ntiles + G - 1) / G;
      int hb = 1;
      while ((1ll << hb) < (long long)per * kGT * kGT) ++hb;
      const size_t hdyn = (size_t)tb.ng * (1 << tb.nbits) * kTabR * sizeof(double) + tabb;
      kl_gram_bwd_hist_kernel<<<dim3(G, L), 256, hdyn, st>>>(tb, x, ldx, n, np_, qs, params, Kinv, S, Sx, nsplit,
                                                             alpha, kdiag, v, 62 - (hb + 1), part, ntiles, covflag, hbon);
    } else {
      kl_gram_bwd_tab_kernel<<<dim3(G, L), 256, dyn + tabb, st>>>(tb, x, ldx, n, np_, qs, params, Kinv, S, Sx,
                                                                  nsplit, alpha, part, ntiles, covflag, hbon);
    }
  }
  if (bucket == 1) {
    kl_gram_bwd_tiles<8, 2, float><<<dim3(G, L), 256, dyn, st>>>(ds, x, ldx, n, np_, qs, params, Kinv, S, Sx, nsplit,
                                                                  alpha, part, ntiles, covflag);
    kl_gram_bwd_tiles<8, 2, double><<<dim3(G, L), 256, dyn, st>>>(ds, x, ldx, n, np_, qs, params, Kinv, S, Sx, nsplit,
                                                                   alpha, part, ntiles, covflag);
  } else {
    kl_gram_bwd_tiles<16, 4, float><<<dim3(G, L), 256, dyn, st>>>(ds, x, ldx, n, np_, qs, params, Kinv, S, Sx,
                                                                   nsplit, alpha, part, ntiles, covflag);
    kl_gram_bwd_tiles<16, 4, double><<<dim3(G, L), 256, dyn, st>>>(ds, x, ldx, n, np_, qs, params, Kinv, S, Sx,
                                                                    nsplit, alpha, part, ntiles, covflag);
  }
  // the binned hyper-gradient (kl_hyper.hip; its kernels exit when the plan is off, the table kernel when it is on)
  if (hbws) LVAE_TRY(kl_hyper_bwd(spec, x, ldx, n, np_, L, params, Kinv, v, alpha, kdiag, hbws, part, G, st));
  kl_gram_bwd_reduce<<<dim3(spec->n_params + 1, L), 256, 0, st>>>(pinfo, spec->n_params, part, G, params, gkl,
                                                                  dparams, dnoise);
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
