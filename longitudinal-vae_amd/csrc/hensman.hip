// hensman.hip -- Hensman mini-batch KL upper bound of the L-VAE (elbo_functions.py:144-216), its
// analytic adjoint (what autograd computes through it), and the natural-gradient update of the
// inducing posterior (training.py:129-135).  fp64 throughout; batched over the L latent dims.
//
// Per latent dim (B = P_b T rows, subject blocks p of T rows):
//   K0xz = k0(x, z) [B,M]  K0zz = k0(z, z) + eps I  K0_p = k0(x_p, x_p)  B_p = k1(x_p, x_p) + noise I
//   iK = K0zz^-1, iB_p = B_p^-1, iH = H^-1 (+ log-dets)         spd_inv_small
//   t = iK m, r = K0xz t - mu, s = iB r, iBK = iB K0xz, Q = K0xz^T iBK, Y = iK H iK
//   A = r.s, Bt = sum diag(iB) v, C = sum log|B_p|, D = sum iB.K0 - sum Q.iK, E = sum Y.Q, F = sum logv
//   kl_u = 1/2 (sum iK.H + m.t - M + log|K0zz| - log|H|)
//   kld = sum_l [P_tot/P_b 1/2 (A+Bt+C+D+E-F) + kl_u] - L P_tot T / 2
//   natural gradient: grad_m = -iK K0xz^T iB mu + Bn m, grad_H = 1/2(-iH + Bn), Bn = iK Q iK + iK
// Adjoint (g = dL/dkld, c = g P_tot / (2 P_b), h = g / 2):
//   dmu = -2c s, dlogv = c (diag(iB) v - 1), Xq = c (Y - iK)
//   dK0xz = 2c s t^T + 2 iBK Xq
//   G_iK = c (2 (K0xz^T s) m^T - Q + Z + Z^T) + h (H + m m^T),  Z = Q iK H
//   dK0zz = -iK G_iK iK + h iK
//   dK0_p = c iB_p
//   dB_p = c (iB - s s^T - iB V iB - iB K0 iB)_p - iBK_p Xq iBK_p^T
//   (Adam path) dm = 2c iK K0xz^T s + g t,  dH = c iK Q iK + h (iK - iH)
#include "common.hpp"
#include "gram_bwd.hpp"
#include "prof.hpp"

namespace lvae {


int spd_inv_small_f64(int n, int batch, const double* A, int64_t stride, double* Ainv, int64_t stride_out,
                      double* logdet, int32_t* info, hipStream_t st);
int spd_inv_small2_f64(int n, int nb0, const double* A0, int64_t stride0, double* Ainv0, int64_t stride_out0,
                       double* logdet0, int32_t* info0, int nb1, const double* A1, int64_t stride1, double* Ainv1,
                       int64_t stride_out1, double* logdet1, int32_t* info1, hipStream_t st);
int gemm_small_f64(int ta, int tb, int m, int n, int k, double alpha, const double* A, int lda, int64_t sa1,
                   int64_t sa2, const double* B, int ldb, int64_t sb1, int64_t sb2, double beta, double* C, int ldc,
                   int64_t sc1, int64_t sc2, int nb1, int nb2, hipStream_t st);

namespace {

constexpr int kHnSlices = 8;  // workgroups per latent dim of hn_reduce_kernel

struct HWs {
  // [L,B,M]
  double *K0xz, *iBK, *dK0xz, *tBM;
  // [L,M,M]
  double *K0zz, *iK, *iH, *Q, *iKH, *Y, *Xq, *Z, *GiK, *T1, *dK0zz, *Bn, *iKQ, *tMM;
  // [L,P_b,T,T]
  double *K0st, *Bst, *iB, *VB, *iBVB, *K0iB, *iBK0iB, *QB, *GB, *GK0;
  // vectors
  double *t, *v1, *w, *a, *tM;  // [L,M]
  double *y, *r, *s, *u;        // [L,B]
  double *ldK, *ldB, *ldH, *epsv, *part, *gpart;
  int32_t* info;
  size_t bytes;
  HWs(char* base, const lvae_hensman_dims& d) {
    size_t off = 0;
    auto take = [&](size_t n) {
      double* p = base ? (double*)(base + off) : nullptr;
      off += align256(n * sizeof(double));
      return p;
    };
    const size_t L = d.L, M = d.M, B = (size_t)d.P_b * d.T, TT = (size_t)d.P_b * d.T * d.T;
    K0xz = take(L * B * M); iBK = take(L * B * M); dK0xz = take(L * B * M); tBM = take(L * B * M);
    double** mm[] = {&K0zz, &iK, &iH, &Q, &iKH, &Y, &Xq, &Z, &GiK, &T1, &dK0zz, &Bn, &iKQ, &tMM};
    for (auto p : mm) *p = take(L * M * M);
    double** tt[] = {&K0st, &Bst, &iB, &VB, &iBVB, &K0iB, &iBK0iB, &QB, &GB, &GK0};
    for (auto p : tt) *p = take(L * TT);
    double** vm[] = {&t, &v1, &w, &a, &tM};
    for (auto p : vm) *p = take(L * M);
    double** vb[] = {&y, &r, &s, &u};
    for (auto p : vb) *p = take(L * B);
    ldK = take(L);
    ldB = take(L * d.P_b);
    ldH = take(L);
    epsv = take(L);
    part = take(L * 16 * kHnSlices);
    info = (int32_t*)take(L * (2 + d.P_b));
    // Gram-adjoint partials of the four Grams (gram.hip, kGBChunk = 1024 elements per chunk, <= 145 slots)
    const size_t chunks = (B * M + 1023) / 1024 + (M * M + 1023) / 1024 + 2 * ((TT + 1023) / 1024);
    gpart = take(L * chunks * 145);
    bytes = off;
  }
};

// varying T: row q of subject p is valid iff q < seg[p] (seg == NULL: all rows)
__device__ inline bool seg_valid(const int32_t* __restrict__ seg, int p, int q) { return !seg || q < seg[p]; }

// padding rows of a varying-T batch: K0xz rows -> 0, K0_p rows/cols -> 0, B_p rows/cols -> I
__global__ void hn_seg_mask_kernel(int L, int P_b, int T, int M, const int32_t* __restrict__ seg,
                                   double* __restrict__ K0xz, double* __restrict__ K0st, double* __restrict__ Bst) {
  const int64_t B = (int64_t)P_b * T, nxz = (int64_t)L * B * M, TT = (int64_t)T * T, nst = (int64_t)L * P_b * TT;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < nxz) {
    const int64_t row = (e / M) % B;
    const int p = (int)(row / T), q = (int)(row % T);
    if (!seg_valid(seg, p, q)) K0xz[e] = 0.0;
  } else if (e < nxz + nst) {
    const int64_t f = e - nxz;
    const int p = (int)((f / TT) % P_b), i = (int)((f % TT) / T), j = (int)(f % T);
    if (!seg_valid(seg, p, i) || !seg_valid(seg, p, j)) {
      K0st[f] = 0.0;
      Bst[f] = (i == j) ? 1.0 : 0.0;
    }
  }
}

__global__ void fill_kernel(double* p, int n, double v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

// r[l][i] = y[l][i] - mu[i][l]
__global__ void resid_kernel(const double* __restrict__ y, const double* __restrict__ mu, int B, int L, int T,
                             const int32_t* __restrict__ seg, double* __restrict__ r) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * L) return;
  const int l = e / B, i = e % B;
  r[e] = seg_valid(seg, i / T, i % T) ? y[e] - mu[(int64_t)i * L + l] : 0.0;
}

// per-dim partial sums, each dim's elements split over kHnSlices workgroups (more reads in flight than one
// workgroup per dim): part[l][slice][0..] = A, Bt, C, D1, D2, E, F, tr1, qf1, ldK, ldH
__global__ __launch_bounds__(256) void hn_reduce_kernel(int M, int P_b, int T, int L, const double* __restrict__ r,
                                                        const double* __restrict__ s, const double* __restrict__ iB,
                                                        const double* __restrict__ logv,
                                                        const double* __restrict__ ldB,
                                                        const double* __restrict__ K0st,
                                                        const double* __restrict__ Q, const double* __restrict__ iK,
                                                        const double* __restrict__ Y, const double* __restrict__ H,
                                                        const double* __restrict__ m, const double* __restrict__ t,
                                                        const double* __restrict__ ldK,
                                                        const double* __restrict__ ldH,
                                                        const int32_t* __restrict__ seg, double* __restrict__ part) {
  __shared__ double red[4];
  const int l = blockIdx.x, sl = blockIdx.y, tid = threadIdx.x + 256 * sl;
  constexpr int kStep = 256 * kHnSlices;
  const int B = P_b * T;
  const int64_t MM = (int64_t)M * M, TT = (int64_t)P_b * T * T;
  double A = 0, Bt = 0, C = 0, D1 = 0, D2 = 0, E = 0, F = 0, tr1 = 0, qf1 = 0;
  for (int i = tid; i < B; i += kStep) {
    A += r[(int64_t)l * B + i] * s[(int64_t)l * B + i];
    const int p = i / T, q = i % T;
    if (!seg_valid(seg, p, q)) continue;
    const double lv = logv[(int64_t)i * L + l];
    Bt += iB[l * TT + (int64_t)p * T * T + q * T + q] * exp(lv);
    F += lv;
  }
  for (int p = tid; p < P_b; p += kStep) C += ldB[(int64_t)l * P_b + p];
  for (int64_t e = tid; e < TT; e += kStep) D1 += iB[l * TT + e] * K0st[l * TT + e];
  for (int64_t e = tid; e < MM; e += kStep) {
    const double q = Q[l * MM + e], ik = iK[l * MM + e];
    D2 += q * ik;
    // E = sum Y^T .* Q = sum Y .* Q (Y symmetric up to rounding: use the transposed element as the reference)
    const int i = (int)(e / M), j = (int)(e % M);
    E += Y[l * MM + (int64_t)j * M + i] * q;
    tr1 += ik * H[l * MM + (int64_t)j * M + i];
  }
  for (int i = tid; i < M; i += kStep) qf1 += m[(int64_t)l * M + i] * t[(int64_t)l * M + i];
  double vals[9] = {A, Bt, C, D1, D2, E, F, tr1, qf1};
  double* pp = part + ((int64_t)l * kHnSlices + sl) * 16;
#pragma unroll
  for (int q = 0; q < 9; ++q) {
    const double v = block_sum<256>(vals[q], red);
    if (threadIdx.x == 0) pp[q] = v;
  }
  if (threadIdx.x == 0) {
    pp[9] = sl == 0 ? ldK[l] : 0.0;
    pp[10] = sl == 0 ? ldH[l] : 0.0;
  }
}

__global__ void hn_final_kernel(int L, int M, double P_tot, int P_b, double n_total, const double* __restrict__ part,
                                double* __restrict__ kld) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double tot = 0.0;
  const double c0 = P_tot / (double)P_b;
  for (int l = 0; l < L; ++l) {
    double p[11];  // the slices' sums, in slice order
    for (int q = 0; q < 11; ++q) {
      p[q] = 0.0;
      for (int sl = 0; sl < kHnSlices; ++sl) p[q] += part[((int64_t)l * kHnSlices + sl) * 16 + q];
    }
    const double inner = p[0] + p[1] + p[2] + (p[3] - p[4]) + p[5] - p[6];
    const double klu = 0.5 * (p[7] + p[8] - (double)M + p[9] - p[10]);
    tot += c0 * 0.5 * inner + klu;
  }
  kld[0] = tot - (double)L * n_total / 2.0;
}

// y = alpha * x + beta * y  (n elements), optional scale from device scalar: alpha *= *g, beta *= *g
__global__ void axpby_kernel(int64_t n, double alpha, const double* __restrict__ x, double beta,
                             double* __restrict__ y, const double* __restrict__ ga, const double* __restrict__ gb) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const double al = ga ? alpha * ga[0] : alpha;
  const double be = gb ? beta * gb[0] : beta;
  y[e] = al * x[e] + (be == 0.0 ? 0.0 : be * y[e]);
}

// z = ax * x + ay * y (+ az * w), coefficients optionally scaled by device scalar g
__global__ void lincomb_kernel(int64_t n, double ax, const double* x, double ay, const double* y, double* z,
                               const double* __restrict__ g,
                               int scale_x, int scale_y) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const double gg = g ? g[0] : 1.0;
  const double cx = scale_x ? ax * gg : ax, cy = scale_y ? ay * gg : ay;
  z[e] = cx * x[e] + (y ? cy * y[e] : 0.0);
}

// dmu[i][l] = -2c s[l][i];  dlogv[i][l] = c (iB_ii v_i - 1)
__global__ void hn_bwd_vec_kernel(int P_b, int T, int L, double k, const double* __restrict__ g,
                                  const double* __restrict__ s, const double* __restrict__ iB,
                                  const double* __restrict__ logv, const int32_t* __restrict__ seg,
                                  double* __restrict__ dmu, double* __restrict__ dlogv) {
  const int B = P_b * T;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * L) return;
  const int l = e / B, i = e % B, p = i / T, q = i % T;
  const double c = k * g[0];
  dmu[(int64_t)i * L + l] = -2.0 * c * s[e];
  const double d = iB[((int64_t)l * P_b + p) * T * T + q * T + q];
  dlogv[(int64_t)i * L + l] = seg_valid(seg, p, q) ? c * (d * exp(logv[(int64_t)i * L + l]) - 1.0) : 0.0;
}

// X[l][i][j] += a * u[l][i] * v[l][j]  (a scaled by device g)
__global__ void outer_add_kernel(int L, int n1, int n2, double a, const double* __restrict__ g,
                                 const double* __restrict__ u, const double* __restrict__ v,
                                 double* __restrict__ X) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)L * n1 * n2) return;
  const int l = (int)(e / ((int64_t)n1 * n2));
  const int64_t rem = e - (int64_t)l * n1 * n2;
  const int i = (int)(rem / n2), j = (int)(rem % n2);
  X[e] += a * g[0] * u[(int64_t)l * n1 + i] * v[(int64_t)l * n2 + j];
}

// G_iK = c (2 v1 m^T - Q + Z + Z^T) + h (H + m m^T)
__global__ void giK_kernel(int L, int M, double kc, double kh, const double* __restrict__ g,
                           const double* __restrict__ v1, const double* __restrict__ m,
                           const double* __restrict__ Q, const double* __restrict__ Z,
                           const double* __restrict__ H, double* __restrict__ G) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t MM = (int64_t)M * M;
  if (e >= L * MM) return;
  const int l = (int)(e / MM);
  const int i = (int)((e % MM) / M), j = (int)(e % M);
  const double c = kc * g[0], h = kh * g[0];
  const double* mm = m + (int64_t)l * M;
  const int64_t b = l * MM;
  G[e] = c * (2.0 * v1[(int64_t)l * M + i] * mm[j] - Q[e] + Z[e] + Z[b + (int64_t)j * M + i]) +
         h * (H[e] + mm[i] * mm[j]);
}

// VB[l,p][i][j] = v_{l,p,i} iB[l,p][i][j]
__global__ void rowscale_v_kernel(int P_b, int T, int L, const double* __restrict__ logv,
                                  const double* __restrict__ iB, const int32_t* __restrict__ seg,
                                  double* __restrict__ VB) {
  const int64_t TT = (int64_t)T * T;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)L * P_b * TT) return;
  const int lp = (int)(e / TT), l = lp / P_b, p = lp % P_b;
  const int i = (int)((e % TT) / T);
  VB[e] = seg_valid(seg, p, i) ? exp(logv[((int64_t)p * T + i) * L + l]) * iB[e] : 0.0;
}

// GB = c (iB - s s^T - iBVB - iBK0iB) - QB ;  GK0 = c iB
__global__ void gb_kernel(int P_b, int T, int L, double kc, const double* __restrict__ g,
                          const double* __restrict__ iB, const double* __restrict__ s,
                          const double* __restrict__ iBVB, const double* __restrict__ iBK0iB,
                          const double* __restrict__ QB, const int32_t* __restrict__ seg,
                          double* __restrict__ GB, double* __restrict__ GK0) {
  const int64_t TT = (int64_t)T * T;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)L * P_b * TT) return;
  const int lp = (int)(e / TT), l = lp / P_b, p = lp % P_b;
  const int i = (int)((e % TT) / T), j = (int)(e % T);
  const double c = kc * g[0];
  const int B = P_b * T;
  const double si = s[(int64_t)l * B + p * T + i], sj = s[(int64_t)l * B + p * T + j];
  const bool ok = seg_valid(seg, p, i) && seg_valid(seg, p, j);
  GB[e] = ok ? c * (iB[e] - si * sj - iBVB[e] - iBK0iB[e]) - QB[e] : 0.0;
  GK0[e] = ok ? c * iB[e] : 0.0;
}

// Y[l][i][j] += a * X[l][j][i]
__global__ void add_transpose_kernel(int L, int M, double a, const double* __restrict__ X, double* __restrict__ Y) {
  const int64_t MM = (int64_t)M * M;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= L * MM) return;
  const int64_t l = e / MM;
  const int i = (int)((e % MM) / M), j = (int)(e % M);
  Y[e] += a * X[l * MM + (int64_t)j * M + i];
}

// info[l]: first failure among K0zz[l] (10000 + col), B_{l,p} (20000 + col), H[l] (30000 + col)
__global__ void hn_info_kernel(int L, int P_b, const int32_t* __restrict__ w, int32_t* __restrict__ info) {
  const int l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= L) return;
  int v = 0;
  if (w[l]) v = 10000 + w[l];
  for (int p = 0; p < P_b && !v; ++p)
    if (w[L + l * P_b + p]) v = 20000 + w[L + l * P_b + p];
  if (!v && w[L + L * P_b + l]) v = 30000 + w[L + L * P_b + l];
  info[l] = v;
}

inline int blocks(int64_t n) { return cdiv(n, 256); }

}  // namespace



static int hensman_check(const lvae_kernel_spec* s0, const lvae_kernel_spec* s1, const lvae_hensman_dims* d) {
  if (!s0 || !spec_bucket(s0)) return -1;
  if (!s1 || !spec_bucket(s1)) return -2;
  if (!d || d->L < 1 || d->M < 1 || d->M > 128 || d->P_b < 1 || d->T < 1 || d->T > 128 || d->Q < 1) return -3;
  return 0;
}

}  // namespace lvae

using namespace lvae;

extern "C" {

size_t lvae_hensman_workspace_size(const lvae_hensman_dims* d) { return HWs(nullptr, *d).bytes; }

size_t lvae_hensman_iH_offset(const lvae_hensman_dims* d) {
  char* const base = reinterpret_cast<char*>(uintptr_t(4096));  // any non-null base: offsets only
  return (size_t)((char*)HWs(base, *d).iH - base);
}

// part 1: everything that needs neither mu nor logv (the Grams, the three inverses, t / y, iBK, Q, iK H iK
// and the data-independent natural-gradient terms) -- a caller can run it beside the encoder; part 2: the
// rest (the residual, s, the sums, u / w / a, grad_m, info); part 0: both, in that order.
int lvae_hensman_fwd_part_f64(int part, const lvae_kernel_spec* spec0, const lvae_kernel_spec* spec1,
                              const lvae_hensman_dims* dp, const double* x, const double* z, const double* m,
                              const double* H, const double* mu, const double* logv, const double* params0,
                              const double* params1, const double* noise, double* kld, double* grad_m,
                              double* grad_H, int32_t* info, void* workspace, void* stream) {
  LVAE_TRY(hensman_check(spec0, spec1, dp));
  if (part < 0 || part > 2) return -18;
  if (!workspace || ((uintptr_t)workspace & 255)) return -17;
  hipStream_t st = (hipStream_t)stream;
  ProfScope ps(LVAE_PH_HENSMAN_FWD, st);
  const lvae_hensman_dims& d = *dp;
  const int L = d.L, M = d.M, P_b = d.P_b, T = d.T, Q = d.Q, B = P_b * T;
  const int64_t MM = (int64_t)M * M, TT = (int64_t)T * T, BM = (int64_t)B * M;
  HWs w((char*)workspace, d);
  const bool ng = d.natural_gradient && grad_m && grad_H;
  const double share = d.ng_prior_share;
  if (part != 2) {
    // Grams (elbo_functions.py:171-176)
    fill_kernel<<<blocks(L), 256, 0, st>>>(w.epsv, L, d.eps);
    const lvae_xview xv{x, 0, 0, Q}, zv{z, 0, (int64_t)M * Q, Q}, xs{x, (int64_t)T * Q, 0, Q};
    // (the four in one launch: gram_multi_f64)
    const lvae_kernel_spec* specs[2] = {spec0, spec1};
    const GramFwdJob jobs[4] = {
        {0, 1, B, M, 0, 0, 0, xv, zv, params0, nullptr, w.K0xz, 0, BM, M},
        {0, 1, M, M, 0, 0, 0, zv, zv, params0, w.epsv, w.K0zz, 0, MM, M},
        {0, P_b, T, T, 0, 0, 0, xs, xs, params0, nullptr, w.K0st, TT, P_b * TT, T},
        {1, P_b, T, T, 0, 0, 0, xs, xs, params1, noise, w.Bst, TT, P_b * TT, T}};
    LVAE_TRY(gram_multi_f64(specs, jobs, 4, L, st));
    if (d.seg_len)
      hn_seg_mask_kernel<<<blocks((int64_t)L * B * M + (int64_t)L * P_b * TT), 256, 0, st>>>(
          L, P_b, T, M, d.seg_len, w.K0xz, w.K0st, w.Bst);
    // factor + inverse (177-186)
    LVAE_TRY(spd_inv_small2_f64(M, L, w.K0zz, MM, w.iK, MM, w.ldK, w.info, L, H, MM, w.iH, MM, w.ldH,
                                w.info + L + L * P_b, st));
    LVAE_TRY(spd_inv_small_f64(T, L * P_b, w.Bst, TT, w.iB, TT, w.ldB, w.info + L, st));
    // t = iK m ; y = K0xz t ; iBK = iB K0xz ; Q = K0xz^T iBK ; Y = iK H iK
    LVAE_TRY(gemm_small_f64(0, 0, M, 1, M, 1.0, w.iK, M, MM, 0, m, 1, M, 0, 0.0, w.t, 1, M, 0, L, 1, st));
    LVAE_TRY(gemm_small_f64(0, 0, B, 1, M, 1.0, w.K0xz, M, BM, 0, w.t, 1, M, 0, 0.0, w.y, 1, B, 0, L, 1, st));
    LVAE_TRY(gemm_small_f64(0, 0, T, M, T, 1.0, w.iB, T, P_b * TT, TT, w.K0xz, M, BM, (int64_t)T * M, 0.0, w.iBK,
                            M, BM, (int64_t)T * M, L, P_b, st));
    LVAE_TRY(gemm_small_f64(1, 0, M, M, B, 1.0, w.K0xz, M, BM, 0, w.iBK, M, BM, 0, 0.0, w.Q, M, MM, 0, L, 1, st));
    LVAE_TRY(gemm_small_f64(0, 0, M, M, M, 1.0, w.iK, M, MM, 0, H, M, MM, 0, 0.0, w.iKH, M, MM, 0, L, 1, st));
    LVAE_TRY(gemm_small_f64(0, 0, M, M, M, 1.0, w.iKH, M, MM, 0, w.iK, M, MM, 0, 0.0, w.Y, M, MM, 0, L, 1, st));
    if (ng) {  // the data-independent natural-gradient terms (208-214)
      // Bn = iK Q iK + share iK ; tM = Bn m ; grad_H = 1/2 (Bn - share iH)
      LVAE_TRY(gemm_small_f64(0, 0, M, M, M, 1.0, w.iK, M, MM, 0, w.Q, M, MM, 0, 0.0, w.iKQ, M, MM, 0, L, 1, st));
      axpby_kernel<<<blocks(L * MM), 256, 0, st>>>(L * MM, share, w.iK, 0.0, w.Bn, nullptr, nullptr);
      LVAE_TRY(gemm_small_f64(0, 0, M, M, M, 1.0, w.iKQ, M, MM, 0, w.iK, M, MM, 0, 1.0, w.Bn, M, MM, 0, L, 1, st));
      LVAE_TRY(gemm_small_f64(0, 0, M, 1, M, 1.0, w.Bn, M, MM, 0, m, 1, M, 0, 0.0, w.tM, 1, M, 0, L, 1, st));
      lincomb_kernel<<<blocks(L * MM), 256, 0, st>>>(L * MM, 0.5, w.Bn, -0.5 * share, w.iH, grad_H, nullptr, 0, 0);
    }
  }
  if (part != 1) {
    // r = y - mu ; s = iB r
    resid_kernel<<<blocks((int64_t)B * L), 256, 0, st>>>(w.y, mu, B, L, T, d.seg_len, w.r);
    LVAE_TRY(gemm_small_f64(0, 0, T, 1, T, 1.0, w.iB, T, P_b * TT, TT, w.r, 1, B, T, 0.0, w.s, 1, B, T, L, P_b, st));
    // partial sums + total (189-204)
    hn_reduce_kernel<<<dim3(L, kHnSlices), 256, 0, st>>>(M, P_b, T, L, w.r, w.s, w.iB, logv, w.ldB, w.K0st, w.Q, w.iK, w.Y, H, m,
                                        w.t, w.ldK, w.ldH, d.seg_len, w.part);
    hn_final_kernel<<<1, 64, 0, st>>>(L, M, d.P_tot, P_b, d.n_total > 0.0 ? d.n_total : d.P_tot * T, w.part, kld);
    if (ng) {  // u = iB mu ; w = K0xz^T u ; a = iK w ; grad_m = Bn m - a
      LVAE_TRY(gemm_small_f64(0, 0, T, 1, T, 1.0, w.iB, T, P_b * TT, TT, mu, L, 1, (int64_t)T * L, 0.0, w.u, 1, B,
                              T, L, P_b, st));
      LVAE_TRY(gemm_small_f64(1, 0, M, 1, B, 1.0, w.K0xz, M, BM, 0, w.u, 1, B, 0, 0.0, w.w, 1, M, 0, L, 1, st));
      LVAE_TRY(gemm_small_f64(0, 0, M, 1, M, 1.0, w.iK, M, MM, 0, w.w, 1, M, 0, 0.0, w.a, 1, M, 0, L, 1, st));
      lincomb_kernel<<<blocks((int64_t)L * M), 256, 0, st>>>((int64_t)L * M, 1.0, w.tM, -1.0, w.a, grad_m, nullptr,
                                                              0, 0);
    }
    // info: first failing matrix (K0zz, then B_p, then H) per latent dim
    if (info) hn_info_kernel<<<blocks(L), 256, 0, st>>>(L, P_b, w.info, info);
  }
  LVAE_CHECK_LAUNCH();
  return 0;
}

int lvae_hensman_fwd_f64(const lvae_kernel_spec* spec0, const lvae_kernel_spec* spec1, const lvae_hensman_dims* dp,
                         const double* x, const double* z, const double* m, const double* H, const double* mu,
                         const double* logv, const double* params0, const double* params1, const double* noise,
                         double* kld, double* grad_m, double* grad_H, int32_t* info, void* workspace, void* stream) {
  return lvae_hensman_fwd_part_f64(0, spec0, spec1, dp, x, z, m, H, mu, logv, params0, params1, noise, kld, grad_m,
                                   grad_H, info, workspace, stream);
}

int lvae_hensman_bwd_f64(const lvae_kernel_spec* spec0, const lvae_kernel_spec* spec1, const lvae_hensman_dims* dp,
                         const double* x, const double* z, const double* m, const double* H, const double* mu,
                         const double* logv, const double* params0, const double* params1, const double* noise,
                         const double* gkld, double* dmu, double* dlogv, double* dparams0, double* dparams1,
                         double* dnoise, double* dm, double* dH, void* workspace, void* stream) {
  (void)mu;
  (void)noise;
  LVAE_TRY(hensman_check(spec0, spec1, dp));
  if (!workspace || ((uintptr_t)workspace & 255)) return -21;
  hipStream_t st = (hipStream_t)stream;
  ProfScope ps(LVAE_PH_HENSMAN_BWD, st);
  const lvae_hensman_dims& d = *dp;
  const int L = d.L, M = d.M, P_b = d.P_b, T = d.T, Q = d.Q, B = P_b * T;
  const int64_t MM = (int64_t)M * M, TT = (int64_t)T * T, BM = (int64_t)B * M, LTT = (int64_t)L * P_b * TT;
  const double kc = d.P_tot / (2.0 * P_b), kh = 0.5;
  HWs w((char*)workspace, d);
  // mu / logv
  hn_bwd_vec_kernel<<<blocks((int64_t)B * L), 256, 0, st>>>(P_b, T, L, kc, gkld, w.s, w.iB, logv, d.seg_len, dmu,
                                                            dlogv);
  // Xq = c (Y - iK)
  lincomb_kernel<<<blocks(L * MM), 256, 0, st>>>(L * MM, kc, w.Y, -kc, w.iK, w.Xq, gkld, 1, 1);
  // dK0xz = 2 iBK Xq + 2c s t^T
  LVAE_TRY(gemm_small_f64(0, 0, B, M, M, 2.0, w.iBK, M, BM, 0, w.Xq, M, MM, 0, 0.0, w.dK0xz, M, BM, 0, L, 1, st));
  outer_add_kernel<<<blocks((int64_t)L * BM), 256, 0, st>>>(L, B, M, 2.0 * kc, gkld, w.s, w.t, w.dK0xz);
  // v1 = K0xz^T s ; Z = Q iK H ; G_iK ; dK0zz = -iK G_iK iK + h iK
  LVAE_TRY(gemm_small_f64(1, 0, M, 1, B, 1.0, w.K0xz, M, BM, 0, w.s, 1, B, 0, 0.0, w.v1, 1, M, 0, L, 1, st));
  LVAE_TRY(gemm_small_f64(0, 0, M, M, M, 1.0, w.Q, M, MM, 0, w.iKH, M, MM, 0, 0.0, w.Z, M, MM, 0, L, 1, st));
  giK_kernel<<<blocks(L * MM), 256, 0, st>>>(L, M, kc, kh, gkld, w.v1, m, w.Q, w.Z, H, w.GiK);
  LVAE_TRY(gemm_small_f64(0, 0, M, M, M, 1.0, w.iK, M, MM, 0, w.GiK, M, MM, 0, 0.0, w.T1, M, MM, 0, L, 1, st));
  lincomb_kernel<<<blocks(L * MM), 256, 0, st>>>(L * MM, kh, w.iK, 0.0, nullptr, w.dK0zz, gkld, 1, 0);
  LVAE_TRY(gemm_small_f64(0, 0, M, M, M, -1.0, w.T1, M, MM, 0, w.iK, M, MM, 0, 1.0, w.dK0zz, M, MM, 0, L, 1, st));
  // dB_p and dK0_p
  rowscale_v_kernel<<<blocks(LTT), 256, 0, st>>>(P_b, T, L, logv, w.iB, d.seg_len, w.VB);
  LVAE_TRY(gemm_small_f64(0, 0, T, T, T, 1.0, w.iB, T, P_b * TT, TT, w.VB, T, P_b * TT, TT, 0.0, w.iBVB, T,
                          P_b * TT, TT, L, P_b, st));
  LVAE_TRY(gemm_small_f64(0, 0, T, T, T, 1.0, w.K0st, T, P_b * TT, TT, w.iB, T, P_b * TT, TT, 0.0, w.K0iB, T,
                          P_b * TT, TT, L, P_b, st));
  LVAE_TRY(gemm_small_f64(0, 0, T, T, T, 1.0, w.iB, T, P_b * TT, TT, w.K0iB, T, P_b * TT, TT, 0.0, w.iBK0iB, T,
                          P_b * TT, TT, L, P_b, st));
  LVAE_TRY(gemm_small_f64(0, 0, T, M, M, 1.0, w.iBK, M, BM, (int64_t)T * M, w.Xq, M, MM, 0, 0.0, w.tBM, M, BM,
                          (int64_t)T * M, L, P_b, st));
  LVAE_TRY(gemm_small_f64(0, 1, T, T, M, 1.0, w.tBM, M, BM, (int64_t)T * M, w.iBK, M, BM, (int64_t)T * M, 0.0, w.QB,
                          T, P_b * TT, TT, L, P_b, st));
  gb_kernel<<<blocks(LTT), 256, 0, st>>>(P_b, T, L, kc, gkld, w.iB, w.s, w.iBVB, w.iBK0iB, w.QB, d.seg_len, w.GB,
                                          w.GK0);
  // hyper-parameter gradients through the four Grams
  (void)zero_async(dparams0, sizeof(double) * L * spec0->n_params, st);
  (void)zero_async(dparams1, sizeof(double) * L * spec1->n_params, st);
  if (dnoise) (void)zero_async(dnoise, sizeof(double) * L, st);
  const lvae_xview xv{x, 0, 0, Q}, zv{z, 0, (int64_t)M * Q, Q}, xs{x, (int64_t)T * Q, 0, Q};
  {
    const GramBwdJob jobs[4] = {
        {0, xv, zv, 1, B, M, 0, params0, w.dK0xz, 0, BM, M, dparams0, nullptr, 0, 0},
        {0, zv, zv, 1, M, M, 0, params0, w.dK0zz, 0, MM, M, dparams0, nullptr, 0, 0},
        {0, xs, xs, P_b, T, T, 0, params0, w.GK0, TT, P_b * TT, T, dparams0, nullptr, 0, 0},
        {1, xs, xs, P_b, T, T, 0, params1, w.GB, TT, P_b * TT, T, dparams1, dnoise, 0, 0}};
    const lvae_kernel_spec* specs[2] = {spec0, spec1};
    LVAE_TRY(gram_bwd_multi_f64(specs, jobs, 4, L, w.gpart, st));
  }
  // Adam path: gradients wrt m and H
  if (!d.natural_gradient && dm && dH) {
    LVAE_TRY(gemm_small_f64(0, 0, M, 1, M, 1.0, w.iK, M, MM, 0, w.v1, 1, M, 0, 0.0, w.tM, 1, M, 0, L, 1, st));
    lincomb_kernel<<<blocks((int64_t)L * M), 256, 0, st>>>((int64_t)L * M, 2.0 * kc, w.tM, 1.0, w.t, dm, gkld, 1, 1);
    LVAE_TRY(gemm_small_f64(0, 0, M, M, M, 1.0, w.iK, M, MM, 0, w.Q, M, MM, 0, 0.0, w.iKQ, M, MM, 0, L, 1, st));
    lincomb_kernel<<<blocks(L * MM), 256, 0, st>>>(L * MM, kh, w.iK, -kh, w.iH, dH, gkld, 1, 1);
    LVAE_TRY(gemm_small_f64(0, 0, M, M, M, 1.0, w.iKQ, M, MM, 0, w.iK, M, MM, 0, 0.0, w.tMM, M, MM, 0, L, 1, st));
    axpby_kernel<<<blocks(L * MM), 256, 0, st>>>(L * MM, kc, w.tMM, 1.0, dH, gkld, nullptr);
  }
  LVAE_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------------------------------
// natural-gradient update (training.py:129-135)
// ------------------------------------------------------------------------------------------
size_t lvae_natgrad_workspace_size(int L, int M) {
  const size_t mm = align256((size_t)L * M * M * sizeof(double)), v = align256((size_t)L * M * sizeof(double));
  return 3 * mm + 3 * v + align256((size_t)L * sizeof(double)) + align256((size_t)2 * L * sizeof(int32_t));
}

// iHn = iH + lr (gH + gH^T) in one pass (was a copy, an axpy and a transpose-add)
// (and inf0[0..L) = 0 when H^-1 came from the caller: no factorisation of H here -- a kernel store, not a
// hipMemsetAsync node: see DESIGN.md section 5 on the captured memsets)
__global__ void natgrad_ih_kernel(int L, int M, double lr, const double* __restrict__ iH, const double* __restrict__ gH,
                                  double* __restrict__ iHn, int32_t* __restrict__ inf0) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, MM = (int64_t)M * M;
  if (inf0 && e < L) inf0[e] = 0;
  if (e >= L * MM) return;
  const int64_t b = e / MM, r = (e % MM) / M, c = e % M;
  iHn[e] = iH[e] + lr * (gH[e] + gH[b * MM + c * M + r]);
}

// y = v - lr gm + 2 lr gw
__global__ void natgrad_y_kernel(int64_t n, double lr, const double* __restrict__ v, const double* __restrict__ gm,
                                 const double* __restrict__ gw, double* __restrict__ y) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n) y[e] = v[e] - lr * gm[e] + 2.0 * lr * gw[e];
}

// commit: (m, H) <- (mn, Hn) for EVERY dim only if all factorisations of all dims (H^-1 when it was computed here,
// iH'^-1) succeeded, as the reference's batched torch.cholesky raises before anything is assigned
// (training.py:130-134); info[l] = dim l's first failure's LAPACK code (H's, else iH''s), 0 = ok
__global__ void natgrad_commit_kernel(int L, int M, const int32_t* __restrict__ inf, const double* __restrict__ Hn,
                                      const double* __restrict__ mn, double* __restrict__ H, double* __restrict__ m,
                                      int32_t* __restrict__ info) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, MM = (int64_t)M * M;
  int bad = 0;
  for (int q = 0; q < 2 * L; ++q) bad |= inf[q];
  if (e < L * MM) {
    if (!bad) H[e] = Hn[e];
  } else if (e < L * MM + (int64_t)L * M) {
    const int64_t q = e - L * MM;
    const int l = (int)(q / M);
    if (!bad) m[q] = mn[q];
    if (q % M == 0 && info) info[l] = inf[l] != 0 ? inf[l] : inf[L + l];
  }
}

int lvae_natgrad_update_f64(int L, int M, double* m, double* H, const double* grad_m, const double* grad_H, double lr,
                            const double* iH_in, int32_t* info, void* workspace, void* stream) {
  if (L < 1) return -1;
  if (M < 1 || M > 128) return -2;
  if (!workspace || ((uintptr_t)workspace & 255)) return -9;
  hipStream_t st = (hipStream_t)stream;
  ProfScope ps(LVAE_PH_NATGRAD, st);
  const int64_t MM = (int64_t)M * M;
  const size_t mmb = align256((size_t)L * MM * sizeof(double)), vb = align256((size_t)L * M * sizeof(double));
  char* base = (char*)workspace;
  double* iH = (double*)base;
  const double* iHc = iH_in ? iH_in : iH;
  double* iHn = (double*)(base + mmb);
  double* Hn = (double*)(base + 2 * mmb);
  double* v = (double*)(base + 3 * mmb);
  double* gw = (double*)(base + 3 * mmb + vb);
  double* y = (double*)(base + 3 * mmb + 2 * vb);
  double* ld = (double*)(base + 3 * mmb + 3 * vb);
  int32_t* inf = (int32_t*)(base + 3 * mmb + 3 * vb + align256((size_t)L * sizeof(double)));
  if (!iH_in) LVAE_TRY(spd_inv_small_f64(M, L, H, MM, iH, MM, ld, inf, st));
  // iH' = iH + lr (gH + gH^T)
  natgrad_ih_kernel<<<blocks(L * MM), 256, 0, st>>>(L, M, lr, iHc, grad_H, iHn, iH_in ? inf : nullptr);
  // v = iH m ; gw = gH m; Hn = iH'^-1; y = v - lr gm + 2 lr gw ; mn = Hn y (into gw, dead after y); then the
  // commit writes (mn, Hn) over (m, H) for the dims whose factorisations succeeded
  LVAE_TRY(gemm_small_f64(0, 0, M, 1, M, 1.0, iHc, M, MM, 0, m, 1, M, 0, 0.0, v, 1, M, 0, L, 1, st));
  LVAE_TRY(gemm_small_f64(0, 0, M, 1, M, 1.0, grad_H, M, MM, 0, m, 1, M, 0, 0.0, gw, 1, M, 0, L, 1, st));
  LVAE_TRY(spd_inv_small_f64(M, L, iHn, MM, Hn, MM, ld, inf + L, st));
  natgrad_y_kernel<<<blocks((int64_t)L * M), 256, 0, st>>>((int64_t)L * M, lr, v, grad_m, gw, y);
  LVAE_TRY(gemm_small_f64(0, 0, M, 1, M, 1.0, Hn, M, MM, 0, y, 1, M, 0, 0.0, gw, 1, M, 0, L, 1, st));
  natgrad_commit_kernel<<<blocks(L * MM + (int64_t)L * M), 256, 0, st>>>(L, M, inf, Hn, gw, H, m, info);
  LVAE_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
