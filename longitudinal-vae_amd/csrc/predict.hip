// predict.hip -- GP posterior mean of the latents at test covariates, for subjects of varying
// length: utils.batch_predict_varying_T (utils.py:115-211), as used by MSE_test_GPapprox
// (model_test.py:85-143).  fp64 (same M x M / T x T systems as the Hensman bound).
//
// Prediction set: P subjects laid out [P, T] (T = longest subject; seg_len[p] valid rows, the
// rest padding), encoder means mu [P*T, L].  Per latent dim:
//   B_p = k1(x_p, x_p) + noise I,  iB = B^-1 (block diagonal),  H = K0zz + K0xz^T iB K0xz
//   mu~ = iB mu - iB K0xz H^-1 K0xz^T iB mu
//   Z(X*) = K0X*z K0zz^-1 K0xz^T mu~ + k1(X*, x[test subjects]) mu~[test subjects]
// The reference's per-subject Python loops become one batched pass (padding rows of K0xz zeroed,
// padding blocks of B set to I, padding rows of mu zeroed by the caller).  The k1 term is the
// reference's dense product over all prediction rows of the test subjects (include[p] = 1),
// evaluated in chunks of test rows.
#include "common.hpp"
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

constexpr int64_t kPredChunkElems = 1 << 24;  // k1(X*, x) chunk: <= 128 MiB of fp64

struct PWs {
  double *K0xz, *iBK, *K0zz, *Hm, *iK, *iH, *Bst, *iB, *iBmu, *t, *muT, *muTm, *w, *v, *a, *b, *K0Xz, *out1, *K1;
  double *ldK, *ldH, *ldB;
  int32_t* info;
  int64_t chunk_rows;
  size_t bytes;
  PWs(char* base, int L, int M, int P, int T, int Nt) {
    size_t off = 0;
    auto take = [&](size_t n) {
      double* p = base ? (double*)(base + off) : nullptr;
      off += align256(n * sizeof(double));
      return p;
    };
    const size_t NP = (size_t)P * T, LMM = (size_t)L * M * M, LTT = (size_t)L * P * T * T;
    K0xz = take(L * NP * M);
    iBK = take(L * NP * M);
    K0zz = take(LMM);
    Hm = take(LMM);
    iK = take(LMM);
    iH = take(LMM);
    Bst = take(LTT);
    iB = take(LTT);
    iBmu = take(L * NP);
    t = take(L * NP);
    muT = take(L * NP);
    muTm = take(L * NP);
    w = take((size_t)L * M);
    v = take((size_t)L * M);
    a = take((size_t)L * M);
    b = take((size_t)L * M);
    K0Xz = take((size_t)L * Nt * M);
    out1 = take((size_t)L * Nt);
    int64_t rows = kPredChunkElems / ((int64_t)L * (int64_t)NP);
    if (rows < 1) rows = 1;
    if (rows > Nt) rows = Nt;
    chunk_rows = rows;
    K1 = take((size_t)L * rows * NP);
    ldK = take(L);
    ldH = take(L);
    ldB = take((size_t)L * P);
    info = (int32_t*)take((size_t)2 * L + (size_t)L * P);
    bytes = off;
  }
};

__device__ inline bool pv(const int32_t* __restrict__ seg, int p, int q) { return q < seg[p]; }

// padding: K0xz rows -> 0, B_p rows/cols -> I
__global__ void pr_mask_kernel(int L, int P, int T, int M, const int32_t* __restrict__ seg, double* __restrict__ K0xz,
                               double* __restrict__ Bst) {
  const int64_t NP = (int64_t)P * T, nxz = (int64_t)L * NP * M, TT = (int64_t)T * T, nst = (int64_t)L * P * TT;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < nxz) {
    const int64_t row = (e / M) % NP;
    if (!pv(seg, (int)(row / T), (int)(row % T))) K0xz[e] = 0.0;
  } else if (e < nxz + nst) {
    const int64_t f = e - nxz;
    const int p = (int)((f / TT) % P), i = (int)((f % TT) / T), j = (int)(f % T);
    if (!pv(seg, p, i) || !pv(seg, p, j)) Bst[f] = (i == j) ? 1.0 : 0.0;
  }
}

// muT = iBmu - corr ; muTm = muT on the included subjects' valid rows, 0 elsewhere
__global__ void pr_mutilde_kernel(int L, int P, int T, const int32_t* __restrict__ seg,
                                  const int32_t* __restrict__ include, const double* __restrict__ iBmu,
                                  const double* __restrict__ corr, double* __restrict__ muT, double* __restrict__ muTm) {
  const int64_t NP = (int64_t)P * T;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= L * NP) return;
  const int64_t row = e % NP;
  const int p = (int)(row / T), q = (int)(row % T);
  const bool ok = pv(seg, p, q);
  const double v = ok ? iBmu[e] - corr[e] : 0.0;
  muT[e] = v;
  muTm[e] = (ok && include[p]) ? v : 0.0;
}

// K0zz += eps I ; Hm += K0zz
__global__ void pr_eye_add_kernel(int L, int M, double eps, double* __restrict__ K0zz, double* __restrict__ Hm) {
  const int64_t MM = (int64_t)M * M;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= L * MM) return;
  const int i = (int)((e % MM) / M), j = (int)(e % M);
  const double k = K0zz[e] + (i == j ? eps : 0.0);
  K0zz[e] = k;
  Hm[e] += k;
}

// info[l]: first failing factorisation: K0zz (10000 + col), H (30000 + col), B_p (20000 + col)
__global__ void pr_info_kernel(int L, int P, const int32_t* __restrict__ w, int32_t* __restrict__ info) {
  const int l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= L) return;
  int v = 0;
  if (w[l]) v = 10000 + w[l];
  for (int p = 0; p < P && !v; ++p)
    if (w[2 * L + l * P + p]) v = 20000 + w[2 * L + l * P + p];
  if (!v && w[L + l]) v = 30000 + w[L + l];
  info[l] = v;
}

// out[i][l] = out1[l][i]
__global__ void pr_out_kernel(int L, int Nt, const double* __restrict__ out1, double* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)L * Nt) return;
  const int i = (int)(e / L), l = (int)(e % L);
  out[e] = out1[(int64_t)l * Nt + i];
}

inline int nblk(int64_t n) { return cdiv(n, 256); }

}  // namespace
}  // namespace lvae

using namespace lvae;

extern "C" {

size_t lvae_predict_workspace_size(int L, int M, int P, int T, int Nt) {
  return PWs(nullptr, L, M, P, T, Nt > 0 ? Nt : 1).bytes;
}

int lvae_predict_f64(const lvae_kernel_spec* spec0, const lvae_kernel_spec* spec1, int L, int M, int Q, int P, int T,
                     const int32_t* seg_len, const int32_t* include, const double* x, const double* mu,
                     const double* z, int Nt, const double* test_x, const double* params0, const double* params1,
                     const double* noise, double eps, double* out, int32_t* info, void* workspace, void* stream) {
  if (!spec0 || !spec1) return -1;
  if (L < 1 || M < 1 || M > 128) return -3;
  if (P < 1 || T < 1 || T > 128 || Q < 1) return -6;
  if (!seg_len || !include) return -8;
  if (Nt < 0) return -13;
  if (!workspace || ((uintptr_t)workspace & 255)) return -20;
  hipStream_t st = (hipStream_t)stream;
  PWs w((char*)workspace, L, M, P, T, Nt > 0 ? Nt : 1);
  const int NP = P * T;
  const int64_t MM = (int64_t)M * M, TT = (int64_t)T * T, NPM = (int64_t)NP * M;
  // Grams (utils.py:139-160): K0xz [L,NP,M], K0zz + eps I, K0X*z [L,Nt,M], B_p = k1(x_p, x_p) + noise I
  const lvae_xview xv{x, 0, 0, Q}, zv{z, 0, (int64_t)M * Q, Q}, xs{x, (int64_t)T * Q, 0, Q}, tv{test_x, 0, 0, Q};
  LVAE_TRY(lvae_gram_f64(spec0, xv, zv, 1, L, NP, M, params0, nullptr, w.K0xz, 0, NPM, M, stream));
  LVAE_TRY(lvae_gram_f64(spec0, zv, zv, 1, L, M, M, params0, nullptr, w.K0zz, 0, MM, M, stream));
  LVAE_TRY(lvae_gram_f64(spec1, xs, xs, P, L, T, T, params1, noise, w.Bst, TT, (int64_t)P * TT, T, stream));
  if (Nt > 0) LVAE_TRY(lvae_gram_f64(spec0, tv, zv, 1, L, Nt, M, params0, nullptr, w.K0Xz, 0, (int64_t)Nt * M, M, stream));
  pr_mask_kernel<<<nblk((int64_t)L * NPM + (int64_t)L * P * TT), 256, 0, st>>>(L, P, T, M, seg_len, w.K0xz, w.Bst);
  // iB (per subject), iB mu, iB K0xz
  LVAE_TRY(spd_inv_small_f64(T, L * P, w.Bst, TT, w.iB, TT, w.ldB, w.info + 2 * L, st));
  LVAE_TRY(gemm_small_f64(0, 0, T, 1, T, 1.0, w.iB, T, (int64_t)P * TT, TT, mu, L, 1, (int64_t)T * L, 0.0, w.iBmu, 1,
                          NP, T, L, P, st));
  LVAE_TRY(gemm_small_f64(0, 0, T, M, T, 1.0, w.iB, T, (int64_t)P * TT, TT, w.K0xz, M, NPM, (int64_t)T * M, 0.0, w.iBK,
                          M, NPM, (int64_t)T * M, L, P, st));
  // H = K0zz + eps I + K0xz^T iB K0xz  (utils.py:147,171);  K0zz += eps I
  LVAE_TRY(gemm_small_f64(1, 0, M, M, NP, 1.0, w.K0xz, M, NPM, 0, w.iBK, M, NPM, 0, 0.0, w.Hm, M, MM, 0, L, 1, st));
  pr_eye_add_kernel<<<nblk((int64_t)L * MM), 256, 0, st>>>(L, M, eps, w.K0zz, w.Hm);
  LVAE_TRY(spd_inv_small2_f64(M, L, w.K0zz, MM, w.iK, MM, w.ldK, w.info, L, w.Hm, MM, w.iH, MM, w.ldH, w.info + L, st));
  // mu~ = iB mu - iB K0xz H^-1 K0xz^T iB mu
  LVAE_TRY(gemm_small_f64(1, 0, M, 1, NP, 1.0, w.K0xz, M, NPM, 0, w.iBmu, 1, NP, 0, 0.0, w.w, 1, M, 0, L, 1, st));
  LVAE_TRY(gemm_small_f64(0, 0, M, 1, M, 1.0, w.iH, M, MM, 0, w.w, 1, M, 0, 0.0, w.v, 1, M, 0, L, 1, st));
  LVAE_TRY(gemm_small_f64(0, 0, NP, 1, M, 1.0, w.iBK, M, NPM, 0, w.v, 1, M, 0, 0.0, w.t, 1, NP, 0, L, 1, st));
  pr_mutilde_kernel<<<nblk((int64_t)L * NP), 256, 0, st>>>(L, P, T, seg_len, include, w.iBmu, w.t, w.muT, w.muTm);
  if (Nt > 0) {
    // K0X*z K0zz^-1 K0xz^T mu~
    LVAE_TRY(gemm_small_f64(1, 0, M, 1, NP, 1.0, w.K0xz, M, NPM, 0, w.muT, 1, NP, 0, 0.0, w.a, 1, M, 0, L, 1, st));
    LVAE_TRY(gemm_small_f64(0, 0, M, 1, M, 1.0, w.iK, M, MM, 0, w.a, 1, M, 0, 0.0, w.b, 1, M, 0, L, 1, st));
    LVAE_TRY(gemm_small_f64(0, 0, Nt, 1, M, 1.0, w.K0Xz, M, (int64_t)Nt * M, 0, w.b, 1, M, 0, 0.0, w.out1, 1, Nt, 0, L,
                            1, st));
    // + k1(X*, x) mu~[test subjects], chunked over test rows (utils.py:191-209)
    for (int r0 = 0; r0 < Nt; r0 += (int)w.chunk_rows) {
      const int nr = (int)((Nt - r0) < w.chunk_rows ? (Nt - r0) : w.chunk_rows);
      const lvae_xview tc{test_x + (int64_t)r0 * Q, 0, 0, Q};
      LVAE_TRY(lvae_gram_f64(spec1, tc, xv, 1, L, nr, NP, params1, nullptr, w.K1, 0, (int64_t)nr * NP, NP, stream));
      LVAE_TRY(gemm_small_f64(0, 0, nr, 1, NP, 1.0, w.K1, NP, (int64_t)nr * NP, 0, w.muTm, 1, NP, 0, 1.0,
                              w.out1 + r0, 1, Nt, 0, L, 1, st));
    }
    pr_out_kernel<<<nblk((int64_t)L * Nt), 256, 0, st>>>(L, Nt, w.out1, out);
  }
  if (info) pr_info_kernel<<<nblk(L), 256, 0, st>>>(L, P, w.info, info);
  LVAE_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
