/*
 * lvae_hip.h -- C ABI of the MI355X-native Longitudinal-VAE GP-prior ELBO hot path.
 *
 * Every entry point is a plain C function over caller-owned device pointers: no allocation of
 * device memory inside, all work enqueued asynchronously on the caller's hipStream_t (passed as
 * void*), safe to call from several host threads.  Process-wide state is limited to (1) the
 * opt-in phase timer (lvae_prof_*) and (2) the blocked inverses' side stream (lvae_spd_inv_chol_f32,
 * lvae_kl_closed_*): ONE high-priority stream + seven events (fork, prep, c, and
 * two pairs alternating by pass parity) per device, shared by every caller stream, created on first
 * use, kept for the process lifetime, and guarded by a mutex held for each call's whole enqueue
 * sequence (calls from different caller streams serialise on it).  The calls are graph-capturable (the side stream joins
 * the capture through the fork event and is joined back before the call returns).  Return value: 0 = ok, <0 = -(index of the bad argument),
 * LVAE_ERR_LAUNCH on a HIP launch error.  Numerical failure (a non-positive-definite pivot) is
 * NOT a return code (the call is asynchronous): it is written to the device `info` array,
 * LAPACK-style (first failing column + 1, 0 = ok), and the Python layer raises
 * torch.linalg.LinAlgError from it like torch.linalg.cholesky does.
 *
 * Reference interfaces replaced (SidRama/Longitudinal-VAE, /root/reference):
 *   covar_module(x1, x2).evaluate()       -> lvae_gram_*            (GP_model.py:31-144,
 *                                             kernel_gen.py:9-310, call sites elbo_functions.py:22,56,171-174)
 *   autograd of that Gram wrt (scale, lengthscale) -> lvae_gram_bwd_*
 *   torch.cholesky(K1) on N x N           -> lvae_potrf_f64 / _f32 (elbo_functions.py:26)
 *   torch.cholesky_solve(B, LK1)          -> lvae_potrs_f64 / _f32, lvae_trsm_* (elbo_functions.py:27-28)
 *   torch.cholesky / cholesky_solve(I) / log-det on N x N -> lvae_spd_inv_chol_f32
 *                                             (elbo_functions.py:26-29)
 *   KL_closed forward + autograd backward -> lvae_kl_closed_fwd_f32 / _bwd_f32 (elbo_functions.py:8-34)
 *   batched small fp64 factor + inverse   -> lvae_spd_inv_small_f64 (elbo_functions.py:176-186,
 *                                             training.py:130-134)
 *   minibatch_KLD_upper_bound + autograd  -> lvae_hensman_fwd_f64 / _bwd_f64 (elbo_functions.py:144-216)
 *   natural-gradient (m, H) update        -> lvae_natgrad_update_f64 (training.py:129-135)
 */
#ifndef LVAE_HIP_H
#define LVAE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LVAE_MAX_COMP 16   /* additive components per kernel                  */
#define LVAE_MAX_FAC 4     /* product factors per component                   */
#define LVAE_ERR_LAUNCH (-1000)

/* factor kinds (GP_model.py:31-85; periodic/linear are extensions, parity unpinned) */
enum lvae_factor_kind {
  LVAE_CAT = 0,   /* 1[x1_d == x2_d]                                  GP_model.py:52-53 */
  LVAE_BIN = 1,   /* 1[x1_d + x2_d == 2]                              GP_model.py:40-41 */
  LVAE_RBF = 2,   /* exp(-(x1_d-x2_d)^2 / (2 l^2)), param l            GP_model.py:80-85 */
  LVAE_PER = 3,   /* exp(-2 sin^2(pi|x1_d-x2_d|/p) / l^2), params l, p  (extension)       */
  LVAE_LIN = 4    /* x1_d * x2_d                                      (extension)       */
};

/* An additive kernel: sum_r scale_r * prod_f factor_{r,f}.  Parameters are per latent dim
 * (row-major [L, n_params], constrained values); component r's scale is params[scale_idx[r]],
 * a factor's first parameter is params[param_idx[r][f]] (-1 when it has none). */
typedef struct lvae_kernel_spec {
  int32_t n_comp;
  int32_t n_params;
  int32_t n_fac[LVAE_MAX_COMP];
  int32_t scale_idx[LVAE_MAX_COMP];
  int32_t kind[LVAE_MAX_COMP][LVAE_MAX_FAC];
  int32_t dim[LVAE_MAX_COMP][LVAE_MAX_FAC];
  int32_t param_idx[LVAE_MAX_COMP][LVAE_MAX_FAC];
} lvae_kernel_spec;

/* Strided operand of a batched Gram: element (b, l, i, q) at
 *   ptr[b*stride_b + l*stride_l + i*ld + q]     (stride 0 = broadcast)                       */
typedef struct lvae_xview {
  const double* ptr;
  int64_t stride_b;
  int64_t stride_l;
  int64_t ld;
} lvae_xview;

/* ---------------------------------------------------------------------------------------- */
/* Gram                                                                                      */
/* ---------------------------------------------------------------------------------------- */

/* out[b, l, i, j] = sum_r s_r prod_f phi(x1[b,l,i], x2[b,l,j]) + (i == j ? diag[l] : 0)
 * for b < nb, l < L, i < n1, j < n2.  out element (b,l,i,j) at
 * out[b*ostride_b + l*ostride_l + i*ldo + j].  diag may be NULL.  params: [L, n_params] fp64.
 * Replaces covar_module(x1, x2).evaluate() (+ noise * I) in elbo_functions.py:22-23,171-174. */
int lvae_gram_f64(const lvae_kernel_spec* spec, lvae_xview x1, lvae_xview x2, int nb, int L, int n1,
                  int n2, const double* params, const double* diag, double* out, int64_t ostride_b,
                  int64_t ostride_l, int64_t ldo, void* stream);
int lvae_gram_f32(const lvae_kernel_spec* spec, lvae_xview x1, lvae_xview x2, int nb, int L, int n1,
                  int n2, const double* params, const double* diag, float* out, int64_t ostride_b,
                  int64_t ostride_l, int64_t ldo, void* stream);

/* Adjoint of lvae_gram_*: dparams[l, p] (+)= sum_{b,i,j} G[b,l,i,j] * d out[b,l,i,j] / d params[l,p]
 * (diag term excluded; d/d diag is returned separately in ddiag[l] = sum_{b,i} G[b,l,i,i] when
 * ddiag != NULL).  G strided like out.  Results are ADDED to dparams / ddiag (fp64), in a fixed
 * order (deterministic).  workspace: lvae_gram_bwd_workspace_size(nb, L, n1, n2) bytes.        */
size_t lvae_gram_bwd_workspace_size(int nb, int L, int n1, int n2);
int lvae_gram_bwd_f64(const lvae_kernel_spec* spec, lvae_xview x1, lvae_xview x2, int nb, int L, int n1,
                      int n2, const double* params, const double* G, int64_t gstride_b,
                      int64_t gstride_l, int64_t ldg, double* dparams, double* ddiag, void* workspace,
                      void* stream);

/* ---------------------------------------------------------------------------------------- */
/* Regime B: exact KL over the full N x N covariance (elbo_functions.py:8-34), batched over L */
/* latent dims.  Arithmetic: fp32 storage; every GEMM on the f16 matrix cores with the       */
/* 3-product hi / lo split (fp32-equivalent, ~2^-22 of max|operand| per product; power-of-two */
/* split scales per 256 x 256 block from each block's exact max, so any K scale / noise level */
/* that fp32 itself can represent is safe); K^-1 mu refined once in fp64.  Covariance padded  */
/* to Np = lvae_kl_closed_padded_n(n) (identity on the padding).                              */
/* ---------------------------------------------------------------------------------------- */
int lvae_kl_closed_padded_n(int n);
/* bytes of device workspace the fwd+bwd pair needs (kept between the two calls) */
size_t lvae_kl_closed_workspace_size(int n, int L);

/* kl[l] = 1/2 (tr(K^-1 V) + mu^T K^-1 mu - n + log|K| - sum log v),  K = Gram_l(x, x) + noise_l I.
 * x: [n, ldx] fp64 covariates; mu, logv: element (i, l) at mu[i*ld_mu + l] (fp64);
 * params [L, n_params] fp64; noise [L] fp64; kl [L] fp64; info [L] int32.
 * workspace: lvae_kl_closed_workspace_size(n, L) bytes, 256-B aligned.
 * need_bwd != 0 also writes the backward's S-GEMM operand (fp16 planes of K^-1 diag(sqrt v),
 * one power-of-two scale per dim) into the workspace; the backward requires a need_bwd forward. */
int lvae_kl_closed_fwd_f32(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int L,
                           const double* params, const double* noise, const double* mu, const double* logv,
                           int ld_mu, double* kl, int32_t* info, void* workspace, int need_bwd,
                           void* stream);
/* The same forward in two calls, for callers that overlap the factorisation with the work that
 * produces (mu, logv) (the encoder): _factor_f32 needs only the covariates and hyperparameters
 * (Gram + the blocked Cholesky inverse: K^-1, log|K|, info into the workspace); _reduce_f32 then
 * takes mu / logv (alpha = K^-1 mu with one fp64 refinement step -- the residual mu - K alpha0 is
 * evaluated from the covariates in fp64, hence spec / x / params / noise again, the same as the
 * factor's -- the trace and quadratic terms, kl, and with need_bwd the S-GEMM operand).  factor then
 * reduce on one stream (or with the reduce stream waiting on the factor's) equals
 * lvae_kl_closed_fwd_f32.  One reduce per factor: the reduce (diag K^-1 refinement) and the backward
 * reuse the factor's triangular-inverse planes in the workspace.                                 */
int lvae_kl_closed_factor_f32(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int L,
                              const double* params, const double* noise, int32_t* info, void* workspace,
                              void* stream);
int lvae_kl_closed_reduce_f32(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int L,
                              const double* params, const double* noise, const double* mu, const double* logv,
                              int ld_mu, double* kl, void* workspace, int need_bwd, void* stream);

/* Backward of lvae_kl_closed_fwd_f32 given dL/dkl[l] = gkl[l]:
 *   dmu[i,l] = gkl_l (K^-1 mu)_i,  dlogv[i,l] = gkl_l/2 (v_i (K^-1)_ii - 1),
 *   dparams[l,:] = gkl_l sum_ij G_ij dK_ij/dparams,  dnoise[l] = gkl_l tr(G),
 *   G = 1/2 (K^-1 - K^-1 V K^-1 - K^-1 mu mu^T K^-1).
 * Outputs are OVERWRITTEN.  Workspace must be the one the forward filled.                   */
int lvae_kl_closed_bwd_f32(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int L,
                           const double* params, const double* mu, const double* logv, int ld_mu,
                           const double* gkl, double* dmu, double* dlogv, double* dparams, double* dnoise,
                           void* workspace, void* stream);
/* The same backward in its two independent halves (lvae_kl_closed_bwd_f32 = _latent then _hyper), for
 * callers that start the encoder's backward on d/d(mu, logv) while the hyper-parameter half (the
 * S = K^-1 V K^-1 GEMM and the Gram adjoint: ~all of the backward's time) still runs. Either order. */
int lvae_kl_closed_bwd_latent_f32(int n, int L, const double* logv, int ld_mu, const double* gkl, double* dmu,
                                  double* dlogv, void* workspace, void* stream);
int lvae_kl_closed_bwd_hyper_f32(const lvae_kernel_spec* spec, const double* x, int ldx, int n, int L,
                                 const double* params, const double* gkl, double* dparams, double* dnoise,
                                 void* workspace, void* stream);

/* diag(K^-1) in fp64 for ill-conditioned dims (kl_refine.hip): the reduce estimates each dim's
 * diagonal error by est_l = (sum_r s_r + noise_l) max_i (K^-1)_ii (the first factor bounds max_i K_ii) and where est_l > tau (env LVAE_KL_REFINE_TAU,
 * default 16; LVAE_KL_REFINE=0 never, =1 always) replaces diag K^-1 by one fp64 Newton step,
 * 2 X_jj - (X K X)_jj (the trace term and dlogv; the reference's cholesky_solve(I) is fp64,
 * elbo_functions.py:27-31).  This copies the last reduce's est [L] (fp64) and flag [L] (int32, 1:
 * refined) to device buffers, on `stream`.  No reference counterpart (diagnostic).                  */
int lvae_kl_closed_refine_state(int n, int L, const void* workspace, double* est, int32_t* flag, void* stream);

/* The backward's hyper-parameter half takes one of two routes, decided on the device from the covariates by the
 * factor (kl_hyper.hip): the S = K^-1 V K^-1 GEMM + the Gram adjoint, or -- for the table family of kernels on
 * integer-coded covariates with the "big" (id) covariate in contiguous runs -- the binned route (bin sums of
 * K^-1 and the id runs' blocks, no S; env LVAE_KL_HYPER=0 forces the GEMM route).  This copies the last
 * factor's choice (int32: 1 = binned) to a device buffer, on `stream`.  No reference counterpart (diagnostic). */
int lvae_kl_closed_hyper_state(int n, int L, const void* workspace, int32_t* on, void* stream);

/* A^-1 and log|A| of L padded SPD matrices by a blocked Cholesky factorisation, triangular inverse
 * and product (LAPACK potrf + trtri + lauum, 256-wide blocks; the inverse lvae_kl_closed_* use):
 * potrf's pivot blocks factored and inverted in LDS (fp32 MFMA), its panel / rank-256 trailing
 * updates and trtri / lauum's whole-block GEMMs on the f16 cores with the 3-product split; the next
 * pivot runs on a side stream beside each trailing update.  np % 256 == 0; A [L, np, np] (lower
 * 256-block tiles read, overwritten); Ainv [L, np, np] full symmetric out; logdet [L]; info [L]
 * LAPACK-style (first bad column + 1); scratch: lvae_spd_inv_chol_scratch_size(np, L) bytes, 256-B
 * aligned.  Backward-stable in the Cholesky sense: |I - A Ainv| ~ cond(A) 2^-24 (the rounds 1-2 block
 * Gauss-Jordan sweep, ~100x less accurate at cond 1e5, is retired: csrc/retired/spd_sweep.hip, not built).
 * Replaces torch.cholesky + cholesky_solve(I) + the log-det (elbo_functions.py:26-29).         */
size_t lvae_spd_inv_chol_scratch_size(int np_, int L);
int lvae_spd_inv_chol_f32(int np_, int L, float* A, void* scratch, float* Ainv, double* logdet, int32_t* info,
                          void* stream);

/* ---------------------------------------------------------------------------------------- */
/* N x N factor / solve (potrf.hip): the reference's own LAPACK calls on K1,                   */
/*   LK1 = torch.cholesky(K1);  torch.cholesky_solve(B, LK1);  logdet = 2 sum log diag(LK1)    */
/* (elbo_functions.py:26-29), batched over L matrices: element (l, i, j) of a matrix argument   */
/* at ptr[l*stride + i*ld + j].  Factors are lower triangular with a zero strict upper part    */
/* (torch.cholesky's output); only the lower triangle of A is read.  info[l] LAPACK-style.     */
/* ---------------------------------------------------------------------------------------- */
/* Lout <- chol(A) in fp64, log|A| into logdet[l]: 64-wide blocked right-looking potrf, the panel
 * by substitution (as LAPACK's trsm), the trailing update on the fp64 matrix cores.  Lout may be
 * A itself (in place; then ldo == lda and stride_o == stride_a).  No workspace.              */
int lvae_potrf_f64(int n, int L, const double* A, int64_t lda, int64_t stride_a, double* Lout, int64_t ldo,
                   int64_t stride_o, double* logdet, int32_t* info, void* stream);
/* The same in fp32 through the exact KL's own factorisation (chol_inv.hip: 256-wide blocks, the
 * pivot blocks on fp32 MFMA in LDS, panels and trailing updates on the f16 cores with the 3-product
 * split, ~2^-22 of each 256-block's max per product).  A is copied into the workspace (padded to a
 * multiple of 256 with the identity), so Lout may alias A.  workspace:
 * lvae_potrf_f32_workspace_size(n, L) bytes, 256-B aligned.  n <= 16384.                       */
size_t lvae_potrf_f32_workspace_size(int n, int L);
int lvae_potrf_f32(int n, int L, const float* A, int64_t lda, int64_t stride_a, float* Lout, int64_t ldo,
                   int64_t stride_o, double* logdet, int32_t* info, void* workspace, void* stream);
/* B [n, nrhs] <- op(Lf)^-1 B in place, op = Lf (trans = 0) or Lf^T (trans = 1), Lf lower
 * triangular (e.g. lvae_potrf_*'s output).  Blocked over 64 rows: the 64 x 64 diagonal blocks are
 * inverted first into the workspace (lvae_trsm_workspace_size(n, L) bytes, 256-B aligned), then one
 * workgroup per 64 columns of B sweeps the block rows in dependency order on the fp64 matrix cores.
 * The f32 variant reads / writes fp32 and computes in fp64.                                      */
size_t lvae_trsm_workspace_size(int n, int L);
int lvae_trsm_f64(int trans, int n, int nrhs, int L, const double* Lf, int64_t ldl, int64_t stride_l, double* B,
                  int64_t ldb, int64_t stride_b, void* workspace, void* stream);
int lvae_trsm_f32(int trans, int n, int nrhs, int L, const float* Lf, int64_t ldl, int64_t stride_l, float* B,
                  int64_t ldb, int64_t stride_b, void* workspace, void* stream);
/* B <- A^-1 B given Lf = chol(A): torch.cholesky_solve(B, Lf) (elbo_functions.py:27-28; also
 * cholesky_solve(eye, LK1) = K1^-1).  Workspace as lvae_trsm_*.                                */
int lvae_potrs_f64(int n, int nrhs, int L, const double* Lf, int64_t ldl, int64_t stride_l, double* B, int64_t ldb,
                   int64_t stride_b, void* workspace, void* stream);
int lvae_potrs_f32(int n, int nrhs, int L, const float* Lf, int64_t ldl, int64_t stride_l, float* B, int64_t ldb,
                   int64_t stride_b, void* workspace, void* stream);

/* ---------------------------------------------------------------------------------------- */
/* Regime A: Hensman SVI, fp64 (elbo_functions.py:144-216; training.py:129-135)             */
/* ---------------------------------------------------------------------------------------- */

/* Batched SPD factor + inverse of small matrices (n <= 128), one workgroup per matrix:
 * Ainv[b] = A[b]^-1, logdet[b] = log|A[b]|, info[b].  A, Ainv element (b,i,j) at [b*stride + i*n + j]. */
int lvae_spd_inv_small_f64(int n, int batch, const double* A, int64_t stride, double* Ainv,
                           int64_t stride_out, double* logdet, int32_t* info, void* stream);

/* Batched small fp64 GEMM: C[b] = alpha op(A[b]) op(B[b]) + beta C[b],
 * with b = (b1, b2), b1 < nb1, b2 < nb2, offsets b1*s?1 + b2*s?2.  op = transpose when t? != 0. */
int lvae_gemm_small_f64(int ta, int tb, int m, int n, int k, double alpha, const double* A, int lda,
                        int64_t sa1, int64_t sa2, const double* B, int ldb, int64_t sb1, int64_t sb2,
                        double beta, double* C, int ldc, int64_t sc1, int64_t sc2, int nb1, int nb2,
                        void* stream);

/* Hensman bound sizes: L latent dims, M inducing points, P_b subjects x T time points, Q covariates */
typedef struct lvae_hensman_dims {
  int32_t L, M, P_b, T, Q;
  double P_tot;            /* subjects in the data set (scale P_tot / P_b)                     */
  double eps;              /* jitter on K0zz                                                   */
  int32_t natural_gradient;
  double ng_prior_share;   /* weight of the data-independent part (iK m, iK, iH) in grad_m /   */
                           /* grad_H: 1 for one process; 1/world under data parallelism, so a  */
                           /* SUM all-reduce of the per-rank directions equals the union batch */
  const int32_t* seg_len;  /* varying T (minibatch_KLD_upper_bound_iter, elbo_functions.py:219-307): */
                           /* device [P_b] valid rows per subject, rows T_p..T-1 of subject p are  */
                           /* padding (masked out of every term); NULL = all T rows valid          */
  double n_total;          /* N of the constant -L N / 2; 0 -> P_tot * T                          */
} lvae_hensman_dims;

size_t lvae_hensman_workspace_size(const lvae_hensman_dims* d);
/* Byte offset inside the Hensman workspace of H^-1 [L, M, M] as left by lvae_hensman_fwd_f64
 * (valid until the workspace is reused; lets the natural-gradient update skip re-inverting H). */
size_t lvae_hensman_iH_offset(const lvae_hensman_dims* d);

/* Forward of minibatch_KLD_upper_bound: kld (scalar, sum over L), grad_m [L,M], grad_H [L,M,M]
 * (natural_gradient only; may be NULL otherwise).  x [P_b*T, Q], z [L, M, Q], m [L, M], H [L, M, M],
 * mu / logv [P_b*T, L] (fp64, row-major), params0 [L, P0], params1 [L, P1], noise [L].          */
int lvae_hensman_fwd_f64(const lvae_kernel_spec* spec0, const lvae_kernel_spec* spec1,
                         const lvae_hensman_dims* d, const double* x, const double* z, const double* m,
                         const double* H, const double* mu, const double* logv, const double* params0,
                         const double* params1, const double* noise, double* kld, double* grad_m,
                         double* grad_H, int32_t* info, void* workspace, void* stream);
/* The same forward in two parts on one workspace (part 0: both): part 1 needs neither mu nor logv
 * (Grams, the K0zz / B_p / H inverses, iK m, K0xz iK m, Q = K0xz^T B^-1 K0xz, iK H iK and the
 * data-independent natural-gradient terms incl. grad_H) and can run beside the encoder; part 2 (the
 * residual, the sums -> kld, grad_m, info) then reads mu / logv.  Same results as the one call.    */
int lvae_hensman_fwd_part_f64(int part, const lvae_kernel_spec* spec0, const lvae_kernel_spec* spec1,
                              const lvae_hensman_dims* d, const double* x, const double* z, const double* m,
                              const double* H, const double* mu, const double* logv, const double* params0,
                              const double* params1, const double* noise, double* kld, double* grad_m,
                              double* grad_H, int32_t* info, void* workspace, void* stream);

/* Backward given dL/dkld = *gkld (device scalar): dmu, dlogv [P_b*T, L]; dparams0 [L,P0],
 * dparams1 [L,P1], dnoise [L]; dm [L,M], dH [L,M,M] when !natural_gradient (else may be NULL).
 * Outputs are OVERWRITTEN.                                                                   */
int lvae_hensman_bwd_f64(const lvae_kernel_spec* spec0, const lvae_kernel_spec* spec1,
                         const lvae_hensman_dims* d, const double* x, const double* z, const double* m,
                         const double* H, const double* mu, const double* logv, const double* params0,
                         const double* params1, const double* noise, const double* gkld, double* dmu,
                         double* dlogv, double* dparams0, double* dparams1, double* dnoise, double* dm,
                         double* dH, void* workspace, void* stream);

/* Natural-gradient update of the inducing posterior (training.py:129-135), in place:
 *   iH' = H^-1 + lr (gH + gH^T);  H <- iH'^-1;  m <- H (H^-1 m - lr (gm - 2 gH m)).
 * iH: H^-1 if the caller already has it (e.g. workspace + lvae_hensman_iH_offset after the
 * forward on the same H), else NULL (H is inverted here, as training.py:130-131 does).
 * info[l] (may be NULL): the first failed factorisation of dim l (H's, then iH''s), LAPACK-style;
 * if any dim's factorisation fails, NO dim's (m, H) is changed (the reference's batched
 * torch.cholesky raises before assigning, training.py:130-134).
 * workspace: lvae_natgrad_workspace_size(L, M) bytes.                                        */
size_t lvae_natgrad_workspace_size(int L, int M);
int lvae_natgrad_update_f64(int L, int M, double* m, double* H, const double* grad_m,
                            const double* grad_H, double lr, const double* iH, int32_t* info,
                            void* workspace, void* stream);

/* ConvVAE encoder (VAE.py:44-50): y = max_pool2d(relu(x), 2, 2) over planes = N*C planes of H x W
 * (H, W even) fp32, idx = argmax byte (0..3, row-major in the window, first strict maximum);
 * backward gx = the pooled gradient routed to the argmax where y > 0, 0 elsewhere.            */
int lvae_relu_maxpool2_fwd_f32(const float* x, int64_t planes, int H, int W, float* y, uint8_t* idx,
                               void* stream);
int lvae_relu_maxpool2_bwd_f32(const float* gy, const float* y, const uint8_t* idx, int64_t planes, int H,
                               int W, float* gx, void* stream);
/* The same with the conv's per-channel bias folded in (the conv then runs without one): x is the
 * bias-free conv output [N, C, H, W], y = max_pool2d(relu(x + bias)); the backward also writes
 * db [C] = the conv's bias gradient (deterministic; workspace: lvae_relu_maxpool2_bias_workspace_size
 * bytes).  Replaces nn.Conv2d's bias add and its bias-gradient sum (VAE.py:44-50).             */
size_t lvae_relu_maxpool2_bias_workspace_size(int N, int C);
int lvae_relu_maxpool2_bias_fwd_f32(const float* x, const float* bias, int N, int C, int H, int W, float* y,
                                    uint8_t* idx, void* stream);
int lvae_relu_maxpool2_bias_bwd_f32(const float* gy, const float* y, const uint8_t* idx, int N, int C, int H, int W,
                                    float* gx, float* db, void* workspace, void* stream);
/* The first encoder conv end to end (VAE.py:44-47): x [N, 1, H, W], w [C, 1, 3, 3], bias [C],
 * padding 1 -> y = max_pool2d(relu(conv(x) + bias), 2, 2), idx as above; the full-resolution conv
 * output is never written.                                                                      */
int lvae_conv1_relu_maxpool2_fwd_f32(const float* x, const float* w, const float* bias, int N, int C, int H, int W,
                                     float* y, uint8_t* idx, void* stream);
/* The second encoder conv end to end (VAE.py:48-50): x [N, Cin, H, W], w [C, Cin, 3, 3], bias [C], padding 1 ->
 * y = max_pool2d(relu(conv(x) + bias), 2, 2) and idx as above, in one pass (no full-resolution output, no
 * layout transposes).  Cin == 16, H == W == 18 (the 36 x 36 images after the first pool), C % 16 == 0; -3 for
 * other shapes (conv + lvae_relu_maxpool2_bias_fwd_f32 cover them).                             */
int lvae_conv3x3_relu_maxpool2_fwd_f32(const float* x, const float* w, const float* bias, int N, int Cin, int C, int H,
                                       int W, float* y, uint8_t* idx, void* stream);
/* Weight and bias gradients of a 3x3 / stride-1 / padding-1 conv followed by the fused relu + pool
 * (the encoder convs), from the pooled gradient: dw [C, Cin, 3, 3] and db [C] as sums over the
 * pooled outputs of g * (the 3x3 input patch at the window's argmax) -- the full-resolution
 * gradient is needed only for the input gradient (the first conv's input, the image, needs none).
 * x: the conv input [N, Cin, H, W]; y, idx: the layer's forward outputs.  C * Cin <= 1024 and
 * Cin (H+2)(W+2) + 2 C (H/2)(W/2) floats within 64 KB of LDS (-3 / -4 otherwise).  Deterministic
 * (workspace: lvae_conv3x3_pool_wgrad_workspace_size bytes).                                   */
size_t lvae_conv3x3_pool_wgrad_workspace_size(int N, int C, int Cin);
int lvae_conv3x3_pool_wgrad_f32(const float* gy, const float* y, const uint8_t* idx, const float* x, int N, int C,
                                int Cin, int H, int W, float* dw, float* db, void* workspace, void* stream);
/* The input gradient of the same layer (the second encoder conv, VAE.py:48-50; torch's conv2d backward-data
 * in the reference's autograd): gx [N, Cin, H, W] = the conv's backward-data of the routed gradient (gy at
 * each window's argmax where y > 0), formed per image in LDS, never in HBM.  w [C, Cin, 3, 3].  Cin == 16
 * (-3 otherwise), H W <= 1024 and lvae_conv3x3_pool_dgrad_lds(C, H, W) <= 64 KB (-4 otherwise).      */
size_t lvae_conv3x3_pool_dgrad_lds(int C, int H, int W);
int lvae_conv3x3_pool_dgrad_f32(const float* gy, const float* y, const uint8_t* idx, const float* w, int N, int C,
                                int Cin, int H, int W, float* gx, void* stream);
/* ConvVAE decoder output (VAE.py:75, 124): out = sigmoid(ConvTranspose2d(Cin, 1, 4, stride 2, padding 1)
 * (z) + bias), z [N, Cin, Hi, Wi] (Cin <= 16), w [Cin, 1, 4, 4], bias [1] -> out [N, 1, 2Hi, 2Wi].
 * Backward from g = dLoss/dout and the saved out: gz [N, Cin, Hi, Wi], dw [Cin, 1, 4, 4], db [1]
 * (deterministic; workspace: lvae_deconv2_sigmoid_workspace_size bytes).                        */
size_t lvae_deconv2_sigmoid_workspace_size(int N, int Cin, int Hi, int Wi);
int lvae_deconv2_sigmoid_fwd_f32(const float* z, const float* w, const float* bias, int N, int Cin, int Hi, int Wi,
                                 float* out, void* stream);
int lvae_deconv2_sigmoid_bwd_f32(const float* g, const float* out, const float* z, const float* w, int N, int Cin,
                                 int Hi, int Wi, float* gz, float* dw, float* db, void* workspace, void* stream);
/* ConvVAE decoder's first transposed conv (VAE.py:73, 122): y = relu(ConvTranspose2d(Cin, Cout, 4, stride 2,
 * padding 1)(x) + bias), x [N, Cin, Hi, Wi], w [Cin, Cout, 4, 4], bias [Cout] -> y [N, Cout, 2Hi, 2Wi] (relu:
 * v < 0 -> 0, NaN kept).  Backward from gy = dLoss/dy and the saved y (mask y > 0): dx [N, Cin, Hi, Wi],
 * dw [Cin, Cout, 4, 4], db [Cout] in one pass + a fixed-order partial sum (deterministic; workspace:
 * lvae_deconv4s2_relu_bwd_workspace_size bytes).  Cin == 32, Cout == 16, Hi == Wi == 9; -3 otherwise.       */
int lvae_deconv4s2_relu_fwd_f32(const float* x, const float* w, const float* bias, int N, int Cin, int Cout, int Hi,
                                int Wi, float* y, void* stream);
size_t lvae_deconv4s2_relu_bwd_workspace_size(int N, int Cin, int Cout);
int lvae_deconv4s2_relu_bwd_f32(const float* gy, const float* y, const float* x, const float* w, int N, int Cin,
                                int Cout, int Hi, int Wi, float* dx, float* dw, float* db, void* workspace,
                                void* stream);

/* GP posterior mean of the latents at test covariates (utils.py:115-211 batch_predict_varying_T,
 * called by MSE_test_GPapprox, model_test.py:85-143).  Prediction set laid out [P, T] by subject
 * (seg_len [P] valid rows each; padding rows of x are any finite covariates, of mu must be 0),
 * x [P*T, Q], mu [P*T, L]; include [P] = 1 for subjects that also appear in test_x (the k1 term);
 * z [L, M, Q]; test_x [Nt, Q]; out [Nt, L].  info[l]: 10000/20000/30000 + col for a failed
 * K0zz / B_p / H factorisation.  workspace: lvae_predict_workspace_size(L, M, P, T, Nt) bytes. */
size_t lvae_predict_workspace_size(int L, int M, int P, int T, int Nt);
int lvae_predict_f64(const lvae_kernel_spec* spec0, const lvae_kernel_spec* spec1, int L, int M, int Q, int P,
                     int T, const int32_t* seg_len, const int32_t* include, const double* x,
                     const double* mu, const double* z, int Nt, const double* test_x,
                     const double* params0, const double* params1, const double* noise, double eps,
                     double* out, int32_t* info, void* workspace, void* stream);

/* ---------------------------------------------------------------------------------------- */
/* Phase timing (profiling aid; the only process-wide state of the library).  When enabled, */
/* the composite entry points bracket their phases with hipEvents on the caller's stream;  */
/* lvae_prof_collect synchronises on them, ADDS each phase's elapsed ms into ms[phase],    */
/* the number of bracketed intervals into count[phase], and forgets them.                  */
/* ---------------------------------------------------------------------------------------- */
enum lvae_phase {
  LVAE_PH_GRAM = 0, LVAE_PH_POTRF = 1 /* potrf (or the whole sweep) */, LVAE_PH_POTRI = 2 /* trtri + lauum */, LVAE_PH_KL_REDUCE = 3, LVAE_PH_SYRK = 4,
  LVAE_PH_GRAM_BWD = 5, LVAE_PH_BWD_ELEM = 6, LVAE_PH_HENSMAN_FWD = 7, LVAE_PH_HENSMAN_BWD = 8,
  LVAE_PH_NATGRAD = 9, LVAE_PH_SWEEP_UPD = 10 /* the trailing rank-256 update launches (U2), nested in POTRF */,
  LVAE_PH_HB_SLAB = 11 /* the binned hyper-gradient route's slab pass (kl_hyper.hip), nested in GRAM_BWD */, LVAE_N_PHASES = 12
};
int lvae_prof_enable(int on);
int lvae_prof_collect(double* ms, int32_t* count, int n_phases);

/* library identification: "lvae_hip <version> gfx950" */
const char* lvae_version(void);

/* ---------------------------------------------------------------------------------------- */
/* Glue (glue.hip): the elementwise pieces around the GP and ConvVAE kernels, one launch each    */
/* instead of a chain of framework ops (the steps are launch-paced at small shares).            */
/* ---------------------------------------------------------------------------------------- */
/* ConvVAE.loss_function (VAE.py:144-162) on [B, d] fp32 recon / x / mask, log_vy [d]:
 *   mse[i] = sum_j m (r - x)^2 / (sum_j m, or 1 where that is 0),
 *   nll[i] = sum_j (m (r - x)^2 / (2 exp(log_vy_j)) + (log 2 pi + log_vy_j) / 2);  msum[i] saved for the
 * backward.  The backward takes d mse / d nll (element i at g[i * stride]; stride 0 broadcasts) and writes
 * d recon [B, d] and per-pixel partials of d log_vy, dlv_part [lvae_vae_loss_bwd_partials(B), d] (their
 * column sums are d log_vy).                                                                     */
int lvae_vae_loss_fwd_f32(const float* recon, const float* x, const float* mask, const float* log_vy, int B, int d,
                          float* mse, float* nll, float* msum, void* stream);
size_t lvae_vae_loss_bwd_partials(int B);
int lvae_vae_loss_bwd_f32(const float* recon, const float* x, const float* mask, const float* log_vy, const float* msum,
                          const float* g_mse, int64_t g_mse_stride, const float* g_nll, int64_t g_nll_stride, int B,
                          int d, float* d_recon, float* dlv_part, void* stream);
/* ConvVAE.sample_latent (VAE.py:132-136): z = mu + eps exp(log_var / 2), n fp32 elements; backward
 * d log_var = d z eps exp(log_var / 2) / 2 (d mu = d z).                                         */
int lvae_reparam_fwd_f32(const float* mu, const float* log_var, const float* eps, int64_t n, float* z, void* stream);
int lvae_reparam_bwd_f32(const float* gz, const float* log_var, const float* eps, int64_t n, float* g_log_var,
                         void* stream);
/* The kernels' positivity transform exp(m + softplus(raw - m)) (GP_model.py:31-144) of n_raw [L] fp64
 * parameter tensors into column cols[k] of the [L, P] fp64 matrix out (other columns 1; raws[k], mlogs[k]:
 * host arrays of device pointers, mlogs[k] -> the [1] floor m).  Backward: grad [n_raw, L] =
 * g[l, cols[k]] exp(m + softplus(t)) sigmoid(t), t = raw - m (g element (l, p) at g[l s0 + p s1]).       */
int lvae_param_pack_fwd_f64(int n_raw, int L, int P, const int* cols, const double* const* raws,
                            const double* const* mlogs, double* out, void* stream);
/* The Hensman step's loss terms (training.py:100-120) from the per-image mse / nll [B] (fp32) and the KL
 * bound kld [1] (fp64): rec = c sum mse, nl = c sum nll (fp32), kd = ks kld, net = nl + kd (use_nll) or
 * rec + w kd (fp64).  Backward: d/d mse_i, d/d nll_i (the same for every image, fp32) and d/d kld from the
 * gradients of net / rec / nl / kd (nullptr: zero).                                                   */
/* The ConvVAE's bias + ReLU around its library GEMMs and transposed conv (VAE.py:44-75) on [N, C, HW] fp32
 * (HW = 1: a Linear's [B, F] rows).  Forward: y = relu(y + bias[c]) in place.  Backward: g = gy [y > 0]
 * (relu != 0; y the forward's output; with relu = 0 g is not written: g = gy) and db[c] = sum over n, hw
 * of g (per 64-image chunk partials in workspace [lvae_act_bwd_workspace_size(N, C) bytes], then the
 * chunks in order).  Replaces PyTorch's threshold_backward + the bias reduction of nn.Linear /
 * nn.ConvTranspose2d's backward (VAE.py:62-75).                                                     */
int lvae_bias_relu_fwd_f32(float* y, const float* bias, int N, int C, int HW, void* stream);
size_t lvae_act_bwd_workspace_size(int N, int C);
int lvae_act_bwd_f32(const float* gy, const float* y, int N, int C, int HW, int relu, float* g, float* db,
                     void* workspace, void* stream);
int lvae_step_terms_fwd(const float* mse, const float* nll, int B, const double* kld, float c, double ks, double w,
                        int use_nll, float* rec, float* nl, double* net, double* kd, void* stream);
int lvae_step_terms_bwd(const double* g_net, const float* g_rec, const float* g_nl, const double* g_kd, float c,
                        double ks, double w, int use_nll, float* g_mse, float* g_nll, double* g_kld, void* stream);
int lvae_param_pack_bwd_f64(int n_raw, int L, int P, const int* cols, const double* const* raws,
                            const double* const* mlogs, const double* g, int64_t g_stride0, int64_t g_stride1,
                            double* grad, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* LVAE_HIP_H */
