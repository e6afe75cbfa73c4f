// glue.hip -- the small elementwise pieces around the GP and ConvVAE kernels, one launch each instead of the
// chains of PyTorch ops they replace (the steps are launch-paced at a rank's share of the exact-KL step and
// in the graphed Hensman step, where every op is a ~4.5 us kernel on one queue):
//
//   vae_loss        per-image masked MSE and Gaussian NLL (VAE.py:144-162): one workgroup per image;
//                   backward: d recon and the per-pixel d log_vy partials in one pass over (pixel, image
//                   chunk) tiles
//   reparam         z = mu + eps exp(log_var / 2) (VAE.py:132-136); backward: d log_var (d mu = d z)
//   param_pack      the kernel hyper-parameters exp(m + softplus(raw - m)) (GP_model.py:31-144's
//                   positivity transform) gathered from their separate [L] tensors into the [L, P] matrix
//                   the GP kernels read; backward: d raw, scattered back per tensor
//   bias_act        the ConvVAE's bias + ReLU around its library GEMMs / transposed conv (VAE.py:44-75):
//                   forward bias + ReLU in place over [N, C, HW] (the transposed conv's output); backward
//                   g = gy [y > 0] and the bias gradient sum_{n, hw} g in one pass (per-chunk partials, then
//                   the chunks in order: fixed summation order) -- in place of PyTorch's threshold_backward
//                   and its strided reduce kernel per layer
#include "common.hpp"

namespace lvae {

constexpr float kLog2Pi = 1.8378770664093453f;  // log(2 pi)

// mse[i] = sum_j m (r - x)^2 / max(sum_j m, 1 if 0); nll[i] = sum_j m (r - x)^2 / (2 e^lv_j) + (log 2pi + lv_j) / 2
__global__ __launch_bounds__(256) void vae_loss_fwd_kernel(const float* __restrict__ r, const float* __restrict__ x,
                                                           const float* __restrict__ m, const float* __restrict__ lv,
                                                           int d, float* __restrict__ mse, float* __restrict__ nll,
                                                           float* __restrict__ msum) {
  __shared__ float red[3][4];
  const int i = blockIdx.x, tid = threadIdx.x;
  const int64_t o = (int64_t)i * d;
  float se = 0.f, ms = 0.f, nl = 0.f;
  for (int j = tid; j < d; j += 256) {
    const float df = r[o + j] - x[o + j], mk = m[o + j], l = lv[j];
    const float s = df * df * mk;
    se += s;
    ms += mk;
    nl += s / (2.f * expf(l)) + 0.5f * (kLog2Pi + l);
  }
  se = wave_sum(se);
  ms = wave_sum(ms);
  nl = wave_sum(nl);
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = se;
    red[1][tid >> 6] = ms;
    red[2][tid >> 6] = nl;
  }
  __syncthreads();
  if (tid == 0) {
    const float S = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
    float M = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
    M = M == 0.f ? 1.f : M;
    mse[i] = S / M;
    nll[i] = ((red[2][0] + red[2][1]) + red[2][2]) + red[2][3];
    msum[i] = M;
  }
}

// grid (cdiv(d, 256), cdiv(B, kLossChunk)): thread j of chunk c writes d recon[i, j] for the chunk's images
// and the partial dlv_part[c][j] = sum_i g_nll[i] (1/2 - m (r - x)^2 / (2 e^lv_j))
constexpr int kLossChunk = 64;
__global__ __launch_bounds__(256) void vae_loss_bwd_kernel(const float* __restrict__ r, const float* __restrict__ x,
                                                           const float* __restrict__ m, const float* __restrict__ lv,
                                                           const float* __restrict__ msum, const float* __restrict__ gm,
                                                           int64_t gms, const float* __restrict__ gn, int64_t gns,
                                                           int B, int d, float* __restrict__ dr,
                                                           float* __restrict__ dlv_part) {
  const int j = blockIdx.x * 256 + threadIdx.x, c = blockIdx.y;
  if (j >= d) return;
  const float ie = 1.f / (2.f * expf(lv[j]));
  const int i1 = min(B, (c + 1) * kLossChunk);
  float acc = 0.f;
  for (int i = c * kLossChunk; i < i1; ++i) {
    const int64_t o = (int64_t)i * d + j;
    const float df = r[o] - x[o], mk = m[o], g_m = gm[i * gms], g_n = gn[i * gns];
    dr[o] = 2.f * df * mk * (g_m / msum[i] + g_n * ie);
    acc += g_n * (0.5f - df * df * mk * ie);
  }
  dlv_part[(int64_t)c * d + j] = acc;
}

__global__ void reparam_fwd_kernel(const float* __restrict__ mu, const float* __restrict__ lv,
                                   const float* __restrict__ eps, int64_t n, float* __restrict__ z) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n) z[e] = mu[e] + eps[e] * expf(0.5f * lv[e]);
}

__global__ void reparam_bwd_kernel(const float* __restrict__ gz, const float* __restrict__ lv,
                                   const float* __restrict__ eps, int64_t n, float* __restrict__ glv) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n) glv[e] = 0.5f * gz[e] * eps[e] * expf(0.5f * lv[e]);
}

struct ParamPack {
  int n_raw, L, P;
  int col[64];               // column of raw k in the [L, P] matrix (other columns: 1)
  const double* raw[64];     // [L] each
  const double* mlog[64];    // [1] each: the transform's floor m (log space)
};

// softplus(t) = max(t, 0) + log1p(exp(-|t|)) (PyTorch's threshold 20 form agrees to fp64 rounding)
__device__ inline double softplus64(double t) { return t > 20.0 ? t : log1p(exp(t)); }

__global__ void param_pack_fwd_kernel(ParamPack pk, double* __restrict__ out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= pk.L * pk.P) return;
  const int l = e / pk.P, p = e % pk.P;
  double v = 1.0;
  for (int k = 0; k < pk.n_raw; ++k)
    if (pk.col[k] == p) {
      const double mm = pk.mlog[k][0];
      v = exp(mm + softplus64(pk.raw[k][l] - mm));
    }
  out[e] = v;
}

// d raw_k[l] = g[l, col_k] exp(m + softplus(t)) sigmoid(t), t = raw - m;  grad [n_raw, L]
__global__ void param_pack_bwd_kernel(ParamPack pk, const double* __restrict__ g, int64_t gs0, int64_t gs1,
                                      double* __restrict__ grad) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= pk.n_raw * pk.L) return;
  const int k = e / pk.L, l = e % pk.L;
  const double mm = pk.mlog[k][0], t = pk.raw[k][l] - mm;
  const double z = exp(t), sig = t > 20.0 ? 1.0 : z / (z + 1.0);  // (PyTorch's softplus backward)
  grad[e] = g[l * gs0 + (int64_t)pk.col[k] * gs1] * exp(mm + softplus64(t)) * sig;
}

// the Hensman step's loss terms (training.py:100-120): rec = c sum mse, nl = c sum nll (fp32, as the framework
// ops on fp32 sums), kd = ks kld (fp64), net = (use_nll ? nl + kd : rec + w kd); one workgroup
__global__ __launch_bounds__(256) void step_terms_fwd_kernel(const float* __restrict__ mse,
                                                             const float* __restrict__ nll, int B,
                                                             const double* __restrict__ kld, float c, double ks,
                                                             double w, int use_nll, float* __restrict__ rec_out,
                                                             float* __restrict__ nl_out, double* __restrict__ net_out,
                                                             double* __restrict__ kd_out) {
  __shared__ float red[2][4];
  const int tid = threadIdx.x;
  float a = 0.f, b = 0.f;
  for (int i = tid; i < B; i += 256) {
    a += mse[i];
    b += nll[i];
  }
  a = wave_sum(a);
  b = wave_sum(b);
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = a;
    red[1][tid >> 6] = b;
  }
  __syncthreads();
  if (tid == 0) {
    const float rec = (((red[0][0] + red[0][1]) + red[0][2]) + red[0][3]) * c;
    const float nl = (((red[1][0] + red[1][1]) + red[1][2]) + red[1][3]) * c;
    const double kd = kld[0] * ks;
    rec_out[0] = rec;
    nl_out[0] = nl;
    net_out[0] = use_nll ? (double)nl + kd : (double)rec + w * kd;
    kd_out[0] = kd;
  }
}

// the three gradients of the terms' inputs as scalars: d/d mse_i, d/d nll_i (fp32, the same for every
// image), d/d kld; the output gradients may be absent (nullptr: zero)
__global__ void step_terms_bwd_kernel(const double* __restrict__ g_net, const float* __restrict__ g_rec,
                                      const float* __restrict__ g_nl, const double* __restrict__ g_kd, float c,
                                      double ks, double w, int use_nll, float* __restrict__ g_mse,
                                      float* __restrict__ g_nll, double* __restrict__ g_kld) {
  if (threadIdx.x != 0) return;
  const double gn = g_net ? g_net[0] : 0.0;
  const float gr = g_rec ? g_rec[0] : 0.f, gl = g_nl ? g_nl[0] : 0.f;
  g_mse[0] = c * ((use_nll ? 0.f : (float)gn) + gr);
  g_nll[0] = c * ((use_nll ? (float)gn : 0.f) + gl);
  g_kld[0] = ks * ((use_nll ? gn : w * gn) + (g_kd ? g_kd[0] : 0.0));
}

// ---- bias_act: [N, C, HW] fp32 (HW = 1: a Linear's [B, F] rows) --------------------------------------------
// y = relu(y + b[c]) in place; NaN stays NaN (torch.relu), so a diverging layer shows in the loss
__global__ __launch_bounds__(256) void bias_relu_fwd_kernel(float* __restrict__ y, const float* __restrict__ b, int C,
                                                            int HW, int64_t total) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= total) return;
  const int c = (int)((e / HW) % C);
  const float v = y[e] + b[c];
  y[e] = v < 0.f ? 0.f : v;
}

constexpr int kActRows = 64;  // images (rows) per partial chunk
// HW == 1 (rows of a Linear): grid (cdiv(C, 64), cdiv(N, kActRows)), thread (column tx, row phase ty)
__global__ __launch_bounds__(256) void act_bwd_rows_kernel(const float* __restrict__ gy, const float* __restrict__ y,
                                                           int N, int C, int relu, float* __restrict__ g,
                                                           float* __restrict__ part) {
  __shared__ float red[4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6, c = blockIdx.x * 64 + tx, n0 = blockIdx.y * kActRows;
  float s = 0.f;
  if (c < C) {
    for (int k = ty; k < kActRows && n0 + k < N; k += 4) {
      const int64_t o = (int64_t)(n0 + k) * C + c;
      float v = gy[o];
      if (relu) v = y[o] <= 0.f ? 0.f : v;  // (torch's threshold_backward: NaN y passes the gradient)
      if (g) g[o] = v;
      s += v;
    }
  }
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && c < C) part[(int64_t)blockIdx.y * C + c] = ((red[0][tx] + red[1][tx]) + red[2][tx]) + red[3][tx];
}
// HW > 1 (NCHW): grid (C, cdiv(N, kActRows)), the workgroup sums channel c over its images' HW planes
__global__ __launch_bounds__(256) void act_bwd_chan_kernel(const float* __restrict__ gy, const float* __restrict__ y,
                                                           int N, int C, int HW, int relu, float* __restrict__ g,
                                                           float* __restrict__ part) {
  __shared__ float red[4];
  const int c = blockIdx.x, n0 = blockIdx.y * kActRows, tid = threadIdx.x;
  const int nimg = min(kActRows, N - n0);
  float s = 0.f;
  for (int im = 0; im < nimg; ++im) {  // (the image's contiguous HW plane of channel c)
    const int64_t o0 = ((int64_t)(n0 + im) * C + c) * HW;
    for (int h = tid; h < HW; h += 256) {
      float v = gy[o0 + h];
      if (relu) v = y[o0 + h] <= 0.f ? 0.f : v;
      if (g) g[o0 + h] = v;
      s += v;
    }
  }
  s = wave_sum(s);
  if ((tid & 63) == 0) red[tid >> 6] = s;
  __syncthreads();
  if (tid == 0) part[(int64_t)blockIdx.y * C + c] = ((red[0] + red[1]) + red[2]) + red[3];
}
// db[c] = the chunks' partials in order
__global__ __launch_bounds__(256) void act_bwd_sum_kernel(const float* __restrict__ part, int nchunk, int C,
                                                          float* __restrict__ db) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
#pragma unroll 16
  for (int k = 0; k < nchunk; ++k) s += part[(int64_t)k * C + c];  // (the loads issued ahead of the adds)
  db[c] = s;
}

}  // namespace lvae

using namespace lvae;

extern "C" {

int lvae_vae_loss_fwd_f32(const float* recon, const float* x, const float* mask, const float* log_vy, int B, int d,
                          float* mse, float* nll, float* msum, void* stream) {
  if (!recon || !x || !mask || !log_vy || !mse || !nll || !msum) return -1;
  if (B < 0 || d <= 0) return -2;
  if (B == 0) return 0;
  vae_loss_fwd_kernel<<<B, 256, 0, (hipStream_t)stream>>>(recon, x, mask, log_vy, d, mse, nll, msum);
  LVAE_CHECK_LAUNCH();
  return 0;
}

size_t lvae_vae_loss_bwd_partials(int B) { return (size_t)((B + kLossChunk - 1) / kLossChunk); }

int lvae_vae_loss_bwd_f32(const float* recon, const float* x, const float* mask, const float* log_vy, const float* msum,
                          const float* g_mse, int64_t g_mse_stride, const float* g_nll, int64_t g_nll_stride, int B,
                          int d, float* d_recon, float* dlv_part, void* stream) {
  if (!recon || !x || !mask || !log_vy || !msum || !g_mse || !g_nll || !d_recon || !dlv_part) return -1;
  if (B < 0 || d <= 0) return -2;
  if (B == 0) return 0;
  const dim3 grid(cdiv(d, 256), cdiv(B, kLossChunk));
  vae_loss_bwd_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(recon, x, mask, log_vy, msum, g_mse, g_mse_stride, g_nll,
                                                             g_nll_stride, B, d, d_recon, dlv_part);
  LVAE_CHECK_LAUNCH();
  return 0;
}

int lvae_reparam_fwd_f32(const float* mu, const float* log_var, const float* eps, int64_t n, float* z, void* stream) {
  if (!mu || !log_var || !eps || !z) return -1;
  if (n < 0) return -2;
  if (n == 0) return 0;
  reparam_fwd_kernel<<<cdiv(n, 256), 256, 0, (hipStream_t)stream>>>(mu, log_var, eps, n, z);
  LVAE_CHECK_LAUNCH();
  return 0;
}

int lvae_reparam_bwd_f32(const float* gz, const float* log_var, const float* eps, int64_t n, float* g_log_var,
                         void* stream) {
  if (!gz || !log_var || !eps || !g_log_var) return -1;
  if (n < 0) return -2;
  if (n == 0) return 0;
  reparam_bwd_kernel<<<cdiv(n, 256), 256, 0, (hipStream_t)stream>>>(gz, log_var, eps, n, g_log_var);
  LVAE_CHECK_LAUNCH();
  return 0;
}

static int param_pack_make(int n_raw, int L, int P, const int* cols, const double* const* raws,
                           const double* const* mlogs, ParamPack& pk) {
  if (n_raw < 0 || n_raw > 64 || L <= 0 || P <= 0 || P > 64) return -2;
  if (n_raw > 0 && (!cols || !raws || !mlogs)) return -1;
  pk.n_raw = n_raw;
  pk.L = L;
  pk.P = P;
  for (int k = 0; k < n_raw; ++k) {
    if (!raws[k] || !mlogs[k] || cols[k] < 0 || cols[k] >= P) return -3;
    pk.col[k] = cols[k];
    pk.raw[k] = raws[k];
    pk.mlog[k] = mlogs[k];
  }
  return 0;
}

int lvae_param_pack_fwd_f64(int n_raw, int L, int P, const int* cols, const double* const* raws,
                            const double* const* mlogs, double* out, void* stream) {
  if (!out) return -1;
  ParamPack pk;
  LVAE_TRY(param_pack_make(n_raw, L, P, cols, raws, mlogs, pk));
  param_pack_fwd_kernel<<<cdiv((int64_t)L * P, 256), 256, 0, (hipStream_t)stream>>>(pk, out);
  LVAE_CHECK_LAUNCH();
  return 0;
}

int lvae_param_pack_bwd_f64(int n_raw, int L, int P, const int* cols, const double* const* raws,
                            const double* const* mlogs, const double* g, int64_t g_stride0, int64_t g_stride1,
                            double* grad, void* stream) {
  if (!g || !grad) return -1;
  ParamPack pk;
  LVAE_TRY(param_pack_make(n_raw, L, P, cols, raws, mlogs, pk));
  if (n_raw == 0) return 0;
  param_pack_bwd_kernel<<<cdiv((int64_t)n_raw * L, 256), 256, 0, (hipStream_t)stream>>>(pk, g, g_stride0, g_stride1,
                                                                                        grad);
  LVAE_CHECK_LAUNCH();
  return 0;
}

int lvae_step_terms_fwd(const float* mse, const float* nll, int B, const double* kld, float c, double ks, double w,
                        int use_nll, float* rec, float* nl, double* net, double* kd, void* stream) {
  if (!mse || !nll || !kld || !rec || !nl || !net || !kd) return -1;
  if (B < 0) return -2;
  step_terms_fwd_kernel<<<1, 256, 0, (hipStream_t)stream>>>(mse, nll, B, kld, c, ks, w, use_nll, rec, nl, net, kd);
  LVAE_CHECK_LAUNCH();
  return 0;
}

int lvae_step_terms_bwd(const double* g_net, const float* g_rec, const float* g_nl, const double* g_kd, float c,
                        double ks, double w, int use_nll, float* g_mse, float* g_nll, double* g_kld, void* stream) {
  if (!g_mse || !g_nll || !g_kld) return -1;
  step_terms_bwd_kernel<<<1, 64, 0, (hipStream_t)stream>>>(g_net, g_rec, g_nl, g_kd, c, ks, w, use_nll, g_mse, g_nll,
                                                           g_kld);
  LVAE_CHECK_LAUNCH();
  return 0;
}

int lvae_bias_relu_fwd_f32(float* y, const float* bias, int N, int C, int HW, void* stream) {
  if (!y || !bias) return -1;
  if (N < 0 || C <= 0 || HW <= 0) return -2;
  const int64_t total = (int64_t)N * C * HW;
  if (total == 0) return 0;
  bias_relu_fwd_kernel<<<(unsigned)((total + 255) / 256), 256, 0, (hipStream_t)stream>>>(y, bias, C, HW, total);
  LVAE_CHECK_LAUNCH();
  return 0;
}

size_t lvae_act_bwd_workspace_size(int N, int C) {
  return (size_t)((N + kActRows - 1) / kActRows) * (size_t)(C > 0 ? C : 0) * sizeof(float);
}

int lvae_act_bwd_f32(const float* gy, const float* y, int N, int C, int HW, int relu, float* g, float* db,
                     void* workspace, void* stream) {
  if (!gy || !db || !workspace) return -1;
  if (relu && (!y || !g)) return -1;
  if (N < 0 || C <= 0 || HW <= 0) return -2;
  if (N == 0) {
    if (zero_async(db, (size_t)C * sizeof(float), (hipStream_t)stream) != 0) return LVAE_ERR_LAUNCH;
    return 0;
  }
  const int nchunk = (N + kActRows - 1) / kActRows;
  float* part = (float*)workspace;
  hipStream_t st = (hipStream_t)stream;
  if (HW == 1)
    act_bwd_rows_kernel<<<dim3((C + 63) / 64, nchunk), 256, 0, st>>>(gy, y, N, C, relu, relu ? g : nullptr, part);
  else
    act_bwd_chan_kernel<<<dim3(C, nchunk), 256, 0, st>>>(gy, y, N, C, HW, relu, relu ? g : nullptr, part);
  act_bwd_sum_kernel<<<(C + 255) / 256, 256, 0, st>>>(part, nchunk, C, db);
  LVAE_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
