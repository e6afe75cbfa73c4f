// Microbenchmark of the one-workgroup SPD inverses: ALG 0 = element-wise 4-column Cholesky inverse
// (csrc/sweep.hpp), ALG 1 = 16-block LDL^T inverse with in-register pivot blocks (csrc/blkinv.hpp).
// Wall time per launch (hipEvents) for batches of SPD matrices, fp32 and fp64, and max|A Ai - I|
// on a well-conditioned (X X^T / n + I) and an ill-conditioned (RBF Gram + 1e-6 I, cond ~1e8) input.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I longitudinal-vae_amd/csrc \
//        scripts/micro/chol_inv_bench.hip -o scripts/micro/chol_inv_bench
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "blkinv.hpp"
#include "sweep.hpp"

template <typename T, int TS, int TPW, int ALG>
__global__ __launch_bounds__(64 * TS * TS / TPW) void k_inv(int n, const T* A, T* Ai, double* ld, int32_t* info) {
  const int b = blockIdx.x;
  if constexpr (ALG == 0)
    lvae::chol_inverse<T, TS, TPW>(n, A + (size_t)b * n * n, n, Ai + (size_t)b * n * n, n, ld + b, 0, info + b, 0);
  else
    lvae::blk_inverse<T, TS, TPW>(n, A + (size_t)b * n * n, n, Ai + (size_t)b * n * n, n, ld + b, 0, info + b, 0);
}

template <typename T, int TS, int TPW, int ALG>
void run(int n, int batch, const char* name, bool ill = false) {
  std::vector<T> h((size_t)batch * n * n);
  srand(1);
  for (int b = 0; b < batch; ++b) {
    // A = X X^T / n + I
    std::vector<double> X((size_t)n * n);
    for (auto& v : X) v = (rand() / (double)RAND_MAX - 0.5);
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        double s;
        if (ill) {  // RBF Gram of scattered time points, lengthscale 2.5, + 1e-6 jitter (K0zz-like)
          const double xi = fmod(i * 0.37 + b * 0.11, 16.0), xj = fmod(j * 0.37 + b * 0.11, 16.0);
          s = exp(-(xi - xj) * (xi - xj) / 12.5) + (i == j ? 1e-6 : 0.0);
        } else {
          s = (i == j) ? 1.0 : 0.0;
          for (int k = 0; k < n; ++k) s += X[(size_t)i * n + k] * X[(size_t)j * n + k] / n;
        }
        h[(size_t)b * n * n + (size_t)i * n + j] = (T)s;
      }
  }
  T *dA, *dAi;
  double* dld;
  int32_t* dinfo;
  (void)hipMalloc(&dA, h.size() * sizeof(T));
  (void)hipMalloc(&dAi, h.size() * sizeof(T));
  (void)hipMalloc(&dld, batch * sizeof(double));
  (void)hipMalloc(&dinfo, batch * sizeof(int32_t));
  (void)hipMemcpy(dA, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int nt = 64 * TS * TS / TPW;
  for (int i = 0; i < 3; ++i) k_inv<T, TS, TPW, ALG><<<batch, nt>>>(n, dA, dAi, dld, dinfo);
  (void)hipEventRecord(e0);
  const int reps = 20;
  for (int i = 0; i < reps; ++i) k_inv<T, TS, TPW, ALG><<<batch, nt>>>(n, dA, dAi, dld, dinfo);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  // check matrix 0: ||A Ai - I||_max
  std::vector<T> hi((size_t)n * n);
  (void)hipMemcpy(hi.data(), dAi, hi.size() * sizeof(T), hipMemcpyDeviceToHost);
  double err = 0, amax = 0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double s = 0;
      for (int k = 0; k < n; ++k) s += (double)h[(size_t)i * n + k] * (double)hi[(size_t)k * n + j];
      err = fmax(err, fabs(s - (i == j ? 1.0 : 0.0)));
      amax = fmax(amax, fabs((double)hi[(size_t)i * n + j]));
    }
  double hld = 0;
  int32_t hinfo = 0;
  (void)hipMemcpy(&hld, dld, sizeof(double), hipMemcpyDeviceToHost);
  (void)hipMemcpy(&hinfo, dinfo, sizeof(int32_t), hipMemcpyDeviceToHost);
  printf("%-12s %s n=%4d batch=%4d  %8.1f us/launch   max|A Ai - I| = %.2e  max|Ai| = %.2e  logdet = %.10g info = %d\n",
         name, ill ? "ill " : "well", n, batch, 1000.0 * ms / reps, err, amax, hld, hinfo);
  (void)hipFree(dA);
  (void)hipFree(dAi);
  (void)hipFree(dld);
  (void)hipFree(dinfo);
}

int main() {
  run<double, 8, 4, 0>(120, 16, "chol f64 TS8");
  run<double, 8, 4, 1>(120, 16, "blk  f64 TS8");
  run<double, 8, 4, 0>(120, 16, "chol f64 TS8", true);
  run<double, 8, 8, 1>(120, 16, "blk  f64 8w8", true);
  run<double, 8, 4, 1>(128, 32, "blk  f64 TS8");
  run<double, 8, 8, 1>(120, 16, "blk  f64 8w8");
  run<double, 4, 4, 1>(60, 16, "blk  f64 TS4");
  run<double, 4, 2, 1>(60, 16, "blk  f64 4w2");
  run<double, 2, 2, 1>(30, 16, "blk  f64 TS2");
  run<double, 1, 1, 1>(16, 80, "blk  f64 TS1");
  run<double, 1, 1, 1>(13, 80, "blk  f64 TS1");
  run<float, 8, 4, 0>(128, 16, "chol f32 TS8");
  run<float, 8, 4, 1>(128, 16, "blk  f32 TS8");
  run<float, 8, 8, 1>(128, 16, "blk  f32 8w8");
  return 0;
}
