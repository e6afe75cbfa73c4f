// Microbenchmark of the in-accumulator MFMA Cholesky inverse (csrc/sweep.hpp): wall time per launch
// (hipEvents) for batches of SPD matrices, fp32 and fp64, plus correctness vs a CPU reference.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I longitudinal-vae_amd/csrc \
//        scripts/micro/chol_inv_bench.hip -o scripts/micro/chol_inv_bench
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "sweep.hpp"

template <typename T, int TS, int TPW>
__global__ __launch_bounds__(64 * TS * TS / TPW) void k_inv(int n, const T* A, T* Ai, double* ld, int32_t* info) {
  const int b = blockIdx.x;
  lvae::chol_inverse<T, TS, TPW>(n, A + (size_t)b * n * n, n, Ai + (size_t)b * n * n, n, ld + b, 0, info + b, 0);
}

template <typename T, int TS, int TPW>
void run(int n, int batch, const char* name) {
  std::vector<T> h((size_t)batch * n * n);
  srand(1);
  for (int b = 0; b < batch; ++b) {
    // A = X X^T / n + I
    std::vector<double> X((size_t)n * n);
    for (auto& v : X) v = (rand() / (double)RAND_MAX - 0.5);
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        double s = (i == j) ? 1.0 : 0.0;
        for (int k = 0; k < n; ++k) s += X[(size_t)i * n + k] * X[(size_t)j * n + k] / n;
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
  for (int i = 0; i < 3; ++i) k_inv<T, TS, TPW><<<batch, nt>>>(n, dA, dAi, dld, dinfo);
  (void)hipEventRecord(e0);
  const int reps = 20;
  for (int i = 0; i < reps; ++i) k_inv<T, TS, TPW><<<batch, nt>>>(n, dA, dAi, dld, dinfo);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  // check matrix 0: ||A Ai - I||_max
  std::vector<T> hi((size_t)n * n);
  (void)hipMemcpy(hi.data(), dAi, hi.size() * sizeof(T), hipMemcpyDeviceToHost);
  double err = 0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double s = 0;
      for (int k = 0; k < n; ++k) s += (double)h[(size_t)i * n + k] * (double)hi[(size_t)k * n + j];
      err = fmax(err, fabs(s - (i == j ? 1.0 : 0.0)));
    }
  printf("%-10s n=%4d batch=%4d  %8.1f us/launch   max|A Ai - I| = %.2e\n", name, n, batch, 1000.0 * ms / reps, err);
  (void)hipFree(dA);
  (void)hipFree(dAi);
  (void)hipFree(dld);
  (void)hipFree(dinfo);
}

int main() {
  run<double, 8, 4>(120, 16, "f64 TS8");
  run<double, 8, 4>(128, 32, "f64 TS8");
  run<double, 4, 4>(60, 16, "f64 TS4");
  run<double, 1, 1>(16, 80, "f64 TS1");
  run<float, 8, 4>(128, 16, "f32 TS8");
  run<double, 8, 8>(120, 16, "f64 TS8w8");
  run<float, 8, 8>(128, 16, "f32 TS8w8");
  return 0;
}
