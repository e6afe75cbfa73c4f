#pragma once
#include <hip/hip_runtime.h>
namespace lvae {
void prof_begin(int phase, hipStream_t st);
void prof_end(int phase, hipStream_t st);
struct ProfScope {
  int ph;
  hipStream_t st;
  ProfScope(int p, hipStream_t s) : ph(p), st(s) { prof_begin(p, s); }
  ~ProfScope() { prof_end(ph, st); }
};
}  // namespace lvae
