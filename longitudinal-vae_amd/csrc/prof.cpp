// prof.cpp -- optional hipEvent bracketing of library phases (see lvae_hip.h, "Phase timing").
#include <hip/hip_runtime.h>

#include <mutex>
#include <vector>

#include "lvae_hip.h"
#include "prof.hpp"

namespace lvae {
namespace {
struct Mark {
  int phase;
  hipEvent_t a, b;
};
bool g_on = false;
std::mutex g_mu;
std::vector<Mark> g_marks;
std::vector<hipEvent_t> g_pool;
std::vector<int> g_open;  // indices of marks begun but not ended, per phase (stack)

hipEvent_t get_event() {
  if (!g_pool.empty()) {
    hipEvent_t e = g_pool.back();
    g_pool.pop_back();
    return e;
  }
  hipEvent_t e;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}
}  // namespace

void prof_begin(int phase, hipStream_t st) {
  if (!g_on) return;
  std::lock_guard<std::mutex> lk(g_mu);
  Mark m{phase, get_event(), get_event()};
  if (!m.a || !m.b) return;
  (void)hipEventRecord(m.a, st);
  g_marks.push_back(m);
  g_open.push_back((int)g_marks.size() - 1);
}

void prof_end(int phase, hipStream_t st) {
  if (!g_on) return;
  std::lock_guard<std::mutex> lk(g_mu);
  for (int k = (int)g_open.size() - 1; k >= 0; --k) {
    const int idx = g_open[k];
    if (g_marks[idx].phase == phase) {
      (void)hipEventRecord(g_marks[idx].b, st);
      g_open.erase(g_open.begin() + k);
      return;
    }
  }
}
}  // namespace lvae

extern "C" {
int lvae_prof_enable(int on) {
  lvae::g_on = on != 0;
  return 0;
}

int lvae_prof_collect(double* ms, int32_t* count, int n_phases) {
  std::lock_guard<std::mutex> lk(lvae::g_mu);
  for (auto& m : lvae::g_marks) {
    if (hipEventSynchronize(m.b) != hipSuccess) return LVAE_ERR_LAUNCH;
    float t = 0.f;
    if (hipEventElapsedTime(&t, m.a, m.b) != hipSuccess) return LVAE_ERR_LAUNCH;
    if (m.phase < n_phases) {
      if (ms) ms[m.phase] += t;
      if (count) count[m.phase] += 1;
    }
    lvae::g_pool.push_back(m.a);
    lvae::g_pool.push_back(m.b);
  }
  lvae::g_marks.clear();
  lvae::g_open.clear();
  return 0;
}
}
