// side_stream.cpp -- see side_stream.hpp.
#include "side_stream.hpp"

#include "lvae_hip.h"

namespace lvae {

namespace {
constexpr int kMaxDev = 64;
SideStream g_side[kMaxDev];
}  // namespace

std::recursive_mutex& side_mutex() {
  static std::recursive_mutex mu;
  return mu;
}

int side_stream(SideStream*& out) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return LVAE_ERR_LAUNCH;
  SideStream& sd = g_side[dev];
  if (!sd.s) {
    int least = 0, greatest = 0;
    (void)hipDeviceGetStreamPriorityRange(&least, &greatest);
    if (hipStreamCreateWithPriority(&sd.s, hipStreamNonBlocking, greatest) != hipSuccess) return LVAE_ERR_LAUNCH;
    for (hipEvent_t* e : {&sd.fork, &sd.prep, &sd.c, &sd.u2p[0], &sd.u2p[1], &sd.piv[0], &sd.piv[1], &sd.rbx, &sd.rb})
      if (hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) return LVAE_ERR_LAUNCH;
  }
  out = &sd;
  return 0;
}

}  // namespace lvae
