// side_stream.hpp -- the one high-priority side stream (per device) on which the blocked inverses
// (spd_sweep.hip, chol_inv.hip) run their critical chain of pivot-block kernels beside the bulk updates.
#pragma once
#include <hip/hip_runtime.h>

#include <mutex>

namespace lvae {

struct SideStream {
  hipStream_t s = nullptr;
  hipEvent_t fork = nullptr, prep = nullptr, c = nullptr, u2p[2] = {}, piv[2] = {};
  hipEvent_t rbx = nullptr, rb = nullptr;  // the binned residual's plan (kl_closed.hip): x ready / plan done
};

// Held for a call's whole enqueue sequence (every record / wait on the side stream and its events);
// recursive: the exact KL's factor call holds it around the inverse's own sequence.
std::recursive_mutex& side_mutex();
// The current device's side stream and events, created on first use and kept for the process
// lifetime: ONE per device, shared by every caller stream (calls from different caller streams
// serialise on it; the enqueue sequences cannot interleave under side_mutex()).  0 or LVAE_ERR_LAUNCH.
int side_stream(SideStream*& out);

}  // namespace lvae
