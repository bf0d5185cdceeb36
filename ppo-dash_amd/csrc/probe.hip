// Diagnostic kernel for the CU-contention measurement (DESIGN.md §7,
// tools/cu_contention.py): a stand-in for a collective's kernel on a side
// stream — `blocks` workgroups that each hold their CU for `ticks` of the
// 100 MHz real-time counter, then record when they started and ended.  Not on
// the training path.
#include "common.h"

namespace {

__global__ void probe_side_kernel(long long ticks, long long* __restrict__ stamps) {
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  long long t = t0;
  while (t - t0 < ticks) {
    __builtin_amdgcn_s_sleep(2);
    t = (long long)__builtin_amdgcn_s_memrealtime();
  }
  if (threadIdx.x == 0) {   // vector stores
    stamps[2 * blockIdx.x] = t0;
    stamps[2 * blockIdx.x + 1] = t;
  }
}

}  // namespace

// stamps: [blocks][2] long long (start, end in 100 MHz ticks of s_memrealtime)
PPO_API int ppo_probe_side_kernel(int blocks, int threads, long long ticks, long long* stamps, void* stream) {
  PPO_REQUIRE(blocks > 0 && threads > 0 && threads <= 1024 && ticks >= 0 && stamps,
              "ppo_probe_side_kernel: blocks=%d threads=%d", blocks, threads);
  probe_side_kernel<<<blocks, threads, 0, as_stream(stream)>>>(ticks, stamps);
  PPO_LAUNCH_CHECK("probe_side_kernel");
  return 0;
}

// the current 100 MHz real-time counter value, read by a one-thread kernel (stamps[0])
namespace {
__global__ void probe_now_kernel(long long* __restrict__ out) {
  out[0] = (long long)__builtin_amdgcn_s_memrealtime();
}
}  // namespace
PPO_API int ppo_probe_now(long long* out, void* stream) {
  PPO_REQUIRE(out, "ppo_probe_now: null");
  probe_now_kernel<<<1, 64, 0, as_stream(stream)>>>(out);
  PPO_LAUNCH_CHECK("probe_now_kernel");
  return 0;
}
