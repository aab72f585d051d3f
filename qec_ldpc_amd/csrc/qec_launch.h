// Kernel launches that carry events (HIP translation units only).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

namespace qec {

// Launches `kernel` with `start` / `stop` (either may be null) marked at the kernel's own start and
// end, so no separate marker packet sits between it and its neighbours: between back-to-back
// launches an hipEventRecord costs ~4 us of GPU time, an event carried by the kernel ~1 us
// (tools/kbench/event_probe.hip, profiles/r06/event_probe.txt).  The decode calls' workspace event
// is carried this way (P7 configs[1] +2..+7 %, profiles/r06/ab/cmp_event_carry.txt).
template <class F, class... Args>
inline void launch_marked(F kernel, dim3 grid, dim3 block, uint32_t smem, hipStream_t st, hipEvent_t start,
                          hipEvent_t stop, Args... args)
{
    if (start != nullptr || stop != nullptr)
        hipExtLaunchKernelGGL(kernel, grid, block, smem, st, start, stop, 0u, args...);
    else
        hipLaunchKernelGGL(kernel, grid, block, smem, st, args...);
}

}  // namespace qec
