// Kernel-duration timing without event gaps: when armed, the next timed launch on this host
// thread records the two events as part of its own dispatch (hipExtLaunchKernelGGL), so their
// elapsed time is the kernel's execution — the figure rocprofv3 reports — not the kernel plus
// the scheduling gaps of separately recorded events.  The launch disarms them.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

namespace aiy {

struct DispatchEvents {
    hipEvent_t start = nullptr, stop = nullptr;
};
extern thread_local DispatchEvents g_dispatch_ev;

template <class K, class... Args>
inline void launch_dispatch_timed(K kernel, dim3 grid, dim3 block, size_t lds, hipStream_t st,
                                  Args... args) {
    if (g_dispatch_ev.start) {
        hipExtLaunchKernelGGL(kernel, grid, block, lds, st, g_dispatch_ev.start,
                              g_dispatch_ev.stop, 0, args...);
        g_dispatch_ev = DispatchEvents{};
    } else {
        kernel<<<grid, block, lds, st>>>(args...);
    }
}

}  // namespace aiy
