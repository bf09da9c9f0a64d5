// Cross-process sweep hand-off of the KS direct schedule under one process per GPU
// (ks_dist.DirectPeers): every rank publishes "sweeps completed" in a slot of a host page all
// ranks map (fine-grained, system-coherent), and waits for its neighbours' slots before a
// sweep reads their columns.  Both are one-wave kernels on the rank's stream, so the hand-off
// is stream-ordered and never blocks the host.  Vector memory operations only.
#include <hip/hip_runtime.h>

#include "aiy_common.hpp"
#include "ipc_dev.hpp"

namespace aiy {

// lanes q with bit q of `mask` set poll slot q until it reaches v (wave_wait_flags)
__global__ __launch_bounds__(64) void flags_wait_kernel(const unsigned long long* flags,
                                                        unsigned long long mask,
                                                        unsigned long long v,
                                                        long long timeout_ticks,
                                                        unsigned long long* err) {
    wave_wait_flags(flags, mask, v, timeout_ticks, err);
}

// slot `q` := v once every earlier operation on the stream has completed (the stream order puts
// this launch after the sweep; the store is a system-scope release)
__global__ __launch_bounds__(64) void flag_set_kernel(unsigned long long* flags, int q,
                                                      unsigned long long v) {
    if (threadIdx.x == 0)
        __hip_atomic_store(flags + (size_t)q * kFlagStride, v, __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

int launch_flags_wait(const unsigned long long* flags, unsigned long long mask,
                      unsigned long long v, long long timeout_ticks, unsigned long long* err,
                      hipStream_t st) {
    flags_wait_kernel<<<1, 64, 0, st>>>(flags, mask, v, timeout_ticks, err);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}
int launch_flag_set(unsigned long long* flags, int q, unsigned long long v, hipStream_t st) {
    flag_set_kernel<<<1, 64, 0, st>>>(flags, q, v);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}
}  // namespace aiy
