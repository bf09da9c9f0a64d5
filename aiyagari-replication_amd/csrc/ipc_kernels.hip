// Cross-process sweep hand-off of the KS direct schedule under one process per GPU
// (ks_dist.DirectPeers): every rank publishes "sweeps completed" in a slot of a host page all
// ranks map (fine-grained, system-coherent), and waits for its neighbours' slots before a
// sweep reads their columns.  Both are one-wave kernels on the rank's stream, so the hand-off
// is stream-ordered and never blocks the host.  Vector memory operations only.
#include <hip/hip_runtime.h>

#include "aiy_common.hpp"

namespace aiy {
constexpr int kFlagStride = 16;  // slots 128 B apart (one cache line each)

// lanes q with bit q of `mask` set poll slot q until it reaches v; a wave that sees no progress
// for `timeout_ticks` of the 100 MHz wall clock sets *err and leaves (a dead neighbour must not
// hang the device: the host checks err and aborts the solve)
__global__ __launch_bounds__(64) void flags_wait_kernel(const unsigned long long* flags,
                                                        unsigned long long mask,
                                                        unsigned long long v,
                                                        long long timeout_ticks,
                                                        unsigned long long* err) {
    const int q = threadIdx.x;
    // an earlier wait of this rank already timed out: the schedule is void, do not wait again
    if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0ull) return;
    const bool mine = (mask >> q) & 1ull;
    const long long t0 = (long long)wall_clock64();
    bool ok = !mine;
    while (!__all(ok)) {
        if (!ok) {
            const unsigned long long f = __hip_atomic_load(flags + (size_t)q * kFlagStride,
                                                           __ATOMIC_ACQUIRE,
                                                           __HIP_MEMORY_SCOPE_SYSTEM);
            ok = f >= v;
        }
        if ((long long)wall_clock64() - t0 > timeout_ticks) {
            if (!ok)
                __hip_atomic_store(err, 1ull + (unsigned long long)q, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
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
