// Device side of the cross-process sweep hand-off (KS direct schedule): polling
// the neighbours' "versions published" slots in the host page every rank maps.  Vector memory
// operations only.
#pragma once
#include <hip/hip_runtime.h>

namespace aiy {
constexpr int kFlagStride = 16;  // slots 128 B apart (one cache line each)

// One wave: lanes q with bit q of `mask` poll slot q (relaxed system-scope loads, s_sleep between
// rounds) until it reaches v; no progress for `timeout_ticks` of the 100 MHz wall clock stores
// 1 + q in *err and gives up (a dead neighbour must not hang the device; the host checks err).
// An err already set returns at once (the schedule is void).  Returns after one system-scope
// acquire (the guide's consumer form: relaxed poll, then ONE acquire), so the wave's later loads
// of the neighbours' memory see what they wrote before publishing.
__device__ inline void wave_wait_flags(const unsigned long long* flags, unsigned long long mask,
                                       unsigned long long v, long long timeout_ticks,
                                       unsigned long long* err) {
    const int q = threadIdx.x & 63;
    if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0ull) return;
    const bool mine = (mask >> q) & 1ull;
    const long long t0 = (long long)wall_clock64();
    bool ok = !mine;
    while (!__all(ok)) {
        if (!ok) {
            const unsigned long long f = __hip_atomic_load(flags + (size_t)q * kFlagStride,
                                                           __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_SYSTEM);
            ok = f >= v;
        }
        if (__all(ok)) break;
        if ((long long)wall_clock64() - t0 > timeout_ticks) {
            if (!ok)
                __hip_atomic_store(err, 1ull + (unsigned long long)q, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope
}
}  // namespace aiy
