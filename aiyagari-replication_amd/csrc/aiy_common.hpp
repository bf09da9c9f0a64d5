// Shared host/device plumbing for the gfx950 solver: status + thread-local error text,
// HIP error checking, small device helpers.  No compatibility layers: CDNA4 only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <cstdarg>
#include <string>

#include "../../include/aiyagari_hip.h"
#include "aiy_math.h"

namespace aiy {

// ---------------------------------------------------------------- errors (host)
void set_error(const char* fmt, ...);
int fail(int code, const char* fmt, ...);
// Wait for an event without parking the thread in the runtime: hipEventQuery in a loop (spin,
// then yield).  Several host threads each blocked in hipEventSynchronize slowed one another's
// launches 2-4x (the GE driver's concurrent solves, tools/ge_concurrency.py); polling does not.
int wait_event(hipEvent_t ev);

#define AIY_HIP(call)                                                                  \
    do {                                                                               \
        hipError_t e_ = (call);                                                        \
        if (e_ != hipSuccess)                                                          \
            return ::aiy::fail(AIY_HIP_ERROR, "%s failed: %s (%s:%d)", #call,          \
                               hipGetErrorString(e_), __FILE__, __LINE__);             \
    } while (0)

#define AIY_TRY(expr)                \
    do {                             \
        int rc_ = (expr);            \
        if (rc_ != AIY_OK) return rc_; \
    } while (0)

// ---------------------------------------------------------------- device helpers
__device__ __forceinline__ int readfirst(int x) { return __builtin_amdgcn_readfirstlane(x); }
// bijective XCD-aware block order (cdna_hip_programming.md T1): blocks with equal b % 8 share
// an XCD and receive consecutive logical ids
__device__ __forceinline__ int xcd_remap(int b, int G) {
    const int q = G / 8, r = G % 8, x = b % 8, slot = b / 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + slot;
}
__device__ __forceinline__ int readlane_i(int x, int l) { return __builtin_amdgcn_readlane(x, l); }
// lane l's double (l wave-uniform) as a wave-uniform value: two v_readlane_b32, no memory
__device__ __forceinline__ double readlane_d(double x, int l) {
    unsigned long long u = __builtin_bit_cast(unsigned long long, x);
    unsigned lo = __builtin_amdgcn_readlane((int)(unsigned)u, l);
    unsigned hi = __builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// DPP lane moves (no LDS round trip, unlike __shfl_xor's ds_bpermute): lanes whose source is
// outside the pattern's row keep their own value.  Controls: quad_perm [1,0,3,2] = 0xB1 (lane
// ^ 1), [2,3,0,1] = 0x4E (lane ^ 2), row_shl:4 = 0x104 (lane + 4 within a row of 16),
// row_mirror = 0x140, row_half_mirror = 0x141, row_bcast:15 = 0x142, row_bcast:31 = 0x143.
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ unsigned dpp_u32(unsigned x) {
    return (unsigned)__builtin_amdgcn_update_dpp((int)x, (int)x, CTRL, ROWS, 0xf, false);
}
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ unsigned long long dpp_u64(unsigned long long x) {
    const unsigned lo = dpp_u32<CTRL, ROWS>((unsigned)x);
    const unsigned hi = dpp_u32<CTRL, ROWS>((unsigned)(x >> 32));
    return ((unsigned long long)hi << 32) | lo;
}
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ double dpp_d(double x) {
    return __builtin_bit_cast(double, dpp_u64<CTRL, ROWS>(__builtin_bit_cast(unsigned long long, x)));
}
// max over the wave of an unsigned 64-bit key, valid in lane 63 (DPP reduction ladder)
__device__ __forceinline__ unsigned long long wave_max_u64_lane63(unsigned long long k) {
    auto mx = [](unsigned long long a, unsigned long long b) { return a > b ? a : b; };
    k = mx(k, dpp_u64<0xB1>(k));
    k = mx(k, dpp_u64<0x4E>(k));
    k = mx(k, dpp_u64<0x141>(k));
    k = mx(k, dpp_u64<0x140>(k));
    k = mx(k, dpp_u64<0x142, 0xa>(k));
    k = mx(k, dpp_u64<0x143, 0xc>(k));
    return k;
}
// the same ladder on a 32-bit signed key (a quarter of the 64-bit ladder's instructions)
__device__ __forceinline__ int wave_max_i32_lane63(int k) {
    k = max(k, (int)dpp_u32<0xB1>((unsigned)k));
    k = max(k, (int)dpp_u32<0x4E>((unsigned)k));
    k = max(k, (int)dpp_u32<0x141>((unsigned)k));
    k = max(k, (int)dpp_u32<0x140>((unsigned)k));
    k = max(k, (int)dpp_u32<0x142, 0xa>((unsigned)k));
    k = max(k, (int)dpp_u32<0x143, 0xc>((unsigned)k));
    return k;
}

// first k in [0, n) with a[k] >= x  (== count of a[k] < x), a non-decreasing.
__device__ __forceinline__ int lower_bound_dev(const double* __restrict__ a, int n, double x) {
    int lo = 0, hi = n;
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (a[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
// largest i with x[i] <= q clamped to [0, n-2]  (interp1 segment; np_oracle / aiy_oracle
// use the same rule)
__device__ __forceinline__ int seg_of_dev(const double* __restrict__ x, int n, double q) {
    int lo = 0, hi = n;
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (x[mid] <= q) lo = mid + 1;
        else hi = mid;
    }
    int i = lo - 1;
    i = i < 0 ? 0 : i;
    i = i > n - 2 ? n - 2 : i;
    return i;
}

// seg_of_dev(x, n, q) searched inside segments [lo_s, hi_s] only, when q provably lies there
// (x[lo_s] <= q unless lo_s == 0, q < x[hi_s + 1] unless hi_s == n - 2): the same answer in
// log2(hi_s - lo_s) dependent loads; otherwise (or for NaN q) the full search
__device__ __forceinline__ int seg_range_dev(const double* __restrict__ x, int n, double q,
                                             int lo_s, int hi_s) {
    const bool ok = (lo_s <= 0 || x[lo_s] <= q) && (hi_s >= n - 2 || q < x[hi_s + 1]) && q == q &&
                    lo_s <= hi_s;
    if (!ok) return seg_of_dev(x, n, q);
    int lo = max(lo_s, 0) + 1, hi = min(hi_s, n - 2) + 1;
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (x[mid] <= q) lo = mid + 1;
        else hi = mid;
    }
    return lo - 1;
}

// IEEE-ordered key for a non-negative double: uint64 compare == double compare
__device__ __forceinline__ unsigned long long nonneg_key(double x) {
    return (unsigned long long)aiy_dbits(x);
}

// ---------------------------------------------------------------- max |Δ| reduction
// max|v_new - v_old| ignoring NaN (MATLAB max(..., 'all')): wave shuffles, then LDS across
// the block's waves, then ONE atomicMax per block on IEEE bits (order-independent, hence
// deterministic) into slot blockIdx % kDiffSlots, so no single address is contended.
constexpr int kDiffSlots = 64;
__device__ __forceinline__ void block_max_to_slots(bool ok, double d,
                                                   unsigned long long* __restrict__ slots) {
    __shared__ unsigned long long s_key[16];
    __shared__ int s_any[16];
    unsigned long long key = ok ? (unsigned long long)aiy_dbits(d) : 0ull;
    int any = __ballot(ok) != 0ull;
    key = wave_max_u64_lane63(key);
    {
        const unsigned lo = __builtin_amdgcn_readlane((int)(unsigned)key, 63);
        const unsigned hi = __builtin_amdgcn_readlane((int)(unsigned)(key >> 32), 63);
        key = ((unsigned long long)hi << 32) | lo;
    }
    const int wave = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    if ((threadIdx.x & 63) == 0) {
        s_key[wave] = key;
        s_any[wave] = any;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long k = 0;
        int a = 0;
        for (int q = 0; q < nw; ++q) {
            k = s_key[q] > k ? s_key[q] : k;
            a |= s_any[q];
        }
        if (a) {
            unsigned long long* sl = slots + 2 * (blockIdx.x % kDiffSlots);
            atomicMax(sl, k);
            atomicOr(sl + 1, 1ull);
        }
    }
}

// the same for a one-wave workgroup: the wave's maximum goes straight from lane 0 to the slot —
// no LDS, no workgroup barrier (whose release fence would make the wave wait for all of its
// output stores before the atomics could issue)
__device__ __forceinline__ void wave_max_to_slots(bool ok, double d,
                                                  unsigned long long* __restrict__ slots) {
    unsigned long long key = ok ? (unsigned long long)aiy_dbits(d) : 0ull;
    const bool any = __ballot(ok) != 0ull;
    key = wave_max_u64_lane63(key);
    const unsigned lo = __builtin_amdgcn_readlane((int)(unsigned)key, 63);
    const unsigned hi = __builtin_amdgcn_readlane((int)(unsigned)(key >> 32), 63);
    key = ((unsigned long long)hi << 32) | lo;
    if (any && (threadIdx.x & 63) == 0) {
        unsigned long long* sl = slots + 2 * (blockIdx.x % kDiffSlots);
        atomicMax(sl, key);
        atomicOr(sl + 1, 1ull);
    }
}

inline int is_int_ge(double x, double lo) {
    return x >= lo && x < 64 && (double)(int64_t)x == x;
}

}  // namespace aiy
