// Device helpers shared by the Bellman kernels (bellman_kernels.hip: table / init / screen /
// tree / plain; bellman_wide_kernels.hip: the small-grid one-launch sweep): the screening
// constants, the exact candidate value in the literal MATLAB order, the staged screen values,
// the (max value, first index) merge and the expectation EV(i,k) in m order.
#pragma once
#include <hip/hip_runtime.h>

#include "aiy_common.hpp"

namespace aiy {

constexpr double kTau = 1.4210854715202004e-14;  // 2^-46 (error analysis: DESIGN.md §5 A1)
constexpr double kThr = 0.99999999999999644729;  // 1 - 2^-48
constexpr float kThr32 = 0.999998092651367f;      // 1 - 2^-19 (exact in fp32)
constexpr float kBig32 = 1.152921504606847e18f;   // 2^60: fp32-path range guard

typedef float f32x2 __attribute__((ext_vector_type(2)));

// fp64 → fp32 rounded outward by one step past round-to-nearest: a rigorous upper (lower)
// bound of the real value even with the fp64 rounding of x's own computation
__device__ __forceinline__ float f32_up(double x) { return nextafterf((float)x, __builtin_inff()); }
__device__ __forceinline__ float f32_dn(double x) { return nextafterf((float)x, -__builtin_inff()); }

template <int NP>
__device__ __forceinline__ f32x2 ipow2(f32x2 c) {
    static_assert(NP >= 1 && NP <= 8, "screen exponent");
    if constexpr (NP == 1) return c;
    f32x2 c2 = c * c;
    if constexpr (NP == 2) return c2;
    if constexpr (NP == 3) return c2 * c;
    f32x2 c4 = c2 * c2;
    if constexpr (NP == 4) return c4;
    if constexpr (NP == 5) return c4 * c;
    if constexpr (NP == 6) return c4 * c2;
    if constexpr (NP == 7) return (c4 * c2) * c;
    return c4 * c4;
}

// exact value of candidate (c, l, k) in the literal MATLAB order
template <int NP, bool LAB>
__device__ __forceinline__ double bell_val(double c, double ev, double sigma, double dis) {
    double u;
    if constexpr (NP > 0) {
        double p = 1.0 / aiy_ipow(c, NP);  // c.^(1-sigma), sigma = NP + 1
        if constexpr ((NP & (NP - 1)) == 0)
            u = (p - 1) * (-1.0 / NP);  // 1 - sigma = -2^m: the division is exact scaling
        else
            u = (p - 1) / (1 - sigma);
    } else {
        if (!LAB && sigma == 1.0) u = aiy_log(c);  // Aiyagari_VFI.m:74-75 (labour script: no branch)
        else u = (aiy_pow(c, 1.0 - sigma) - 1) / (1 - sigma);
    }
    if constexpr (LAB) return (u - dis) + ev;  // Labor_VFI.m:95-99
    else return u + ev;                        // Aiyagari_VFI.m:79
}

// Screen values t[m] = dd[m]·max(cx[m], 0)^NP of M independent (candidate or bound, state)
// pairs, computed stage by stage with scheduling barriers between the stages so that the M
// chains interleave.  On gfx950 a dependent fp64 VALU op waits ~16-18 cycles for its operand
// while independent ones issue every ~4-6 (tools/micro/fp64_latency.hip): written per pair the
// compiler emits each pair's 5-deep chain back to back and the wave stalls on every op.  The
// operation sequence per pair is aiy_ipow's, so every t is the unstaged expression's bit for
// bit and the screen's rounding analysis is unchanged.
#define AIY_SCHED_BARRIER() __builtin_amdgcn_sched_barrier(0)
template <int NP, int M>
__device__ __forceinline__ void screen_t(double (&t)[M], const double (&cx)[M],
                                         const double (&dd)[M]) {
    double c[M], p[M];
#pragma unroll
    for (int m = 0; m < M; ++m) c[m] = fmax(cx[m], 0.0);
    AIY_SCHED_BARRIER();
#pragma unroll
    for (int m = 0; m < M; ++m) p[m] = c[m];
    constexpr int top = 31 - __builtin_clz((unsigned)NP);
#pragma unroll
    for (int b = top - 1; b >= 0; --b) {
#pragma unroll
        for (int m = 0; m < M; ++m) p[m] = p[m] * p[m];
        AIY_SCHED_BARRIER();
        if ((NP >> b) & 1) {
#pragma unroll
            for (int m = 0; m < M; ++m) p[m] = p[m] * c[m];
            AIY_SCHED_BARRIER();
        }
    }
#pragma unroll
    for (int m = 0; m < M; ++m) t[m] = dd[m] * p[m];
}
// pairs per stage group: 8 candidates × the sub-states of a lane, at most ~16 chains
template <int RL>
struct StageGroup {
    static constexpr int G = RL <= 2 ? 8 : (RL <= 4 ? 4 : 1);
};

// (max value, first index) merge; NaN never enters (MATLAB max omits NaN)
__device__ __forceinline__ bool lexi_take(double val, int q, double& best, int& idx) {
    if (val != val) return false;
    if (idx < 0 || val > best || (val == best && q < idx)) {
        best = val;
        idx = q;
        return true;
    }
    return false;
}

// the same rule without branches (selects only), so that independent evaluations ahead of a
// run of merges stay in one basic block and their dependency chains interleave
__device__ __forceinline__ void lexi_take_sel(double val, int q, double& best, int& idx) {
    const bool take = (val == val) & ((idx < 0) | (val > best) | ((val == best) & (q < idx)));
    best = take ? val : best;
    idx = take ? q : idx;
}

// screening bar of (best, dis_l):  n·(best + dis) − τ·n·(|best| + |dis|)
__device__ __forceinline__ double screen_B(double best, int idx, double dis, int np) {
    if (idx < 0) return -__builtin_inf();
    double nd = (double)np;
    return nd * (best + dis) - kTau * nd * (fabs(best) + fabs(dis));
}

template <bool LAB>
__device__ __forceinline__ double cash(double x, double y, double Ll) {
    if constexpr (LAB) return x + y * Ll;  // (1+r)a_j + (w s_i) L_l   (Labor_VFI.m:81)
    else return x + y;                     // (1+r)a_j + w s_i          (Aiyagari_VFI.m:72)
}

// EV(i,k) = Σ_m (β·P(i,m))·V(m,k) in m order (Aiyagari_VFI.m:79).  Eight rows at a time, every
// load of a chunk (the V column and the P row, at indices clamped into range) in flight before
// the ordered sum, and every term used unconditionally (a row past N adds +0.0, which leaves
// the sum bit for bit as it is: it never holds −0.0).  A load guarded by `m < N` gets sunk
// into its guarded use, after the first wait: one dependent round trip per row (7 in the
// small-grid sweep's prologue before this form).
__device__ __forceinline__ double table_ev(int N, int Na, const double* __restrict__ P,
                                           const double* __restrict__ V, double beta, int i,
                                           int k) {
    double acc = 0.0;
    for (int m0 = 0; m0 < N; m0 += 8) {
        double pm[8], vv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int m = min(m0 + u, N - 1);
            pm[u] = P[i * N + m];
            vv[u] = V[(size_t)m * Na + k];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const double term = (beta * pm[u]) * vv[u];
            acc = acc + (m0 + u < N ? term : 0.0);
        }
    }
    return acc;
}
__device__ __forceinline__ double table_D(double ev, int np) {
    double ne = (double)np * ev;
    return (ne + 1.0) + kTau * (fabs(ne) + 1.0);
}

}  // namespace aiy
