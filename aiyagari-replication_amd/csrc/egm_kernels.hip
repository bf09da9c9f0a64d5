// A4 / A5 — EGM inversion + interpolation step on gfx950.
//   A4: Aiyagari_EGM.m:75-107 (GE copy :177-211)
//   A5: Aiyagari_Endogenous_Labor_EGM.m:68-104 (GE copy :174-211)
// Arrays are [N][Na] (== MATLAB's Na x N policy_c, column j = productivity state).
//
// Kernel 1 (one thread per (j, a)): u'(c_m) once per (m, a), the Euler right-hand side
//   Σ_m ((β(1+r))·P(j,m))·c_m^-σ in m order (:80-85), c̃ = RHS^(-1/σ) (:88) and the endogenous
//   grid â = ((c̃ + a) − w s_j)/(1+r) (:92) — with the labour FOC l = ((w s_j) c̃^-σ / φ)^(1/θ)
//   (:86) and â = ((c̃ + a) − (w s_j) l)/(1+r) (:87) in A5.
// Kernel 2 (one thread per (j, a)): interp1(â_j, y, a_grid(a), 'linear', 'extrap') on the
//   monotone â_j (y = a_grid in A4, c̃_j in A5), the borrowing clamp, the recovered policies,
//   and max|c_next − c| ignoring NaN (:106) via atomicMax on IEEE bits.  It also flags a
//   non-increasing â_j (MATLAB's interp1 would sort or error there).
// HBM-bound: 24 B per state per iteration (c in, c_next out, policy_k out), +8 B with labour.
#include "aiy_common.hpp"
#include "dispatch.hpp"
#include "egm.hpp"

namespace aiy {

__device__ __forceinline__ double uprime_dev(double c, double sigma, int ns) {
    return ns > 0 ? 1.0 / aiy_ipow(c, ns) : aiy_pow(c, -sigma);  // c.^(-sigma)
}

__device__ __forceinline__ double labor_dev(double c, double ws, double sigma, int ns,
                                            double phi, double theta) {
    double x = (ws * uprime_dev(c, sigma, ns)) / phi;  // u_prime_l_inv(w s .* u_prime_c(c))
    return (1.0 / theta == 1.0) ? x : aiy_pow(x, 1.0 / theta);
}

// Kernel 1: one workgroup per 64 asset nodes, one wave per productivity state.  Phase 1: wave m
// evaluates u'(c_m) for its 64 nodes into LDS (once per (m, a), as the script's vectorised
// u_prime_c(policy_c) does).  Phase 2: wave j forms the Euler sum over m in m order from LDS,
// then one non-integer power and the endogenous grid — one pow per thread instead of N in a
// row, and N times as many waves in flight.  The first workgroup also clears this step's diff
// slots and flags (the interp kernel of the same step accumulates into them).
__global__ __launch_bounds__(1024) void egm_rhs_kernel(EgmArgs A) {
    __shared__ double s_up[16][64];
    const int lane = threadIdx.x & 63;
    const int m = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // blockDim = 64·N
    const int N = A.N, Na = A.Na;
    const int a_i = blockIdx.x * 64 + lane;
    const bool ok = a_i < Na;
    if (blockIdx.x == 0) {  // blockDim = 64·N may be smaller than the 2·kDiffSlots words
        for (int q = threadIdx.x; q < 2 * kDiffSlots; q += blockDim.x) A.diff[q] = 0ull;
        if (threadIdx.x == 0) *A.flags = 0u;
    }
    const int j = m;
    const double coef0 = A.beta * (1 + A.r);
    double pj[16];  // row j of βP-ready weights, scalar loads issued before the barrier
#pragma unroll
    for (int q = 0; q < 16; ++q) pj[q] = q < N ? coef0 * A.P[j * N + q] : 0.0;
    s_up[m][lane] = ok ? uprime_dev(A.c[(size_t)m * Na + a_i], A.sigma, A.ns) : 0.0;
    __syncthreads();
    if (!ok) return;
    double acc = 0.0;
#pragma unroll
    for (int q = 0; q < 16; ++q)
        if (q < N) acc = acc + pj[q] * s_up[q][lane];
    const double cn = aiy_pow(acc, -1.0 / A.sigma);  // :88
    const double ws = A.w * A.s[j];
    const double ag = A.a[a_i];
    double ah;
    if (A.labor) {
        const double ls = labor_dev(cn, ws, A.sigma, A.ns, A.phi, A.theta);
        ah = ((cn + ag) - ws * ls) / (1 + A.r);
    } else {
        ah = ((cn + ag) - ws) / (1 + A.r);
    }
    A.ahat[(size_t)j * Na + a_i] = ah;
    if (A.labor) A.cnext[(size_t)j * Na + a_i] = cn;  // (A4 interpolates a_grid, not c̃)
}

// #{k in [lo, hi) : x[k] <= q} + lo for a per-lane query (binary search, global memory)
__device__ __forceinline__ int count_le(const double* __restrict__ x, int lo, int hi, double q) {
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (x[mid] <= q) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// Kernel 2: one wave per (j, 64 consecutive asset nodes).  interp1's segment is
// clamp(#{k : â_k <= a}, 1, Na−1) − 1 (seg_of_dev).  The wave's queries a_grid(a0..a0+63)
// are increasing, so on an increasing â every lane's count lies between the counts of the
// first and the last query.  Those two come from a 64-ary search (each round, 64 lanes load
// 64 evenly spaced pivots and one ballot narrows the range 64-fold: 3 dependent rounds at
// Na = 20,000 instead of 15); the â values between them (≤ 256) are staged in LDS in one round
// trip and each lane finishes its count there.  A wider spread (or a non-increasing â, which
// the flag turns into an error) falls back to a per-lane search over the narrowed range, so
// the count — and everything after it — is the plain binary search's.
// interp1 of row j's 64 queries a_grid(a0 .. a0+63), a0 = 64·tile (one wave): writes
// policy_c_next (cout), policy_k (and policy_l), flags a non-increasing â; returns whether the
// lane holds a query and sets its |Δc| (d) and policy_c_next (cn).  s_xw / s_yw: the wave's
// 256-double LDS windows of x = â_j and y (a_grid in A4, c̃_j in A5).
// Dependent memory rounds per wave (round 4): (1) the two segment hints, with every load that
// does not depend on them in flight beside them (the query, policy_c for |Δc|, the monotonicity
// pair); (2) the window of x AND y around the hinted segments; everything after the count comes
// from LDS.  (Round 3 re-read x[sgi], x[sgi+1], y[sgi], y[sgi+1] from memory after the count —
// a third dependent round per step.)  Same values, same operations: bit for bit the plain
// binary search + interpolation.
__device__ __forceinline__ bool egm_interp_wave(const EgmArgs& A, int j, int tile,
                                                double* s_xw, double* s_yw, double& d, double& cn,
                                                long long* cy = nullptr) {
    const int lane = threadIdx.x & 63;
    const int Na = A.Na;
    if (cy) cy[0] = (long long)__builtin_amdgcn_s_memtime();
    const int a0 = tile * 64, a_i = a0 + lane;
    const int last = min(63, Na - 1 - a0);
    const bool okl = lane <= last;
    const size_t t = (size_t)j * Na + (okl ? a_i : a0);
    const double* __restrict__ x = A.ahat + (size_t)j * Na;
    const double* __restrict__ y = A.labor ? A.cnext + (size_t)j * Na : A.a;
    // round 1: independent loads together
    const double q = A.a[okl ? a_i : a0 + last];
    const double c_old = A.c[t];
    int h0 = -1, h1 = -1;
    if (A.seg) {
        h0 = A.seg[(size_t)j * Na + a0];
        h1 = A.seg[(size_t)j * Na + a0 + last];
    }
    // the previous step's segments as hints: the wave stages x and y over [h_first − 16,
    // h_last + 18) (h = the first and the last lane's segment) in LDS in one round trip and every
    // lane checks that its count #{k : x_k <= q} lies inside — x_{lo−1} <= q < x_{hi} — before
    // finishing it there; if any lane's does not (segments moved further, or no hints yet), the
    // wave runs the full 64-ary search below.  The count, hence everything after it, is the
    // search's.
    int sgi = -1, e0 = -1;  // e0: the segment's index in the LDS windows (window path)
    if (A.seg) {
        const int wlo = max(min(h0, h1) - 16, 0), whi = min(max(h0, h1) + 18, Na);
        if (h0 >= 0 && h1 >= 0 && h0 <= Na - 2 && h1 <= Na - 2 && whi - wlo + 2 <= 256) {
            // s_xw[0] = x_{wlo−1} (−inf at 0), s_xw[1 + u] = x_{wlo+u}, s_xw[n−1] = x_{whi} (+inf
            // at Na), s_yw the same y: all loads in flight, then the LDS writes
            const int n = whi - wlo + 2;
            double v[4], vy[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int k = wlo - 1 + u * 64 + lane;
                const bool in = u * 64 + lane < n && k >= 0 && k < Na;
                v[u] = in ? x[k] : 0.0;
                vy[u] = in ? y[k] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int e = u * 64 + lane, k = wlo - 1 + e;
                if (e < n) {
                    s_xw[e] = k < 0 ? -__builtin_inf() : (k >= Na ? __builtin_inf() : v[u]);
                    s_yw[e] = vy[u];
                }
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            const bool inl = s_xw[0] <= q;     // count >= wlo
            const bool inr = q < s_xw[n - 1];  // count <= whi
            if (__ballot(okl && !(inl && inr)) == 0ull) {
                int lo = 1, hi = n - 1;  // 1 + #{k in [wlo, whi) : x_k <= q} over s_xw[1 .. n−1)
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (s_xw[mid] <= q) lo = mid + 1;
                    else hi = mid;
                }
                int c = wlo + lo - 1 - 1;  // count − 1
                c = c < 0 ? 0 : c;
                sgi = c > Na - 2 ? Na - 2 : c;
                e0 = sgi - wlo + 1;  // in [0, n − 2]; e0 and e0 + 1 hold real x and y (see DESIGN)
            }
        }
    }
    if (cy) cy[1] = (long long)__builtin_amdgcn_s_memtime();
    if (sgi < 0) {
    const double q0 = readlane_d(q, 0), q1 = readlane_d(q, last);
    int lo0 = 0, hi0 = Na, lo1 = 0, hi1 = Na;
    while (lo0 < hi0 || lo1 < hi1) {  // wave-uniform bounds
        const int st0 = max((hi0 - lo0 + 63) >> 6, 1), st1 = max((hi1 - lo1 + 63) >> 6, 1);
        const int k0 = lo0 + (lane + 1) * st0 - 1, k1 = lo1 + (lane + 1) * st1 - 1;
        const bool v0 = k0 < hi0, v1 = k1 < hi1;
        const double x0 = v0 ? x[k0] : 0.0, x1 = v1 ? x[k1] : 0.0;
        const int c0 = __popcll(__ballot(v0 && x0 <= q0));
        const int c1 = __popcll(__ballot(v1 && x1 <= q1));
        if (lo0 < hi0) {
            const int nh = lo0 + (c0 + 1) * st0 - 1;
            lo0 += c0 * st0;
            hi0 = nh < hi0 ? nh : hi0;
        }
        if (lo1 < hi1) {
            const int nh = lo1 + (c1 + 1) * st1 - 1;
            lo1 += c1 * st1;
            hi1 = nh < hi1 ? nh : hi1;
        }
    }
    // every lane's count is in [lo0, lo1] (increasing â and queries)
    int cnt;
    const int span = lo1 - lo0;
    __builtin_amdgcn_wave_barrier();  // (window reads above, if any, are done)
    if (span >= 0 && span <= 256) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = lo0 + u * 64 + lane;
            if (u * 64 + lane < span) s_xw[u * 64 + lane] = x[k];
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        int lo = 0, hi = span;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (s_xw[mid] <= q) lo = mid + 1;
            else hi = mid;
        }
        cnt = lo0 + lo;
    } else {
        cnt = count_le(x, min(lo0, lo1), max(lo0, lo1), q);
    }
    sgi = cnt - 1;
    sgi = sgi < 0 ? 0 : sgi;
    sgi = sgi > Na - 2 ? Na - 2 : sgi;
    }
    // the hints of the next step: only the tile's first and last lanes' segments are read
    if (A.seg && okl && (lane == 0 || lane == last)) A.seg[t] = sgi;
    if (cy) cy[2] = (long long)__builtin_amdgcn_s_memtime();
    d = 0.0;
    cn = 0.0;
    if (!okl) return false;
    double x0, x1, y0, y1;
    if (e0 >= 0) {  // from the LDS windows
        x0 = s_xw[e0];
        x1 = s_xw[e0 + 1];
        y0 = s_yw[e0];
        y1 = s_yw[e0 + 1];
    } else {
        x0 = x[sgi];
        x1 = x[sgi + 1];
        y0 = y[sgi];
        y1 = y[sgi + 1];
    }
    const double tt = (q - x0) / (x1 - x0);
    double g = y0 + tt * (y1 - y0);
    const double ws = A.w * A.s[j];
    if (A.labor) {
        if (q < A.amin) g = A.amin;  // :91 (a no-op for a_grid >= amin)
        cn = g;
        const double l = labor_dev(g, ws, A.sigma, A.ns, A.phi, A.theta);  // :95
        const double k = ((1 + A.r) * q + ws * l) - g;                       // :98
        A.pk[t] = k < 0 ? 0.0 : k;                                           // :99
        if (A.pl) A.pl[t] = l;
    } else {
        if (g < A.amin) g = A.amin;  // :98
        A.pk[t] = g;
        cn = ((1 + A.r) * q + ws) - g;  // :102
    }
    A.cout[t] = cn;
    d = fabs(cn - c_old);
    if (cy) {
        __builtin_amdgcn_s_waitcnt(0);  // (instrumentation) the loads above have landed
        cy[3] = (long long)__builtin_amdgcn_s_memtime();
    }
    return true;
}

// (instrumentation) one record per wave: entry/exit wall clock, XCC, then shader cycles of
// the phases: search, window count, interpolation loads, the rest (RHS of t+1 / reduction)
__device__ __forceinline__ void egm_trace(const EgmArgs& A, int rec, long long t_in,
                                          const long long* cy, int ncy) {
    if ((threadIdx.x & 63) != 0) return;
    const long long now = (long long)__builtin_amdgcn_s_memtime();
    long long* tr = A.trace + 16 * (size_t)rec;
    tr[0] = t_in;
    tr[1] = (long long)wall_clock64();
    tr[2] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));  // HW_REG_XCC_ID
    for (int p = 1; p < ncy; ++p) tr[2 + p] = cy[p] - cy[p - 1];
    tr[2 + ncy] = now - cy[ncy - 1];
}

// interp1 needs an increasing â_j: a non-increasing adjacent pair of the wave's 64 nodes sets
// the flag word (the reference's interp1 would sort or fail, Aiyagari_EGM.m:95).  The pair is
// loaded after the interpolation's dependent rounds (issued with the interpolation in the
// register budget, they had pushed the chained kernel into scratch) and tested at the end.
struct EgmOrderPair {
    double xm, xc;
    bool ok;
};
__device__ __forceinline__ EgmOrderPair egm_order_load(const EgmArgs& A, int j, int tile) {
    const int a_i = tile * 64 + (threadIdx.x & 63);
    const double* __restrict__ x = A.ahat + (size_t)j * A.Na;
    const bool ok = a_i > 0 && a_i < A.Na;
    return {ok ? x[a_i - 1] : 0.0, ok ? x[a_i] : 1.0, ok};
}
__device__ __forceinline__ void egm_order_check(const EgmArgs& A, const EgmOrderPair& p) {
    if (p.ok && !(p.xm < p.xc)) atomicOr(A.flags, 1u);
}

__global__ __launch_bounds__(256) void egm_interp_kernel(EgmArgs A, int ntile) {
    __shared__ double s_x[4][256];
    __shared__ double s_y[4][256];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wv = blockIdx.x * 4 + wave;
    bool ok = false;
    double d = 0.0;
    long long cy[4] = {0, 0, 0, 0};
    const long long t_in = A.trace ? (long long)wall_clock64() : 0;
    if (wv < A.N * ntile) {  // wave-uniform
        const int j = wv / ntile, tile = wv - j * ntile;
        double cn;
        ok = egm_interp_wave(A, j, tile, s_x[wave], s_y[wave], d, cn, A.trace ? cy : nullptr) &&
             d == d;
        egm_order_check(A, egm_order_load(A, j, tile));
    }
    block_max_to_slots(ok, d, A.diff);
    if (A.trace && wv < A.N * ntile) egm_trace(A, wv, t_in, cy, 4);
}

// Chained steps for large grids (the speculative solve, Na > 1,024): ONE launch per step in
// the steady state.  The Euler RHS of a node needs policy_c at that node for every m only, so
// the workgroup that produces step t's policy_c_next on a tile of 64 nodes (wave j: interp1 of
// row j, as egm_interp_kernel) holds step t+1's inputs there and forms step t+1's RHS and â on
// the same tile (as egm_rhs_kernel, u'(c_m) through LDS) into the other â/c̃ buffer.  The
// interp1 of step t+1 then runs in the next launch, after every â of step t+1 exists.  Same
// operations on the same values as rhs + interp, so bit for bit the two-launch step.  The first
// workgroup clears step t+1's slot set and flag word (diff_clear) for the next launch.
// TR: the instrumented instantiation (per-wave phase trace, aiy_ws_set_timing bit 2); the
// production one has no trace plumbing at all — a runtime-selected pointer to the cycle stamps
// had put them (and 144 B per lane) in scratch memory.
template <bool TR>
__global__ __launch_bounds__(1024) void egm_chain_kernel(EgmArgs A) {
    __shared__ double s_x[16][256];
    __shared__ double s_y[16][256];
    __shared__ double s_up[16][64];
    const int lane = threadIdx.x & 63;
    const int m = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // blockDim = 64·N
    const int N = A.N, Na = A.Na;
    if (blockIdx.x == 0 && A.diff_clear)
        for (int q = threadIdx.x; q < kEgmSlotWords; q += blockDim.x) A.diff_clear[q] = 0ull;
    const int j = m;
    const double coef0 = A.beta * (1 + A.r);
    double pj[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) pj[q] = q < N ? coef0 * A.P[j * N + q] : 0.0;
    double d, cn;
    long long cy[4] = {0, 0, 0, 0};
    const long long t_in = TR ? (long long)wall_clock64() : 0;
    const bool okl = egm_interp_wave(A, j, blockIdx.x, s_x[m], s_y[m], d, cn, TR ? cy : nullptr);
    const bool ok = okl && d == d;
    const EgmOrderPair ord = egm_order_load(A, j, blockIdx.x);  // (latency under the RHS below)
    // step t+1's Euler RHS on this tile: u'(policy_c_next) of every row through LDS
    const int a_i = blockIdx.x * 64 + lane;
    s_up[m][lane] = okl ? uprime_dev(cn, A.sigma, A.ns) : 0.0;
    __syncthreads();
    if (okl) {
        double acc = 0.0;
#pragma unroll
        for (int q = 0; q < 16; ++q)
            if (q < N) acc = acc + pj[q] * s_up[q][lane];
        const double c2 = aiy_pow(acc, -1.0 / A.sigma);  // :88
        const double ws = A.w * A.s[j];
        const double ag = A.a[a_i];  // (the interp query: an L1 hit)
        double ah;
        if (A.labor) {
            const double ls = labor_dev(c2, ws, A.sigma, A.ns, A.phi, A.theta);
            ah = ((c2 + ag) - ws * ls) / (1 + A.r);
        } else {
            ah = ((c2 + ag) - ws) / (1 + A.r);
        }
        A.ahat_next[(size_t)j * Na + a_i] = ah;
        if (A.labor) A.cnext_next[(size_t)j * Na + a_i] = c2;  // (A4 interpolates a_grid, not c̃)
    }
    egm_order_check(A, ord);
    block_max_to_slots(ok, d, A.diff);
    if constexpr (TR) egm_trace(A, blockIdx.x * N + j, t_in, cy, 4);
}

// Small grids (the scripts' Na = 400, up to 1,024): one launch per step, one workgroup per productivity
// state j.  At these sizes a step is two launches' fixed cost (≈ 6 µs each, at Na = 400 as at
// 20,000), not work, so the row's whole step runs in one workgroup: the Euler RHS and â_j as
// egm_rhs_kernel (u'(c_m) per (m, a) recomputed per row — N·Na divisions, a few per thread), â_j
// (and c̃_j in A5) staged in LDS, then interp1 as egm_interp_kernel with the count by a plain
// binary search of the LDS row (the same count on a non-decreasing â).  Workgroup j owns diff
// slot j outright — {max|Δc| bits, bit 0: some finite Δc | bit 1: â_j not increasing} — and
// workgroup 0 clears the other slots and the flag word, so nothing is cleared and accumulated
// by different workgroups of one launch.
// (kEgmFusedMaxNa = 1,024, egm.hpp: one state per thread — measured 8.8 vs 12.0 us per step
// at Na = 400, 27.6 vs 11.7 at 4,096 with 4 per thread)
__global__ __launch_bounds__(1024) void egm_fused_kernel(EgmArgs A) {
    __shared__ double s_x[kEgmFusedMaxNa];
    __shared__ double s_y[kEgmFusedMaxNa];
    __shared__ unsigned long long s_key[16];
    __shared__ int s_fl[16];
    const int j = blockIdx.x, N = A.N, Na = A.Na;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (j == 0) {
        for (int q = N + threadIdx.x; q < kDiffSlots; q += blockDim.x) {
            A.diff[2 * q] = 0ull;
            A.diff[2 * q + 1] = 0ull;
        }
        if (threadIdx.x == 0) *A.flags = 0u;
    }
    const double coef0 = A.beta * (1 + A.r);
    const double ws = A.w * A.s[j];
    for (int a_i = threadIdx.x; a_i < Na; a_i += blockDim.x) {  // :80-92 (labour :80-87)
        double cq[16];  // every c_q(a) load in flight before the ordered Euler sum
#pragma unroll
        for (int q = 0; q < 16; ++q) cq[q] = q < N ? A.c[(size_t)q * Na + a_i] : 1.0;
        double acc = 0.0;
#pragma unroll
        for (int q = 0; q < 16; ++q)
            if (q < N) acc = acc + (coef0 * A.P[j * N + q]) * uprime_dev(cq[q], A.sigma, A.ns);
        const double cn = aiy_pow(acc, -1.0 / A.sigma);
        const double ag = A.a[a_i];
        double ah;
        if (A.labor) {
            const double ls = labor_dev(cn, ws, A.sigma, A.ns, A.phi, A.theta);
            ah = ((cn + ag) - ws * ls) / (1 + A.r);
        } else {
            ah = ((cn + ag) - ws) / (1 + A.r);
        }
        s_x[a_i] = ah;
        s_y[a_i] = A.labor ? cn : ag;
    }
    __syncthreads();
    unsigned long long key = 0ull;
    bool ok = false, bad = false;
    for (int a_i = threadIdx.x; a_i < Na; a_i += blockDim.x) {  // :93-106 (labour :88-104)
        const size_t t = (size_t)j * Na + a_i;
        const double q = A.labor ? A.a[a_i] : s_y[a_i];  // a_grid(a_i) (A4 staged it in s_y)
        int lo = 0, hi = Na;  // #{k : â_k <= q}
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (s_x[mid] <= q) lo = mid + 1;
            else hi = mid;
        }
        int sgi = lo - 1;
        sgi = sgi < 0 ? 0 : sgi;
        sgi = sgi > Na - 2 ? Na - 2 : sgi;
        const double x0 = s_x[sgi], x1 = s_x[sgi + 1];
        const double tt = (q - x0) / (x1 - x0);
        double g = s_y[sgi] + tt * (s_y[sgi + 1] - s_y[sgi]);
        if (a_i > 0 && !(s_x[a_i - 1] < s_x[a_i])) bad = true;
        double cn;
        if (A.labor) {
            if (q < A.amin) g = A.amin;
            cn = g;
            const double l = labor_dev(g, ws, A.sigma, A.ns, A.phi, A.theta);
            const double k = ((1 + A.r) * q + ws * l) - g;
            A.pk[t] = k < 0 ? 0.0 : k;
            if (A.pl) A.pl[t] = l;
        } else {
            if (g < A.amin) g = A.amin;
            A.pk[t] = g;
            cn = ((1 + A.r) * q + ws) - g;
        }
        A.cout[t] = cn;
        const double d = fabs(cn - A.c[t]);
        if (d == d) {
            const unsigned long long kb = (unsigned long long)aiy_dbits(d);
            key = kb > key ? kb : key;
            ok = true;
        }
    }
    key = wave_max_u64_lane63(key);
    const unsigned lo32 = __builtin_amdgcn_readlane((int)(unsigned)key, 63);
    const unsigned hi32 = __builtin_amdgcn_readlane((int)(unsigned)(key >> 32), 63);
    const int fl = (__ballot(ok) != 0ull ? 1 : 0) | (__ballot(bad) != 0ull ? 2 : 0);
    if (lane == 0) {
        s_key[wave] = ((unsigned long long)hi32 << 32) | lo32;
        s_fl[wave] = fl;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long k = 0ull;
        int f = 0;
        for (int v = 0; v < (int)(blockDim.x >> 6); ++v) {
            k = s_key[v] > k ? s_key[v] : k;
            f |= s_fl[v];
        }
        A.diff[2 * j] = k;
        A.diff[2 * j + 1] = (unsigned long long)f;
    }
}

int launch_egm_rhs(const EgmArgs& A, hipStream_t st) {
    if (A.N > 16) return fail(AIY_BAD_SHAPE, "EGM kernels support N <= 16 productivity states");
    egm_rhs_kernel<<<(A.Na + 63) / 64, 64 * A.N, 0, st>>>(A);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}

int launch_egm_chain(const EgmArgs& A, hipStream_t st) {
    if (A.N > 16) return fail(AIY_BAD_SHAPE, "EGM kernels support N <= 16 productivity states");
    if (A.trace)
        launch_dispatch_timed(egm_chain_kernel<true>, dim3((A.Na + 63) / 64), dim3(64 * A.N), 0, st, A);
    else
        launch_dispatch_timed(egm_chain_kernel<false>, dim3((A.Na + 63) / 64), dim3(64 * A.N), 0, st, A);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}

int launch_egm_step(const EgmArgs& A, hipStream_t st) {
    if (A.N > 16) return fail(AIY_BAD_SHAPE, "EGM kernels support N <= 16 productivity states");
    if (A.fused && A.Na >= 2 && A.Na <= kEgmFusedMaxNa) {
        egm_fused_kernel<<<A.N, 1024, 0, st>>>(A);
        AIY_HIP(hipGetLastError());
        return AIY_OK;
    }
    const int ntile = (A.Na + 63) / 64;
    egm_rhs_kernel<<<ntile, 64 * A.N, 0, st>>>(A);
    AIY_HIP(hipGetLastError());
    egm_interp_kernel<<<(A.N * ntile + 3) / 4, 256, 0, st>>>(A, ntile);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}

}  // namespace aiy
