// A10 (new; the reference has no histogram — SURVEY §8(a) A10) — stationary distribution by
// histogram iteration:  λ'(m,k) = Σ_i P(i,m) · mass(i,k),  mass(i,k) = Σ_{j→k} λ(i,j).
//
// Scatter-free transpose-gather.  The policy maps j to a destination key k(j) (the grid index
// for a VFI policy; the bracket of a' for an off-grid EGM policy, whose mass is split between
// k and k+1 as a lottery).  Optimal policies are monotone in j (increasing differences,
// Topkis), so each key's preimage is ONE contiguous run of j, and the runs of consecutive keys
// are adjacent: the whole policy is a CSR offset row per productivity state,
// off(i,k) = #{j : k(i,j) < k}.
//   prepare (once per policy)  keys, lottery weights, offsets (binary search of the key row),
//                              flags: non-monotone keys, index out of range.
//   push (one launch per push) a workgroup owns 64 destinations k and all N states: wave i
//                              gathers mass(i,k) from its run(s) (no atomics), LDS, then wave
//                              m projects λ'(m,k) = Σ_i P(i,m)·mass(i,k) in i order and folds
//                              max|λ'−λ| into the diff slots.
// The terms of a destination are summed in the order dist.hpp defines (ascending j, chunks of
// kDistChunk): runs of ≤ 32 terms are summed by their own lane; a longer run is split over the
// wave, one chunk per lane, and its chunk sums are folded in order — so the borrowing-
// constraint run does not serialise a lane for hundreds of dependent additions.
// N > 16 (more states than one workgroup's waves): one thread per (i,k) sums its run(s) from
// global memory, then a projection launch — same additions, two launches per push.
// Fallback (non-monotone policy): one thread per (i,k) scans the row in order, same chunking.
#include "aiy_common.hpp"
#include "dispatch.hpp"
#include "dist.hpp"

#include <algorithm>

namespace aiy {

__global__ void dist_keys_kernel(DistArgs A) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= A.N * A.Na) return;
    const int Na = A.Na;
    int key;
    if (A.lottery) {
        double x = A.kp[t];
        const double a0 = A.a[0], an = A.a[Na - 1];
        x = x < a0 ? a0 : x;
        x = x > an ? an : x;
        key = seg_of_dev(A.a, Na, x);
        A.wr[t] = (x - A.a[key]) / (A.a[key + 1] - A.a[key]);
    } else {
        key = A.idx[t];
        if (key < 0 || key >= Na) {
            atomicOr(A.flags, 2u);  // invalid index
            key = key < 0 ? 0 : Na - 1;
        }
    }
    A.key[t] = key;
}

// off(i,k) for k = 0..Na (lower bound of k in the key row) + the monotonicity check
__global__ void dist_offsets_kernel(DistArgs A) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int Na = A.Na, W = Na + 1;
    if (t >= A.N * W) return;
    const int i = t / W, k = t - i * W;
    const int* __restrict__ row = A.key + (size_t)i * Na;
    if (k >= 1 && k < Na && row[k - 1] > row[k]) atomicOr(A.flags, 1u);
    int lo = 0, hi = Na;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (row[mid] < k) lo = mid + 1;
        else hi = mid;
    }
    A.off[t] = lo;
}

// term of source j for a destination whose lottery run of the node below ends at js; the
// source arrays are indexed from `base` (0 for the global rows, the wave's first source for
// its LDS copy)
template <bool LOT>
__device__ __forceinline__ double dist_term(const double* __restrict__ lam,
                                            const double* __restrict__ wr, int j, int js,
                                            int base) {
    if (!LOT) return lam[j - base];
    const double w = wr[j - base];
    return j < js ? lam[j - base] * w : lam[j - base] * (1 - w);
}

// sequential sum of the terms of sources [b, e) (e − b ≤ kDistChunk), 8 loads in flight
template <bool LOT>
__device__ __forceinline__ double dist_chunk(const double* __restrict__ lam,
                                             const double* __restrict__ wr, int b, int e,
                                             int js, int base) {
    double part = 0.0;
    for (int t0 = b; __ballot(t0 < e) != 0ull; t0 += 8) {  // wave-uniform trip count
        double x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            x[u] = (t0 + u < e) ? dist_term<LOT>(lam, wr, t0 + u, js, base) : 0.0;
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (t0 + u < e) part = part + x[u];
    }
    return part;
}

// a destination's mass from its run(s) [jb, je) in the A10 order: short runs by the lane's own
// sequential sum (== the chunked sum for L <= G); long runs one at a time, lane c summing
// chunks c, c + 64, ... and the chunk sums folded in chunk order with wave-uniform reads
template <bool LOT>
__device__ __forceinline__ double dist_mass(const double* __restrict__ lam,
                                            const double* __restrict__ wr, int jb, int js,
                                            int je, int base) {
    const int lane = threadIdx.x & 63;
    const int L = je - jb;
    constexpr int G = kDistChunk;
    double tot = dist_chunk<LOT>(lam, wr, jb, L <= G ? je : jb, js, base);
    unsigned long long lm = __ballot(L > G);
    while (lm) {
        const int q = __builtin_ctzll(lm);
        lm &= lm - 1;
        const int qb = readlane_i(jb, q), qs = readlane_i(js, q), qL = readlane_i(L, q);
        const int nch = (qL + G - 1) / G;
        double total = 0.0;
        for (int c0 = 0; c0 < nch; c0 += 64) {
            const int c = c0 + lane;
            const int b = qb + c * G;
            const int e = c < nch ? min(b + G, qb + qL) : b;
            const double part = dist_chunk<LOT>(lam, wr, b, e, qs, base);
            const int nc = min(64, nch - c0);
            for (int u = 0; u < nc; ++u) total = total + readlane_d(part, u);
        }
        if (lane == q) tot = total;
    }
    return tot;
}

// the same sums for a wave whose sources [rb, re) are staged in LDS (re − rb <= kDistStage):
// the long runs' chunks are summed all at once — the wave's chunk c goes to lane c (every long
// run has more than G terms, so at most kDistStage/G + kDistStage/(G+1) <= 64 chunks: one
// pass) — and each long run's chunk sums are folded in chunk order.  The chunk → run map and
// the folds walk the (few) long-run lanes in scalar loops: readlane/v_cndmask, no LDS.
template <bool LOT>
__device__ __forceinline__ double dist_mass_staged(const double* __restrict__ lam,
                                                   const double* __restrict__ wr, int jb,
                                                   int js, int je, int base) {
    const int lane = threadIdx.x & 63;
    const int L = je - jb;
    constexpr int G = kDistChunk;
    static_assert(kDistStage / G + kDistStage / (G + 1) <= 64, "long-run chunks exceed a wave");
    double tot = dist_chunk<LOT>(lam, wr, jb, L <= G ? je : jb, js, base);
    const unsigned long long lm = __ballot(L > G);
    if (lm == 0ull) return tot;
    // chunk lane c: the run q it belongs to, that run's bounds and its chunk index
    int cb = 0, qb = 0, qs = 0, qL = 0, qc = 0;
    for (unsigned long long m = lm; m; m &= m - 1) {
        const int q = __builtin_ctzll(m);
        const int nq = (readlane_i(L, q) + G - 1) / G;
        if (lane >= cb && lane < cb + nq) {
            qb = readlane_i(jb, q);
            qs = readlane_i(js, q);
            qL = readlane_i(L, q);
            qc = cb;
        }
        cb += nq;  // wave-uniform: the chunks so far
    }
    const int b = qb + (lane - qc) * G;
    const int e = lane < cb ? min(b + G, qb + qL) : b;
    const double part = dist_chunk<LOT>(lam, wr, b, e, qs, base);
    // folds in chunk order, one long run after another
    int c0 = 0;
    for (unsigned long long m = lm; m; m &= m - 1) {
        const int q = __builtin_ctzll(m);
        const int nq = (readlane_i(L, q) + G - 1) / G;
        double total = 0.0;
        for (int u = 0; u < nq; ++u) total = total + readlane_d(part, c0 + u);
        if (lane == q) tot = total;
        c0 += nq;
    }
    return tot;
}

// One push: a workgroup owns 64 destinations k and all N states.  The sources of a wave's 64
// destinations are one contiguous range [rb, re) of row i (runs of consecutive keys are
// adjacent), so the wave first copies λ (and the lottery weights) of that range into LDS with
// coalesced loads — all in flight at once — and every lane then sums its run from LDS: one
// global round trip per wave instead of one per 8 terms of the longest run.  A range longer than
// kDistStage (a degenerate policy piling many sources on few keys) is summed from global
// memory as before (A.stage, set at launch: ≤ kDistStage within a 64 KB staging budget);
// the additions and their order are the same either way.
template <bool LOT>
__global__ __launch_bounds__(1024) void dist_push_kernel(DistArgs A) {
    __shared__ double s_mass[kDistPushMaxN][64];
    extern __shared__ double s_src[];  // [N][stage] λ, then [N][stage] weights (LOT)
    const int lane = threadIdx.x & 63;
    const int i = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // blockDim = 64·N
    // every kernel argument in one batch of scalar loads (otherwise fetched in dependent rounds)
    asm volatile("" ::"s"(A.N), "s"(A.Na), "s"(A.P), "s"(A.lam), "s"(A.off), "s"(A.wr),
                 "s"(A.out), "s"(A.diff), "s"(A.stage), "s"(A.diff_clear), "s"(A.trace));
    const int N = A.N, Na = A.Na;
    const int k0 = blockIdx.x * 64, k = k0 + lane;
    double pm[kDistPushMaxN];  // column m = i of P (the projection's weights), loads first
#pragma unroll
    for (int q = 0; q < kDistPushMaxN; ++q) pm[q] = q < N ? A.P[q * N + i] : 0.0;
    const bool ok = k < Na;
    // (instrumentation) shader-cycle stamps of the phases of this wave
    long long cy[6] = {0, 0, 0, 0, 0, 0};
    const long long t_in = A.trace ? (long long)wall_clock64() : 0;
    if (A.trace) cy[0] = (long long)__builtin_amdgcn_s_memtime();
    if (blockIdx.x == 0 && A.diff_clear)  // the next push's slots (a different set)
        for (int q = threadIdx.x; q < 2 * kDiffSlots; q += blockDim.x) A.diff_clear[q] = 0ull;
    const int* __restrict__ off = A.off + (size_t)i * (Na + 1);
    const double* __restrict__ lam = A.lam + (size_t)i * Na;
    const double* __restrict__ wr = LOT ? A.wr + (size_t)i * Na : nullptr;
    int jb = 0, js = 0, je = 0;
    if (ok) {
        js = off[k];
        je = off[k + 1];
        jb = (LOT && k > 0) ? off[k - 1] : js;
    }
    const int last = min(63, Na - 1 - k0);
    const int rb = readlane_i(jb, 0), re = readlane_i(je, last);
    const int S = re - rb;  // wave-uniform
    if (A.trace) cy[1] = (long long)__builtin_amdgcn_s_memtime();
    double tot;
    if (S <= A.stage) {
        double* sl = s_src + (size_t)i * A.stage;
        double* sw = s_src + (size_t)(N + i) * A.stage;
        // every load in flight at once: the loads under a wave-uniform guard (clamped
        // addresses), the LDS writes after them (a load and its store in one guarded block
        // would wait for each load in turn)
        const int nu = (S + 63) >> 6;
        double vl[kDistStage / 64], vw[kDistStage / 64];
#pragma unroll
        for (int u = 0; u < kDistStage / 64; ++u) {
            const int x = rb + min(u * 64 + lane, S - 1);
            vl[u] = u < nu ? lam[x] : 0.0;
            vw[u] = (LOT && u < nu) ? wr[x] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < kDistStage / 64; ++u) {
            const int x = u * 64 + lane;
            if (x < S) {
                sl[x] = vl[u];
                if (LOT) sw[x] = vw[u];
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        if (A.trace) cy[2] = (long long)__builtin_amdgcn_s_memtime();
        tot = dist_mass_staged<LOT>(sl, sw, jb, js, je, rb);
    } else {
        if (A.trace) cy[2] = (long long)__builtin_amdgcn_s_memtime();
        tot = dist_mass<LOT>(lam, wr, jb, js, je, 0);
    }
    s_mass[i][lane] = tot;
    if (A.trace) cy[3] = (long long)__builtin_amdgcn_s_memtime();
    __syncthreads();
    const int m = i;
    double d = 0.0;
    bool okd = false;
    if (ok) {
        double acc = 0.0;
        double ms[kDistPushMaxN];  // all LDS reads in flight before the ordered sum
#pragma unroll
        for (int q = 0; q < kDistPushMaxN; ++q) ms[q] = q < N ? s_mass[q][lane] : 0.0;
#pragma unroll
        for (int q = 0; q < kDistPushMaxN; ++q)
            if (q < N) acc = acc + pm[q] * ms[q];
        const size_t t = (size_t)m * Na + k;
        A.out[t] = acc;
        d = fabs(acc - A.lam[t]);
        okd = (d == d);
    }
    if (A.trace) cy[4] = (long long)__builtin_amdgcn_s_memtime();
    block_max_to_slots(okd, d, A.diff);
    if (A.trace && lane == 0) {
        cy[5] = (long long)__builtin_amdgcn_s_memtime();
        long long* tr = A.trace + 16 * ((size_t)blockIdx.x * N + i);
        tr[0] = t_in;
        tr[1] = (long long)wall_clock64();
        tr[2] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));  // HW_REG_XCC_ID
        tr[3] = S;
        tr[4] = __popcll(__ballot(je - jb > kDistChunk));
        for (int p = 1; p < 6; ++p) tr[4 + p] = cy[p] - cy[p - 1];  // off, stage, mass, proj, out
    }
}

// exact fallback for non-monotone policies: every j of the row, in order, chunked as above
__global__ void dist_gather_scan_kernel(DistArgs A) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= A.N * A.Na) return;
    const int Na = A.Na;
    const int i = t / Na, k = t - i * Na;
    const int* __restrict__ key = A.key + (size_t)i * Na;
    const double* __restrict__ lam = A.lam + (size_t)i * Na;
    const double* __restrict__ wr = A.lottery ? A.wr + (size_t)i * Na : nullptr;
    double total = 0.0, part = 0.0;
    int n = 0;
    for (int j = 0; j < Na; ++j) {
        const int q = key[j];
        double x;
        if (q == k) x = A.lottery ? lam[j] * (1 - wr[j]) : lam[j];
        else if (A.lottery && q + 1 == k) x = lam[j] * wr[j];
        else continue;
        part = part + x;
        if (++n == kDistChunk) {
            total = total + part;
            part = 0.0;
            n = 0;
        }
    }
    if (n) total = total + part;
    A.mass[t] = total;
}

// monotone plan with N > 16 (more states than the push workgroup's 16 waves): one thread per
// destination (i,k) sums its run(s) [jb, je) from global memory in the A10 order (ascending j,
// chunks of kDistChunk, chunk sums in order — the same additions as dist_mass), into A.mass;
// dist_project_kernel then forms λ' for any N.
template <bool LOT>
__global__ void dist_gather_runs_kernel(DistArgs A) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= A.N * A.Na) return;
    const int Na = A.Na;
    const int i = t / Na, k = t - i * Na;
    const int* __restrict__ off = A.off + (size_t)i * (Na + 1);
    const double* __restrict__ lam = A.lam + (size_t)i * Na;
    const double* __restrict__ wr = LOT ? A.wr + (size_t)i * Na : nullptr;
    const int js = off[k], je = off[k + 1];
    const int jb = (LOT && k > 0) ? off[k - 1] : js;
    double total = 0.0, part = 0.0;
    int n = 0;
    for (int j = jb; j < je; ++j) {
        part = part + dist_term<LOT>(lam, wr, j, js, 0);
        if (++n == kDistChunk) {
            total = total + part;
            part = 0.0;
            n = 0;
        }
    }
    if (n) total = total + part;
    A.mass[t] = total;
}

__global__ void dist_project_kernel(DistArgs A) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    bool ok = false;
    double d = 0.0;
    if (t < A.N * A.Na) {
        const int N = A.N, Na = A.Na;
        const int m = t / Na, k = t - m * Na;
        double acc = 0.0;
        for (int i = 0; i < N; ++i) acc = acc + A.P[i * N + m] * A.mass[(size_t)i * Na + k];
        A.out[t] = acc;
        d = fabs(acc - A.lam[t]);
        ok = (d == d);
    }
    block_max_to_slots(ok, d, A.diff);
}

// K = Σ_i Σ_j λ(i,j)·a_j: fixed-order block sums (deterministic), folded by one block
__global__ void dist_capital_kernel(const double* __restrict__ lam, const double* __restrict__ a,
                                    int N, int Na, double* __restrict__ part) {
    __shared__ double sh[256];
    double acc = 0.0;
    const int n = N * Na;
    for (int t = blockIdx.x * 256 + threadIdx.x; t < n; t += gridDim.x * 256)
        acc = acc + lam[t] * a[t % Na];
    sh[threadIdx.x] = acc;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) sh[threadIdx.x] = sh[threadIdx.x] + sh[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = sh[0];
}
__global__ void fold_kernel(const double* __restrict__ part, int n, double* __restrict__ out) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        double acc = 0.0;
        for (int q = 0; q < n; ++q) acc = acc + part[q];
        out[0] = acc;
    }
}

int launch_dist_prepare(const DistArgs& A, hipStream_t st) {
    const int n = A.N * A.Na, nw = A.N * (A.Na + 1);
    dist_keys_kernel<<<(n + 255) / 256, 256, 0, st>>>(A);
    dist_offsets_kernel<<<(nw + 255) / 256, 256, 0, st>>>(A);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}

int launch_dist_push(const DistArgs& A, bool fallback, hipStream_t st) {
    if (A.N < 1) return fail(AIY_BAD_SHAPE, "histogram kernels need N >= 1");
    const int n = A.N * A.Na;
    if (!fallback && A.N > kDistPushMaxN) {  // general N: run gather + projection
        const int g = (n + 255) / 256;
        if (A.lottery) dist_gather_runs_kernel<true><<<g, 256, 0, st>>>(A);
        else dist_gather_runs_kernel<false><<<g, 256, 0, st>>>(A);
        dist_project_kernel<<<g, 256, 0, st>>>(A);
    } else if (!fallback) {
        const int g = (A.Na + 63) / 64;
        // staging budget 64 KB per workgroup (two resident per CU beside s_mass)
        const int per = A.N * (A.lottery ? 16 : 8);
        DistArgs B = A;
        B.stage = std::min(kDistStage, (65536 / per) & ~63);
        const size_t lds = (size_t)B.stage * per;
        if (A.lottery) launch_dispatch_timed(dist_push_kernel<true>, dim3(g), dim3(64 * A.N), lds, st, B);
        else launch_dispatch_timed(dist_push_kernel<false>, dim3(g), dim3(64 * A.N), lds, st, B);
    } else {
        const int g = (n + 255) / 256;
        dist_gather_scan_kernel<<<g, 256, 0, st>>>(A);
        dist_project_kernel<<<g, 256, 0, st>>>(A);
    }
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}

int launch_dist_capital(const double* lam, const double* a, int N, int Na, double* part,
                        double* out, hipStream_t st) {
    constexpr int kBlocks = 256;
    dist_capital_kernel<<<kBlocks, 256, 0, st>>>(lam, a, N, Na, part);
    fold_kernel<<<1, 64, 0, st>>>(part, kBlocks, out);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}

}  // namespace aiy
