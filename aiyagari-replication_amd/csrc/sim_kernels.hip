// A9 — Monte-Carlo capital supply (Aiyagari_VFI.m:104-129; GE copy :174-193; the same block
// in the three other Aiyagari scripts).  The chain is serial by construction: each step needs
// the previous (z, k).  One wavefront runs it; its 64 lanes cooperate on the two searches of
// every step:
//   z_t = find(rand < cumsum(P(z_{t-1},:)), 1)      lanes m < N compare, ballot, first bit
//   k_t = interp1(a_grid, policy_k(z_t,:), k_{t-1}, 'linear', 'extrap')
//        segment = largest i with a_i <= k_{t-1} (clamped to the end segments), found by a
//        64-ary search: a window of 64 grid points per round, ballot + popcount.
// a_grid and the policy rows are staged in LDS when they fit (Na·(N+1) <= 18432 doubles),
// otherwise read through L1/L2.
// Uniform draws come from the host (MATLAB's rand stream), so the chain is reproducible.
#include <atomic>
#include <algorithm>

#include "aiy_common.hpp"
#include "sim.hpp"

namespace aiy {

constexpr int kSimLdsMax = 18432;  // doubles: 147 KiB of the 160 KiB LDS

template <bool LDS>
__global__ __launch_bounds__(64) void sim_capital_kernel(SimArgs A0) {
    SimArgs A = A0;
    if (A0.C > 1) {  // batched chains: one workgroup per candidate
        A.pol += blockIdx.x * A0.pcs;
        A.U += blockIdx.x * A0.ucs;
        A.out += blockIdx.x;
        A.status += blockIdx.x;
    }
    extern __shared__ double lds[];
    const int lane = threadIdx.x;
    const int N = A.N, Na = A.Na;
    const double* a = A.a;
    const double* pol = A.pol;
    size_t zs = A.zs, as = A.as;
    if constexpr (LDS) {
        for (int k = lane; k < Na; k += 64) lds[k] = A.a[k];
        for (int q = lane; q < N * Na; q += 64) {
            int zz = q / Na, kk = q - zz * Na;
            lds[Na + q] = A.pol[(size_t)zz * A.zs + (size_t)kk * A.as];
        }
        __syncthreads();
        a = lds;
        pol = lds + Na;
        zs = Na;
        as = 1;
    }
    // cumulative transition rows, sequential sums as cumsum does
    __shared__ double cs[16 * 16];
    if (lane == 0) {
        for (int z = 0; z < N; ++z) {
            double acc = 0.0;
            for (int m = 0; m < N; ++m) {
                acc = acc + A.P[z * N + m];
                cs[z * N + m] = acc;
            }
        }
    }
    __syncthreads();
    int z = A.z1;
    double k = A.k1;
    double sum = k;
    if (lane == 0) {
        if (A.sim_k) A.sim_k[0] = k;
        if (A.sim_z) A.sim_z[0] = z;
    }
    int status = 0;
    for (int t = 1; t < A.T; ++t) {
        const double u = A.U[t - 1];
        // ---- state transition
        bool lt = lane < N && u < cs[z * N + lane];
        unsigned long long m = __ballot(lt);
        if (m == 0) {
            status = 1;  // the reference's find() would return empty and error
            break;
        }
        z = __ffsll((long long)m) - 1;
        // ---- segment of k in a_grid: largest i with a[i] <= k, clamped to [0, Na-2]
        int lo = 0, hi = Na;  // invariant: a[lo..] ... answer in [lo-1, hi-1]
        while (hi - lo > 64) {
            int step = (hi - lo + 63) / 64;
            int p = lo + lane * step;
            bool le = p < hi && a[p] <= k;
            int c = __popcll(__ballot(le));
            if (c == 0) {
                hi = lo;
                break;
            }
            lo = lo + (c - 1) * step;
            hi = min(lo + step, hi);
        }
        int cnt;
        {
            int p = lo + lane;
            bool le = p < hi && a[p] <= k;
            cnt = __popcll(__ballot(le));
        }
        int seg = lo + cnt - 1;
        seg = seg < 0 ? 0 : (seg > Na - 2 ? Na - 2 : seg);
        const double* y = pol + (size_t)z * zs;
        double x0 = a[seg], x1 = a[seg + 1];
        double y0 = y[(size_t)seg * as], y1 = y[(size_t)(seg + 1) * as];
        double tt = (k - x0) / (x1 - x0);
        k = y0 + tt * (y1 - y0);
        sum += k;
        if (lane == 0) {
            if (A.sim_k) A.sim_k[t] = k;
            if (A.sim_z) A.sim_z[t] = z;
        }
    }
    if (lane == 0) {
        A.out[0] = sum / (double)A.T;  // mean(sim_k)
        A.status[0] = status;
    }
}

// ---------------------------------------------------------------------------------------------
// Chain kernel (N <= 15).  The state chain z_t does not depend on k, so it leaves the critical
// path: for a chunk of steps the whole block tabulates each step's transition map
//   F_t = { z -> find(u_t < cumsum(P(z,:)), 1) }   (4 bits per z, 15 = find() empty)
// into LDS, and the serial step becomes z_t = (F_t >> 4 z_{t-1}) & 15 on scalars.  The k step
// reads a 64-point window of a_grid and of the policy row around the previous segment in one
// LDS round; every lane evaluates interp1's formula for its own segment while the ballot
// locates k, and the segment's lane is read back (v_readlane) — the division runs in parallel
// with the search instead of after it.  A window that misses k falls back to the 64-ary search.
// Same operations in the same order as sim_capital_kernel, so the path is bit-identical.
constexpr int kSimChunk = 2048;
constexpr int kSimChainLdsMax = 16384;  // doubles for a_grid + policy rows (+16 KB F, 2 KB cs)

__device__ __forceinline__ unsigned long long readlane_u64(unsigned long long v, int l) {
    unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, l);
    unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), l);
    return ((unsigned long long)hi << 32) | lo;
}

template <bool LDS, bool PATH>
__global__ __launch_bounds__(256) void sim_chain_kernel(SimArgs A0) {
    SimArgs A = A0;
    if (A0.C > 1) {  // batched chains: one workgroup per candidate
        A.pol += blockIdx.x * A0.pcs;
        A.U += blockIdx.x * A0.ucs;
        A.out += blockIdx.x;
        A.status += blockIdx.x;
    }
    extern __shared__ double lds[];
    __shared__ unsigned long long F[kSimChunk];
    __shared__ double cs[16 * 16];
    __shared__ int stop_flag;
    const int tid = threadIdx.x, lane = tid & 63;
    // wave-uniform for the compiler too: the chain's control flow and indices stay scalar
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int N = A.N, Na = A.Na;
    const double* a = A.a;
    const double* pol = A.pol;
    size_t zs = A.zs, as = A.as;
    if constexpr (LDS) {
        // rows padded by 64 so a window [w0, w0 + 64] never needs clamping (w0 <= Na - 64, or
        // 0 when Na < 64): the pads are read only by lanes that are never selected
        const int S = Na + 64;
        for (int k = tid; k < S; k += 256) lds[k] = A.a[min(k, Na - 1)];
        for (int q = tid; q < N * S; q += 256) {
            int zz = q / S, kk = q - zz * S;
            lds[S + q] = kk < Na ? A.pol[(size_t)zz * A.zs + (size_t)kk * A.as] : 0.0;
        }
        a = lds;
        pol = lds + S;
        zs = S;
        as = 1;
    }
    if (tid == 0) {  // cumulative transition rows, sequential sums as cumsum does
        for (int z = 0; z < N; ++z) {
            double acc = 0.0;
            for (int m = 0; m < N; ++m) {
                acc = acc + A.P[z * N + m];
                cs[z * N + m] = acc;
            }
        }
        stop_flag = 0;
    }
    __syncthreads();
    const int wmax = Na > 64 ? Na - 64 : 0;
    int z = A.z1;
    double k = A.k1;
    double sum = k;
    int w0 = 0;
    int status = 0;
    double kbuf = k;  // lane (t & 63) holds sim_k(t) until its block of 64 is stored
    int zbuf = z;
    int t_last = 0;
    auto flush = [&](int t) {
        const int base = t & ~63;
        if (PATH && base + lane <= t) {
            if (A.sim_k) A.sim_k[base + lane] = kbuf;
            if (A.sim_z) A.sim_z[base + lane] = zbuf;
        }
    };
    for (int c0 = 1; c0 < A.T; c0 += kSimChunk) {
        const int cn = min(kSimChunk, A.T - c0);
        for (int q = tid; q < cn; q += 256) {
            const double u = A.U[c0 + q - 1];
            unsigned long long f = 0;
            for (int zz = 0; zz < N; ++zz) {
                int m = 15;
                for (int mm = N - 1; mm >= 0; --mm)
                    if (u < cs[zz * N + mm]) m = mm;
                f |= (unsigned long long)m << (4 * zz);
            }
            F[q] = f;
        }
        __syncthreads();
        if (wave == 0) {
            unsigned long long Fv = 0;
            for (int i = 0; i < cn; ++i) {
                const int t = c0 + i;
                if ((i & 63) == 0) Fv = (i + lane < cn) ? F[i + lane] : 0ull;
                const unsigned long long f = readlane_u64(Fv, i & 63);
                const int zn = (int)((f >> (4 * z)) & 15ull);
                if (zn == 15) {  // the reference's find() would return empty and error
                    status = 1;
                    break;
                }
                z = zn;
                const double* y = pol + (size_t)z * zs;
                // ---- window round: every lane evaluates its own segment (indices clamped so
                // the loads need no exec masking; lanes past the grid are never selected)
                const int p = w0 + lane;
                const int p0 = LDS ? p : min(p, Na - 1), p1 = LDS ? p + 1 : min(p + 1, Na - 1);
                const double x0 = a[p0], x1 = a[p1];
                const double y0 = y[(size_t)p0 * as], y1 = y[(size_t)p1 * as];
                const int cnt = __popcll(__ballot(p < Na && x0 <= k));
                const double tt = (k - x0) / (x1 - x0);
                const double kn = y0 + tt * (y1 - y0);
                const int wend = min(w0 + 64, Na);
                int seg = w0 + cnt - 1;
                seg = seg < 0 ? 0 : (seg > Na - 2 ? Na - 2 : seg);
                const int sl = min(max(seg - w0, 0), 63);
                const double kw = readlane_d(kn, sl);  // issued before the rare fallback test
                if ((cnt > 0 || w0 == 0) && (w0 + cnt < wend || wend == Na)) {
                    k = kw;
                } else {  // window missed: largest i with a[i] <= k by 64-ary search
                    int lo = 0, hi = Na;
                    while (hi - lo > 64) {
                        int step = (hi - lo + 63) / 64;
                        int pp = lo + lane * step;
                        bool le = pp < hi && a[pp] <= k;
                        int c = __popcll(__ballot(le));
                        if (c == 0) {
                            hi = lo;
                            break;
                        }
                        lo = lo + (c - 1) * step;
                        hi = min(lo + step, hi);
                    }
                    int pp = lo + lane;
                    int c = __popcll(__ballot(pp < hi && a[pp] <= k));
                    seg = lo + c - 1;
                    seg = seg < 0 ? 0 : (seg > Na - 2 ? Na - 2 : seg);
                    double X0 = a[seg], X1 = a[seg + 1];
                    double Y0 = y[(size_t)seg * as], Y1 = y[(size_t)(seg + 1) * as];
                    double T0 = (k - X0) / (X1 - X0);
                    k = Y0 + T0 * (Y1 - Y0);
                }
                w0 = seg - 31;
                w0 = w0 < 0 ? 0 : (w0 > wmax ? wmax : w0);
                sum += k;
                if constexpr (PATH) {  // the path is only kept when sim_k / sim_z are asked for
                    if (lane == (t & 63)) {
                        kbuf = k;
                        zbuf = z;
                    }
                    t_last = t;
                    if ((t & 63) == 63) flush(t);
                }
            }
            if (status && lane == 0) stop_flag = 1;
        }
        __syncthreads();
        if (stop_flag) break;
    }
    if (wave == 0) {
        if (PATH && (t_last & 63) != 63) flush(t_last);
        if (lane == 0) {
            A.out[0] = sum / (double)A.T;  // mean(sim_k)
            A.status[0] = status;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// A chain's workgroup asks for at least this much LDS so that no other workgroup that uses LDS
// (a solve's sweep blocks in the GE driver) shares its CU: a co-resident block competes with
// the chain's serial wave for issue slots and becomes the straggler of its sweep
// (tools/ge_concurrency.py: 2 solves + 2 chains on shared CUs ran the solves 2.7x slower).
constexpr int kSimExclusiveLds = 88 * 1024;

// Two-wave pipeline (N <= 8, 64 <= Na, Na + 64 <= SS).  One wave running the whole step is
// bound by its instruction issue (~4 cycles per instruction; ~100 per step, half of them scalar
// bookkeeping of the state chain and the window), so the k-independent half moves to a second
// wave: wave 1 walks the state chain z_t = find(u_t < cumsum(P(z_{t-1},:)), 1) one chunk ahead
// (lane 8z + m holds cumsum(P(z,:))(m): one ballot per step) and leaves per step the byte offset
// of row z_t's policy record; wave 0 runs only the k recurrence, ~56 instructions per step:
//   * tables at fixed strides (SS doubles): X0 = a_i (clamped), H = a_{i+1} - a_i, and per row
//     {y_i, y_{i+1} - y_i} — the same subtractions, so t = (k - a_i) / h and k' = y_i + t·dy
//     are sim_chain_kernel's values; one address + immediate offsets per window load;
//   * the window of step t+1 (w0 from step t's segment, row from z_{t+1}) is loaded while step t
//     divides; 32-step unrolled blocks read z offsets with constant lane indices;
//   * every exception (window miss -> 64-ary search) is one branch not taken on the common path.
// w0 stays in [0, Na - 64], so no lane reads past the grid.  A9 chain at Na = 400: 2.54 ->
// 1.58 ms per 10^4 steps, bit-identical (profiles/r05_g30_sim_chain_pipe_ab.txt; the
// reciprocal-table quotient of fastdiv_check.c measured slower, r05_g31).
template <int SS, bool PATH>
__global__ __launch_bounds__(128) void sim_chain_pipe_kernel(SimArgs A0) {
    SimArgs A = A0;
    if (A0.C > 1) {
        A.pol += blockIdx.x * A0.pcs;
        A.U += blockIdx.x * A0.ucs;
        A.out += blockIdx.x;
        A.status += blockIdx.x;
    }
    extern __shared__ double lds[];  // X0[SS] | H[SS] | Y[N][SS][2] = {y_i, y_{i+1} - y_i}
    __shared__ int zoff[2][kSimChunk];
    __shared__ int stop_at;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int N = A.N, Na = A.Na, T = A.T;
    double* X0 = lds;
    double* H = lds + SS;
    double* Y = lds + 2 * SS;
    for (int i = tid; i < SS; i += 128) {
        const double x0 = A.a[min(i, Na - 1)], x1 = A.a[min(i + 1, Na - 1)];
        X0[i] = x0;
        H[i] = x1 - x0;
    }
    for (int q = tid; q < N * SS; q += 128) {
        const int zz = q / SS, i = q - zz * SS;
        const double* row = A.pol + (size_t)zz * A.zs;
        const double y0 = i < Na ? row[(size_t)i * A.as] : 0.0;
        const double y1 = i + 1 < Na ? row[(size_t)(i + 1) * A.as] : 0.0;
        Y[2 * (size_t)q] = y0;
        Y[2 * (size_t)q + 1] = y1 - y0;
    }
    if (tid == 0) stop_at = T;
    // wave 1: lane 8z + m holds cumsum(P(z,:))(m) (sequential sums, as cumsum), -inf elsewhere
    double csl = -__builtin_inf();
    if (wave == 1 && (lane >> 3) < N && (lane & 7) < N) {
        const int zz = lane >> 3, m = lane & 7;
        double acc = 0.0;
        for (int q = 0; q <= m; ++q) acc = acc + A.P[zz * N + q];
        csl = acc;
    }
    int zc = A.z1;
    bool walking = true;
    // steps c0 .. c0 + cn - 1 of the state chain -> out[i] = byte offset of row z_{c0+i} in Y
    auto walk = [&](int c0, int cn, int* out) {
        for (int i0 = 0; i0 < cn && walking; i0 += 64) {
            const double Uv = i0 + lane < cn ? A.U[c0 + i0 + lane - 1] : 0.0;
            int ov = 0;
            const int jn = min(64, cn - i0);
            for (int j = 0; j < jn; ++j) {
                const double u = readlane_d(Uv, j);
                const unsigned row = (unsigned)(__ballot(u < csl) >> (8 * zc)) & 0xFFu;
                if (row == 0) {  // the reference's find() would return empty and error
                    if (lane == 0) stop_at = c0 + i0 + j;
                    walking = false;
                    break;
                }
                zc = __builtin_ctz(row);
                if (lane == j) ov = zc * (SS * 16);
            }
            if (i0 + lane < cn) out[i0 + lane] = ov;
        }
    };
    if (wave == 1 && T > 1) walk(1, min(kSimChunk, T - 1), zoff[0]);
    __syncthreads();
    const int wmax = Na - 64;
    double k = A.k1;
    double sum = k;
    int w0 = 0;
    int status = 0;
    double kbuf = k;
    int zbuf = A.z1;
    int t_last = 0;
    double x0 = 0.0, h = 0.0, y0 = 0.0, dy = 0.0;
    bool primed = false;
    auto ldwin = [&](int w, int zo) {
        const int p = w + lane;
        x0 = X0[p];
        h = H[p];
        const double2 yy = *reinterpret_cast<const double2*>(
            reinterpret_cast<const char*>(Y) + zo + 16 * p);
        y0 = yy.x;
        dy = yy.y;
    };
    auto step = [&](int t, int zo, int zo1) __attribute__((always_inline)) {
        if (__builtin_expect(!primed, 0)) {
            ldwin(w0, zo);
            primed = true;
        }
        const int c = __popcll(__ballot(x0 <= k));
        int sl = min(c - 1, Na - 2 - w0);
        sl = sl < 0 ? 0 : sl;
        int seg = w0 + sl;
        const int hit = ((c > 0) | (w0 == 0)) & ((c < 64) | (w0 == wmax));
        int w0n = seg - 31;
        w0n = w0n < 0 ? 0 : (w0n > wmax ? wmax : w0n);
        const double d = k - x0;
        const double ch = h, cy0 = y0, cdy = dy;
        ldwin(w0n, zo1);  // step t+1's window, issued before this step's division
        __builtin_amdgcn_sched_barrier(0);
        const double kn = cy0 + (d / ch) * cdy;
        const double kw = readlane_d(kn, sl);
        if (__builtin_expect(!hit, 0)) {  // the window missed k: 64-ary search
            int lo = 0, hi = Na;
            while (hi - lo > 64) {
                int stp = (hi - lo + 63) / 64;
                int pp = lo + lane * stp;
                bool le = pp < hi && X0[pp] <= k;
                int cc = __popcll(__ballot(le));
                if (cc == 0) {
                    hi = lo;
                    break;
                }
                lo = lo + (cc - 1) * stp;
                hi = min(lo + stp, hi);
            }
            int pp = lo + lane;
            int cc = __popcll(__ballot(pp < hi && X0[pp] <= k));
            seg = lo + cc - 1;
            seg = seg < 0 ? 0 : (seg > Na - 2 ? Na - 2 : seg);
            w0n = seg - 31;
            w0n = w0n < 0 ? 0 : (w0n > wmax ? wmax : w0n);
            primed = false;
            const double T0 = (k - X0[seg]) / H[seg];
            const double* Yz = reinterpret_cast<const double*>(
                reinterpret_cast<const char*>(Y) + zo) + 2 * seg;
            k = Yz[0] + T0 * Yz[1];
        } else {
            k = kw;
        }
        w0 = w0n;
        sum += k;
        if constexpr (PATH) {
            if (lane == (t & 63)) {
                kbuf = k;
                zbuf = zo / (SS * 16);
            }
            t_last = t;
            if ((t & 63) == 63) {
                const int base = t & ~63;
                if (A.sim_k) A.sim_k[base + lane] = kbuf;
                if (A.sim_z) A.sim_z[base + lane] = zbuf;
            }
        }
    };
    int b = 0;
    for (int c0 = 1; c0 < T; c0 += kSimChunk, b ^= 1) {
        const int cn = min(kSimChunk, T - c0);
        const int lim = min(cn, stop_at - c0);  // steps of this chunk before a find() failure
        if (wave == 1 && walking && c0 + cn < T)
            walk(c0 + cn, min(kSimChunk, T - c0 - cn), zoff[b ^ 1]);
        if (wave == 0) {
            const int* zb = zoff[b];
            int i = 0;
            for (; i + 64 <= lim; i += 64) {
                const int Zv = zb[i + lane];
                const int Zn = i + 64 + lane < lim ? zb[i + 64 + lane] : 0;
#pragma unroll
                for (int j = 0; j < 32; ++j)
                    step(c0 + i + j, __builtin_amdgcn_readlane(Zv, j),
                         __builtin_amdgcn_readlane(Zv, j + 1));
#pragma unroll
                for (int j = 32; j < 64; ++j)
                    step(c0 + i + j, __builtin_amdgcn_readlane(Zv, j),
                         j < 63 ? __builtin_amdgcn_readlane(Zv, j + 1)
                                : __builtin_amdgcn_readlane(Zn, 0));
            }
            if (i < lim) {
                const int Zv = zb[i + lane];
                const int Zn = i + 64 + lane < lim ? zb[i + 64 + lane] : 0;
                for (int j = 0; i + j < lim; ++j)
                    step(c0 + i + j, __builtin_amdgcn_readlane(Zv, j),
                         j < 63 ? __builtin_amdgcn_readlane(Zv, j + 1)
                                : __builtin_amdgcn_readlane(Zn, 0));
            }
            primed = false;  // the last prefetch read a placeholder row
            if (lim < cn) status = 1;
        }
        __syncthreads();
        if (lim < cn) break;
    }
    if (wave == 0) {
        if (PATH && T > 1 && (t_last & 63) != 63) {
            const int base = t_last & ~63;
            if (base + lane <= t_last) {
                if (A.sim_k) A.sim_k[base + lane] = kbuf;
                if (A.sim_z) A.sim_z[base + lane] = zbuf;
            }
        }
        if (PATH && T == 1 && lane == 0) {
            if (A.sim_k) A.sim_k[0] = k;
            if (A.sim_z) A.sim_z[0] = zbuf;
        }
        if (lane == 0) {
            A.out[0] = sum / (double)A.T;
            A.status[0] = status;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Speculative segments (round 6).  The chain is serial, but its two recurrences forget where
// they started: z_t = find(u_t < cumsum(P(z_{t-1},:)), 1) is a composition of maps of a set of
// N states, and k_t = interp1(a, policy_k(z_t,:), k_{t-1}) contracts — two paths driven by the
// same shocks become bit-identical after a few dozen steps (Aiyagari_VFI.m's policy at r = 0.04:
// at most ~210 steps from any start, tools/sim_coalesce.py) and stay identical.  So, in ONE
// workgroup of 16 waves:
//   Z. every thread builds the step maps of its share of t (3 bits per state, 7 = find() empty,
//      absorbing), the block scans their compositions (a Hillis-Steele scan of composed maps),
//      and each thread applies its prefix to z1 and walks its share: z_t for all t, in LDS, and
//      the first empty find() (the chain stops there, as the serial kernel does);
//   K. wave s runs segment s of the k chain, steps [1 + sL, 1 + (s+1)L), from k1 (s = 0) or a
//      guess (k1), with the serial kernel's step (64-lane window, the same operations), storing
//      the path; then repair passes: wave s restarts from the (true) last value of segment s-1
//      and steps until its value equals the stored one bit for bit — from there the stored
//      path is the true one — or overwrites its whole segment; a segment is true once its
//      predecessor was true when its pass started, or became true in the same pass without
//      changing its last value.  Passes repeat until every segment is true (at most 15; one
//      in practice);
//   S. wave 0 sums the path in order (the serial kernel's fp64 accumulation, bit for bit).
// The path, hence K_s, is the serial chain's bit for bit whatever the guesses: every stored
// value is either computed from the true predecessor or equal to such a value.
// (timing probes, results wrong: AIY_PAR_PROBE 1 = no in-order sum, 2 = no repair passes,
// 3 = neither and no segment phase; built only into experiment libraries, never the default)
#ifndef AIY_PAR_PROBE
#define AIY_PAR_PROBE 0
#endif
constexpr int kParWaves = 16;
constexpr int kParMaxT = 16384;  // z_t in LDS (one byte each)

// k_t = interp1(a_grid, policy_k(z_t,:), k_{t-1}) by one wave, the window of sim_chain_pipe_kernel
template <int SS>
struct ParStepper {
    const double* X0;
    const double* H;
    const double* Y;
    int Na, wmax, lane, w0;
    bool primed;
    double x0, h, y0, dy;
    __device__ __forceinline__ void ldwin(int w, int zo) {
        const int p = w + lane;
        x0 = X0[p];
        h = H[p];
        const double2 yy = *reinterpret_cast<const double2*>(reinterpret_cast<const char*>(Y) + zo + 16 * p);
        y0 = yy.x;
        dy = yy.y;
    }
    // zo: byte offset of row z_t in Y; zo1: of row z_{t+1} (its window is loaded under the division)
    __device__ __forceinline__ double step(double k, int zo, int zo1) {
        if (__builtin_expect(!primed, 0)) {
            ldwin(w0, zo);
            primed = true;
        }
        const int c = __popcll(__ballot(x0 <= k));
        int sl = min(c - 1, Na - 2 - w0);
        sl = sl < 0 ? 0 : sl;
        int seg = w0 + sl;
        const int hit = ((c > 0) | (w0 == 0)) & ((c < 64) | (w0 == wmax));
        int w0n = seg - 31;
        w0n = w0n < 0 ? 0 : (w0n > wmax ? wmax : w0n);
        const double d = k - x0;
        const double ch = h, cy0 = y0, cdy = dy;
        ldwin(w0n, zo1);
        __builtin_amdgcn_sched_barrier(0);
        const double kn = cy0 + (d / ch) * cdy;
        double kw = readlane_d(kn, sl);
        if (__builtin_expect(!hit, 0)) {  // the window missed k: 64-ary search
            int lo = 0, hi = Na;
            while (hi - lo > 64) {
                int stp = (hi - lo + 63) / 64;
                int pp = lo + lane * stp;
                bool le = pp < hi && X0[pp] <= k;
                int cc = __popcll(__ballot(le));
                if (cc == 0) {
                    hi = lo;
                    break;
                }
                lo = lo + (cc - 1) * stp;
                hi = min(lo + stp, hi);
            }
            int pp = lo + lane;
            int cc = __popcll(__ballot(pp < hi && X0[pp] <= k));
            seg = lo + cc - 1;
            seg = seg < 0 ? 0 : (seg > Na - 2 ? Na - 2 : seg);
            w0n = seg - 31;
            w0n = w0n < 0 ? 0 : (w0n > wmax ? wmax : w0n);
            primed = false;
            const double T0 = (k - X0[seg]) / H[seg];
            const double* Yz = reinterpret_cast<const double*>(reinterpret_cast<const char*>(Y) + zo) + 2 * seg;
            kw = Yz[0] + T0 * Yz[1];
        }
        w0 = w0n;
        return kw;
    }
};

__device__ __forceinline__ unsigned zmap_compose(unsigned A, unsigned B) {  // A, then B
    unsigned R = 0;
#pragma unroll
    for (int z = 0; z < 8; ++z) R |= ((B >> (3 * ((A >> (3 * z)) & 7u))) & 7u) << (3 * z);
    return R;
}

// the chain's LDS tables (X0[SS] | H[SS] | Y[N][SS][2] = {y_i, y_{i+1} - y_i}), by nthr threads;
// eight elements' loads in flight per thread before their stores (a small workgroup would
// otherwise pay one memory round trip per element)
template <int SS>
__device__ __forceinline__ void par_tables(const SimArgs& A, double* lds, int tid, int nthr) {
    double* X0 = lds;
    double* H = lds + SS;
    double* Y = lds + 2 * SS;
    const int Na = A.Na;
    for (int i = tid; i < SS; i += nthr) {
        const double x0 = A.a[min(i, Na - 1)], x1 = A.a[min(i + 1, Na - 1)];
        X0[i] = x0;
        H[i] = x1 - x0;
    }
    const int nq = A.N * SS;
    for (int q0 = tid; q0 < nq; q0 += 8 * nthr) {
        double y0[8], y1[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int q = q0 + u * nthr;
            const int zz = q / SS, i = q - zz * SS;
            const double* row = A.pol + (size_t)zz * A.zs;
            const bool ok = q < nq;
            y0[u] = ok && i < Na ? row[(size_t)i * A.as] : 0.0;
            y1[u] = ok && i + 1 < Na ? row[(size_t)(i + 1) * A.as] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int q = q0 + u * nthr;
            if (q < nq) {
                Y[2 * (size_t)q] = y0[u];
                Y[2 * (size_t)q + 1] = y1[u] - y0[u];
            }
        }
    }
}

// Z: the state path of one chain by 1,024 threads into zp[0 .. T) (LDS); returns the stop index
// Te (steps 1 .. Te-1 run; Te < T: find() empty at step Te).  Ends with a barrier.
__device__ __forceinline__ int par_zpath(const SimArgs& A, unsigned char* zp, unsigned* s_map,
                                         double* s_cs, int* s_stop) {
    const int tid = threadIdx.x, N = A.N, T = A.T;
    if (tid < 64) {  // cumsum(P(z,:))(m) in order (as cumsum), lanes 8z + m
        const int zz = tid >> 3, m = tid & 7;
        double acc = 0.0;
        if (zz < N && m < N)
            for (int q = 0; q <= m; ++q) acc = acc + A.P[zz * N + q];
        s_cs[tid] = acc;
    }
    if (tid == 0) *s_stop = T;
    __syncthreads();
    const int nst = T - 1;               // steps 1 .. T-1 use u[t - 1]
    const int ch = (nst + 1023) / 1024;  // steps per thread (<= 16: T <= kParMaxT)
    const int t0 = 1 + tid * ch, t1 = min(T, t0 + ch);
    constexpr int kCh = (kParMaxT + 1022) / 1024;
    double ub[kCh];  // this thread's draws, all loads in flight together (both passes use them)
#pragma unroll
    for (int j = 0; j < kCh; ++j) ub[j] = t0 + j < t1 ? A.U[t0 + j - 1] : 0.0;
    auto zmap = [&](int t) __attribute__((always_inline)) -> unsigned {
        const double u = ub[t - t0];
        unsigned M = 7u << 21;  // entry 7 -> 7 (absorbing "find() empty")
#pragma unroll
        for (int z = 0; z < 7; ++z) {
            int e = 7;
#pragma unroll
            for (int m = 7; m >= 0; --m)
                if (z < N && m < N && u < s_cs[8 * z + m]) e = m;  // the first m with u < cumsum
            M |= (unsigned)e << (3 * z);
        }
        return M;
    };
    unsigned agg = 0;
#pragma unroll
    for (int z = 0; z < 8; ++z) agg |= (unsigned)z << (3 * z);  // identity
    const unsigned ident = agg;
#pragma unroll
    for (int j = 0; j < kCh; ++j)
        if (t0 + j < t1) agg = zmap_compose(agg, zmap(t0 + j));
    s_map[tid] = agg;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {  // inclusive scan of the compositions
        const unsigned prev = tid >= off ? s_map[tid - off] : ident;
        __syncthreads();
        if (tid >= off) s_map[tid] = zmap_compose(prev, s_map[tid]);
        __syncthreads();
    }
    const unsigned pre = tid > 0 ? s_map[tid - 1] : ident;
    int z = (int)((pre >> (3 * A.z1)) & 7u);
    int first_bad = T;
#pragma unroll
    for (int j = 0; j < kCh; ++j) {
        const int t = t0 + j;
        if (t < t1) {
            z = (int)((zmap(t) >> (3 * z)) & 7u);
            zp[t] = (unsigned char)z;
            if (z == 7 && first_bad == T) first_bad = t;
        }
    }
    if (first_bad < T) atomicMin(s_stop, first_bad);
    if (tid == 0) zp[0] = (unsigned char)A.z1;
    __syncthreads();
    return *s_stop;
}

// one wave: segment [Ts, Tn) of the k recurrence from k into kp — each step's value parked in
// lane (t − cb) of a register, 64 of them stored together (no per-step store or exec change)
template <int SS, class ZO>
__device__ __forceinline__ void par_segment(ParStepper<SS>& ps, double k, int Ts, int Tn,
                                            const ZO& zo_of, double* kp, int lane) {
    if (AIY_PAR_PROBE == 3) return;
    double buf = 0.0;
    int cb = Ts;
    for (int t = Ts; t < Tn; ++t) {
        k = ps.step(k, zo_of(t), zo_of(t + 1));
        buf = lane == t - cb ? k : buf;
        if (t - cb == 63) {
            kp[cb + lane] = buf;
            cb += 64;
        }
    }
    if (cb < Tn && lane < Tn - cb) kp[cb + lane] = buf;
}

// one wave: repair segment [Ts, Tn) from k (its predecessor's end): step until the value equals
// the stored one bit for bit (from there the stored path is the true one) or overwrite the whole
// segment; returns 1 when the segment's last value changed.  The stored values are read in
// chunks of 64 (one per lane, the next chunk in flight) and read back with v_readlane: no
// dependent global load per step.
template <int SS, class ZO>
__device__ __forceinline__ int par_repair(ParStepper<SS>& ps, double k, int Ts, int Tn,
                                          const ZO& zo_of, double* kp, int lane) {
    ps.primed = false;
    int cb = Ts, chg = 0, t = Ts;
    double sv = Ts + lane < Tn ? kp[Ts + lane] : 0.0;
    double sn = Ts + 64 + lane < Tn ? kp[Ts + 64 + lane] : 0.0;
    double buf = 0.0;  // the rewritten values of chunk cb, one per lane, stored together
    for (; t < Tn; ++t) {
        if (t - cb == 64) {
            kp[cb + lane] = buf;  // the chunk before: every step of it was rewritten
            cb = t;
            sv = sn;
            sn = cb + 64 + lane < Tn ? kp[cb + 64 + lane] : 0.0;
        }
        k = ps.step(k, zo_of(t), zo_of(t + 1));
        const unsigned long long kb = __builtin_bit_cast(unsigned long long, k);
        const unsigned long long sb =
            __builtin_bit_cast(unsigned long long, readlane_d(sv, t - cb));
        if (kb == sb) break;  // the stored path is the true one from here
        buf = lane == t - cb ? k : buf;
        if (t == Tn - 1) chg = 1;
    }
    if (lane < t - cb) kp[cb + lane] = buf;  // the rewritten part of the last chunk
    return chg;
}

// segment s of a chain stopping at Te: steps [Ts, Tn)
__device__ __forceinline__ void par_seg_range(int Te, int s, int& Ts, int& Tn) {
    const int L = (Te - 1 + kParWaves - 1) / kParWaves;  // >= 0
    Ts = 1 + s * L;
    Tn = min(Te, Ts + L);
}

// a segment is true once its predecessor was true when the pass started, or became true in the
// same pass without changing its last value (one thread)
__device__ __forceinline__ void par_resolve(int* res, const int* chg) {
    int prev_old = res[0], prev_new = 1;
    for (int q = 1; q < kParWaves; ++q) {
        const int old = res[q];
        const int nw = old || prev_old || (prev_new && !chg[q - 1]);
        prev_old = old;
        prev_new = nw;
        res[q] = nw;
    }
}

// repair passes until every segment is true (16 waves, zp and the tables in LDS), then the mean
// (wave 0: the sequential fp64 sum k_0 .. k_{Te-1}) and the outputs.  s_res holds the segments'
// state on entry.
template <int SS, class ZO>
__device__ __forceinline__ void par_passes_sum(const SimArgs& A, ParStepper<SS>& ps,
                                               const ZO& zo_of, double* kp, int Te, int* s_res,
                                               int* s_chg, int* s_go) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int Ts, Tn;
    par_seg_range(Te, wave, Ts, Tn);
    for (;;) {
        if (tid == 0) {
            int go = 0;
            for (int q = 0; q < kParWaves; ++q) go |= !s_res[q];
            *s_go = go;
        }
        __syncthreads();
        if (!*s_go) break;
        const bool mine = !s_res[wave];
        const double k = mine ? kp[Ts - 1] : 0.0;  // every start read before any repair writes
        __syncthreads();
        const int chg = mine ? par_repair(ps, k, Ts, Tn, zo_of, kp, lane) : 0;
        if (lane == 0) s_chg[wave] = chg;
        __syncthreads();
        if (tid == 0) par_resolve(s_res, s_chg);
        __syncthreads();
    }
    if (wave == 0 && (AIY_PAR_PROBE == 0 || AIY_PAR_PROBE == 2)) {
        double v = lane < Te ? kp[lane] : 0.0;
        double sum = readlane_d(v, 0);  // sum = k_1 (the serial kernel's start), then in order
        for (int c0 = 0; c0 < Te; c0 += 64) {
            const double vn = c0 + 64 + lane < Te ? kp[c0 + 64 + lane] : 0.0;
            const int n = min(64, Te - c0);
            if (n == 64 && c0 > 0) {
                // 16 values read back per group into distinct registers before their adds, the
                // next group's while these add: the dependent adds wait only on each other
                double x[16], y[16];
#pragma unroll
                for (int j = 0; j < 16; ++j) x[j] = readlane_d(v, j);
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    if (g < 3) {
#pragma unroll
                        for (int j = 0; j < 16; ++j) y[j] = readlane_d(v, 16 * (g + 1) + j);
                    }
#pragma unroll
                    for (int j = 0; j < 16; ++j) sum = sum + x[j];
#pragma unroll
                    for (int j = 0; j < 16; ++j) x[j] = y[j];
                }
            } else {
                for (int j = c0 == 0 ? 1 : 0; j < n; ++j) sum = sum + readlane_d(v, j);
            }
            v = vn;
        }
        if (lane == 0) {
            A.out[0] = sum / (double)A.T;
            A.status[0] = Te < A.T ? 1 : 0;
        }
    }
}

// chain blockIdx.x / per of a batch: its policy, uniforms, outputs and path scratch
__device__ __forceinline__ SimArgs par_chain(const SimArgs& A0, int c, double** kp) {
    SimArgs A = A0;
    *kp = A0.kscr;
    if (A0.C > 1) {
        A.pol += c * A0.pcs;
        A.U += c * A0.ucs;
        A.out += c;
        A.status += c;
        *kp += (size_t)c * A0.T;
    }
    if (A.sim_k) *kp = A.sim_k;  // the path is the output itself (C = 1)
    return A;
}
// the spread variant's scratch after the k paths: state paths [C][T] bytes, then per chain
// {Te, chg[kParWaves]} ints
__device__ __forceinline__ unsigned char* par_zg(const SimArgs& A0, int c) {
    return reinterpret_cast<unsigned char*>(A0.kscr + (size_t)max(A0.C, 1) * A0.T) + (size_t)c * A0.T;
}
__device__ __forceinline__ int* par_ig(const SimArgs& A0, int c) {
    const size_t zb = ((size_t)max(A0.C, 1) * A0.T + 7) & ~(size_t)7;
    return reinterpret_cast<int*>(reinterpret_cast<unsigned char*>(A0.kscr + (size_t)max(A0.C, 1) * A0.T) + zb) +
           (size_t)c * (1 + kParWaves);
}

template <int SS, bool PATH>
__global__ __launch_bounds__(1024) void sim_chain_par_kernel(SimArgs A0) {
    double* kp;
    const SimArgs A = par_chain(A0, blockIdx.x, &kp);
    extern __shared__ double lds[];
    __shared__ unsigned char zp[kParMaxT];
    __shared__ unsigned s_map[1024];
    __shared__ double s_cs[64];
    __shared__ int s_stop, s_go;
    __shared__ int s_res[kParWaves], s_chg[kParWaves];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    par_tables<SS>(A, lds, tid, 1024);
    const int Te = par_zpath(A, zp, s_map, s_cs, &s_stop);  // (its barriers cover the tables)
    const int zrow = SS * 16;
    auto zo_of = [&](int t) __attribute__((always_inline)) { return t < Te ? (int)zp[t] * zrow : 0; };
    int Ts, Tn;
    par_seg_range(Te, wave, Ts, Tn);
    ParStepper<SS> ps{lds, lds + SS, lds + 2 * SS, A.Na, A.Na - 64, lane, 0, false, 0.0, 0.0, 0.0, 0.0};
    if (Ts < Tn) par_segment(ps, A.k1, Ts, Tn, zo_of, kp, lane);
    if (tid == 0) kp[0] = A.k1;
    if (lane == 0) {
        s_res[wave] = wave == 0 || AIY_PAR_PROBE >= 2 ? 1 : (Ts < Tn ? 0 : 1);  // (empty: true)
        s_chg[wave] = 0;
    }
    __syncthreads();
    par_passes_sum(A, ps, zo_of, kp, Te, s_res, s_chg, &s_go);
    if (PATH && A.sim_z)
        for (int t = tid; t < Te; t += 1024) A.sim_z[t] = zp[t];
}

// The spread variant (round 6): the same computation in four launches, so that the 16 segments
// run on 16 CUs (one wave per SIMD) instead of sharing one CU's four SIMDs (four waves each:
// 571 vs 158 ns per step, profiles/r06_g23_sim_par_phases.txt).  Launch 1 (one 1,024-thread
// workgroup per chain): the state path and Te into the scratch.  Launch 2 (16 one-wave
// workgroups per chain): each its segment from the guess.  Launch 3 (same): repair pass 1 of
// every segment s >= 1 from its predecessor's stored end — that end may be rewritten by the
// predecessor's own repair meanwhile, but a start is then only trusted when the predecessor's
// end did not change (par_resolve), so either value read is safe.  Launch 4 (one workgroup per
// chain): the segments' state after pass 1, further passes in one CU if any is still untrusted
// (rare), then the in-order sum.  Same values as sim_chain_par_kernel bit for bit.
template <bool PATH>
__global__ __launch_bounds__(1024) void sim_par_z_kernel(SimArgs A0) {
    double* kp;
    const SimArgs A = par_chain(A0, blockIdx.x, &kp);
    __shared__ unsigned char zp[kParMaxT];
    __shared__ unsigned s_map[1024];
    __shared__ double s_cs[64];
    __shared__ int s_stop;
    const int tid = threadIdx.x;
    const int Te = par_zpath(A, zp, s_map, s_cs, &s_stop);
    unsigned char* zg = par_zg(A0, blockIdx.x);
    for (int t = tid; t < A.T; t += 1024) zg[t] = zp[t];
    if (tid == 0) {
        par_ig(A0, blockIdx.x)[0] = Te;
        kp[0] = A.k1;
    }
    if (PATH && A.sim_z)
        for (int t = tid; t < Te; t += 1024) A.sim_z[t] = zp[t];
}

constexpr int kParSlice = kParMaxT / kParWaves + 2;  // a segment's states [Ts, Tn]
// (256 threads: four waves stage the tables, then wave 0 alone runs the segment)
constexpr int kParSegThreads = 256;
template <int SS, bool FIX>
__global__ __launch_bounds__(kParSegThreads) void sim_par_seg_kernel(SimArgs A0) {
    const int c = blockIdx.x / kParWaves, s = blockIdx.x % kParWaves;
    const int tid = threadIdx.x, lane = tid & 63;
    double* kp;
    const SimArgs A = par_chain(A0, c, &kp);
    int* ig = par_ig(A0, c);
    if (FIX && s == 0) {
        if (tid == 0) ig[1] = 0;
        return;
    }
    const int Te = ig[0];
    int Ts, Tn;
    par_seg_range(Te, s, Ts, Tn);
    if (Ts >= Tn) {
        if (FIX && tid == 0) ig[1 + s] = 0;
        return;
    }
    extern __shared__ double lds[];
    __shared__ int zs[kParSlice];  // the segment's row byte offsets (0 past Te)
    const unsigned char* zg = par_zg(A0, c);
    const int zrow = SS * 16;
    for (int t = Ts + tid; t <= Tn; t += kParSegThreads) zs[t - Ts] = t < Te ? (int)zg[t] * zrow : 0;
    par_tables<SS>(A, lds, tid, kParSegThreads);
    __syncthreads();
    if (tid >= 64) return;
    auto zo_of = [&](int t) __attribute__((always_inline)) { return zs[t - Ts]; };
    ParStepper<SS> ps{lds, lds + SS, lds + 2 * SS, A.Na, A.Na - 64, lane, 0, false, 0.0, 0.0, 0.0, 0.0};
    if (!FIX) {
        par_segment(ps, A.k1, Ts, Tn, zo_of, kp, lane);
    } else {
        const double k = kp[Ts - 1];
        const int chg = AIY_PAR_PROBE >= 2 ? 0 : par_repair(ps, k, Ts, Tn, zo_of, kp, lane);
        if (lane == 0) ig[1 + s] = chg;
    }
}

template <int SS>
__global__ __launch_bounds__(1024) void sim_par_sum_kernel(SimArgs A0) {
    double* kp;
    const SimArgs A = par_chain(A0, blockIdx.x, &kp);
    const int* ig = par_ig(A0, blockIdx.x);
    extern __shared__ double lds[];
    __shared__ unsigned char zp[kParMaxT];
    __shared__ int s_go, s_all;
    __shared__ int s_res[kParWaves], s_chg[kParWaves];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int Te = ig[0];
    if (tid < kParWaves) {
        int Ts, Tn;
        par_seg_range(Te, tid, Ts, Tn);
        s_res[tid] = tid == 0 || Ts >= Tn ? 1 : 0;  // before pass 1 (launch 3)
        s_chg[tid] = ig[1 + tid];
    }
    __syncthreads();
    if (tid == 0) {
        par_resolve(s_res, s_chg);
        int all = 1;
        for (int q = 0; q < kParWaves; ++q) all &= s_res[q];
        s_all = all;
    }
    __syncthreads();
    const int zrow = SS * 16;
    auto zo_of = [&](int t) __attribute__((always_inline)) { return t < Te ? (int)zp[t] * zrow : 0; };
    ParStepper<SS> ps{lds, lds + SS, lds + 2 * SS, A.Na, A.Na - 64, lane, 0, false, 0.0, 0.0, 0.0, 0.0};
    if (!s_all) {  // (rare) more passes, on this CU: the tables and the state path into LDS
        par_tables<SS>(A, lds, tid, 1024);
        const unsigned char* zg = par_zg(A0, blockIdx.x);
        for (int t = tid; t < A.T; t += 1024) zp[t] = zg[t];
        __syncthreads();
    }
    (void)wave;
    par_passes_sum(A, ps, zo_of, kp, Te, s_res, s_chg, &s_go);
}

// the speculative-segment chain; AIY_BAD_SHAPE when it does not apply.  spread: the four-launch
// variant (16 CUs per chain), else one workgroup per chain
int launch_sim_chain_par(const SimArgs& A, hipStream_t st, bool spread) {
    if (A.N < 1 || A.N > 7 || A.Na < 64 || A.T < 2 || A.T > kParMaxT || !A.kscr)
        return fail(AIY_BAD_SHAPE, "speculative chain: N <= 7, Na >= 64, 2 <= T <= 16384, scratch");
    const int S = A.Na + 64;
    const int SS = S <= 512 ? 512 : (S <= 1024 ? 1024 : 0);
    if (!SS) return fail(AIY_BAD_SHAPE, "speculative chain tables exceed LDS");
    const size_t bytes = sizeof(double) * (size_t)(2 + 2 * A.N) * SS;
    const int g = std::max(A.C, 1);
    const bool path = A.sim_k || A.sim_z;
    // the dynamic-LDS limit is raised once per instantiation, to the most any call asks for
#define AIY_LDS_ONCE(K_, SS_)                                                                      \
    do {                                                                                           \
        static std::atomic<bool> lds_set{false};                                                   \
        if (!lds_set) {                                                                            \
            AIY_HIP(hipFuncSetAttribute((const void*)K_, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                        (int)sizeof(double) * (2 + 2 * 7) * SS_));                 \
            lds_set = true;                                                                        \
        }                                                                                          \
    } while (0)
#define AIY_PAR(SS_, PA_)                                                                          \
    do {                                                                                           \
        if (spread) {                                                                              \
            AIY_LDS_ONCE((sim_par_seg_kernel<SS_, false>), SS_);                                   \
            AIY_LDS_ONCE((sim_par_seg_kernel<SS_, true>), SS_);                                    \
            AIY_LDS_ONCE((sim_par_sum_kernel<SS_>), SS_);                                          \
            sim_par_z_kernel<PA_><<<g, 1024, 0, st>>>(A);                                          \
            sim_par_seg_kernel<SS_, false><<<g * kParWaves, kParSegThreads, bytes, st>>>(A);       \
            sim_par_seg_kernel<SS_, true><<<g * kParWaves, kParSegThreads, bytes, st>>>(A);        \
            sim_par_sum_kernel<SS_><<<g, 1024, bytes, st>>>(A);                                    \
        } else {                                                                                   \
            AIY_LDS_ONCE((sim_chain_par_kernel<SS_, PA_>), SS_);                                   \
            sim_chain_par_kernel<SS_, PA_><<<g, 1024, bytes, st>>>(A);                             \
        }                                                                                          \
    } while (0)
    if (SS == 512) {
        if (path) AIY_PAR(512, true);
        else AIY_PAR(512, false);
    } else {
        if (path) AIY_PAR(1024, true);
        else AIY_PAR(1024, false);
    }
#undef AIY_PAR
#undef AIY_LDS_ONCE
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}

// the two-wave chain; AIY_BAD_SHAPE when it does not apply (N > 8, Na < 64, tables past LDS)
int launch_sim_chain_pipe(const SimArgs& A, hipStream_t st) {
    if (A.N < 1 || A.N > 8 || A.Na < 64) return fail(AIY_BAD_SHAPE, "pipe chain: N <= 8, Na >= 64");
    const int S = A.Na + 64;
    const int SS = S <= 512 ? 512 : (S <= 1024 && A.N <= 7 ? 1024 : 0);
    if (!SS) return fail(AIY_BAD_SHAPE, "pipe chain tables exceed LDS");
    const size_t tables = sizeof(double) * (size_t)(2 + 2 * A.N) * SS;
    const size_t bytes = A.exclusive ? std::max(tables, (size_t)kSimExclusiveLds) : tables;
    const int g = std::max(A.C, 1);
    const bool path = A.sim_k || A.sim_z;
    // the dynamic-LDS limit is raised once per instantiation, to the most any call asks for
#define AIY_PIPE(SS_, PA_)                                                                         \
    do {                                                                                           \
        static std::atomic<bool> lds_set{false};                                                   \
        if (!lds_set) {                                                                            \
            constexpr int most = std::max((int)sizeof(double) * (2 + 2 * (SS_ == 512 ? 8 : 7)) * SS_, \
                                          kSimExclusiveLds);                                       \
            AIY_HIP(hipFuncSetAttribute((const void*)sim_chain_pipe_kernel<SS_, PA_>,              \
                                        hipFuncAttributeMaxDynamicSharedMemorySize, most));        \
            lds_set = true;                                                                        \
        }                                                                                          \
        sim_chain_pipe_kernel<SS_, PA_><<<g, 128, bytes, st>>>(A);                                 \
    } while (0)
    if (SS == 512) {
        if (path) AIY_PIPE(512, true);
        else AIY_PIPE(512, false);
    } else {
        if (path) AIY_PIPE(1024, true);
        else AIY_PIPE(1024, false);
    }
#undef AIY_PIPE
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}

int launch_sim_capital(const SimArgs& A, hipStream_t st) {
    if (A.N > 16 || A.N < 1) return fail(AIY_BAD_SHAPE, "simulation supports 1 <= N <= 16");
    const long long need = (long long)A.Na * (A.N + 1);
    // the speculative-segment chain for the GE loop's long chains (T = 10,000: 1.6 ms serial)
    const bool par_ok = A.kscr && A.N <= 7 && A.Na >= 64 && A.Na + 64 <= 1024 && A.T >= 2 &&
                        A.T <= kParMaxT;
    // (par: -1 by size — the spread variant; 1 one workgroup per chain; 2 the spread variant)
    if (par_ok && (A.par > 0 || (A.par < 0 && A.T >= 2048)))
        return launch_sim_chain_par(A, st, A.par != 1);
    if (A.N <= 8 && A.Na >= 64 && (A.Na + 64 <= 512 || (A.Na + 64 <= 1024 && A.N <= 7)))
        return launch_sim_chain_pipe(A, st);
    if (A.N <= 15) {
        const long long need_pad = (long long)(A.Na + 64) * (A.N + 1);
        const bool path = A.sim_k || A.sim_z;
        const int g = std::max(A.C, 1);
        if (need_pad <= kSimChainLdsMax) {
            const size_t tables = sizeof(double) * (size_t)need_pad;
            const size_t bytes = A.exclusive ? std::max(tables, (size_t)kSimExclusiveLds) : tables;
            static std::atomic<bool> lds_set[2] = {false, false};
            if (!lds_set[path]) {  // once per instantiation, to the most any call asks for
                const void* fn = path ? (const void*)sim_chain_kernel<true, true>
                                      : (const void*)sim_chain_kernel<true, false>;
                const int most = std::max((int)sizeof(double) * kSimChainLdsMax, kSimExclusiveLds);
                AIY_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, most));
                lds_set[path] = true;
            }
            if (path) sim_chain_kernel<true, true><<<g, 256, bytes, st>>>(A);
            else sim_chain_kernel<true, false><<<g, 256, bytes, st>>>(A);
        } else {
            if (path) sim_chain_kernel<false, true><<<g, 256, 0, st>>>(A);
            else sim_chain_kernel<false, false><<<g, 256, 0, st>>>(A);
        }
    } else if (need <= kSimLdsMax) {
        sim_capital_kernel<true><<<std::max(A.C, 1), 64, sizeof(double) * need, st>>>(A);
    } else {
        sim_capital_kernel<false><<<std::max(A.C, 1), 64, 0, st>>>(A);
    }
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}

}  // namespace aiy
