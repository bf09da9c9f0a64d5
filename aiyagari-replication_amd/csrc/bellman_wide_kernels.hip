// A1 / A3 on small grids — the whole Bellman sweep in ONE launch, candidates spread wide.
//   A1: Aiyagari_VFI.m:70-83 (GE copy :152-165)             max over a'
//   A3: Aiyagari_Endogenous_Labor_VFI.m:69-112 (GE :176-219)  max over (l, a') column-major
//
// At the scripts' own grid (Na = 400: configs[0] and the labour script of configs[2]) the tree
// sweep (table launch + one or a few waves per 64-state tile walking a bound tree) is a
// dependent chain of two launches over a few hundred waves: ≈ 15 µs (A1) / 38 µs (A3) for
// 1.1 M / 11 M candidates.  Here a workgroup owns 64 states of one row (one per lane) and a
// slice of the candidate range, split over its NW waves; S workgroups split the range of one
// tile further when the work needs more of the chip (labour):
//   1. the expectation EV(i,k) = Σ_m (β·P(i,m))·V(m,k) and the screening key D(i,k) of the
//      workgroup's candidate slice, computed by its threads into LDS (the table kernel's
//      operations, bit for bit: bell_dev.hpp) — no table launch, no EV array in HBM;
//   2. the bar: every lane evaluates exactly one candidate — the last sweep's argmax (hint),
//      or on a cold sweep a′ = a_1 at the level with the largest feasible prefix;
//   3. each wave screens its candidates, eight at a time per labour level: the bound tree's
//      division-free test t = (D_k − B)·c^n ≥ 1 − 2^-48 (true for every candidate whose exact
//      value reaches the running best: DESIGN.md §5 A1), exact value + (max value, first
//      column-major index) merge for the few that pass;
//   4. the waves' bests meet in LDS; with S > 1 each workgroup publishes its 64 partial bests
//      (sc1 stores, drained) and counts itself in with one agent-scope atomic add per tile;
//      the workgroup whose add completes the tile merges the S partials (sc1 loads) — the
//      counter hand-off of MI355X_MICROARCH.md's inter-workgroup visibility table, row 1;
//   5. outputs: v_new, the linear index, policy_k / policy_l / policy_c and max|v_new − v_old|
//      (the merge kernel's rules), and the previous sweep's diff slots folded (block 0).
// Every candidate that can reach the maximum is evaluated exactly in the literal MATLAB order
// and the merge rule is order-independent, so the result is the exhaustive scan's bit for bit.
#include <hip/hip_runtime.h>

#include "aiy_common.hpp"
#include "bell_dev.hpp"
#include "bellman.hpp"

namespace aiy {

// the previous sweep's slot set: folded into fold[0..1] (reduce_slots_kernel's rule) when asked,
// then cleared for the sweep after this one — one wave of block 0, each lane its own two words
__device__ __forceinline__ void wide_fold_clear(unsigned long long* __restrict__ old,
                                                unsigned long long* __restrict__ fold) {
    const int l = threadIdx.x & 63;
    unsigned long long m = old[2 * l];
    const unsigned long long f = old[2 * l + 1];
    if (fold) {
        const int any = __ballot((f & 1ull) != 0ull) != 0ull;
        m = wave_max_u64_lane63(m);
        const unsigned lo = __builtin_amdgcn_readlane((int)(unsigned)m, 63);
        const unsigned hi = __builtin_amdgcn_readlane((int)(unsigned)(m >> 32), 63);
        if (l == 0) {
            fold[0] = ((unsigned long long)hi << 32) | lo;
            fold[1] = any ? 1ull : 0ull;
        }
    }
    old[2 * l] = 0ull;
    old[2 * l + 1] = 0ull;
}

template <int NP, bool LAB, int NW>
__global__ __launch_bounds__(64 * NW) void bell_wide_kernel(
    BellArgs A, int ntile, int S, int lsb, unsigned long long* __restrict__ old_slots,
    unsigned* __restrict__ cnt, unsigned long long* __restrict__ part, int flags) {
    extern __shared__ double2 s_tab[];  // [Na] (a_k, D_k), then [Na] EV_k, [Na / 8] Dmax8
    __shared__ double s_best[NW][64];
    __shared__ int s_idx[NW][64];
    __shared__ int s_kfl[kWideMaxNl + 1];  // per level: the tile's feasible range; [Nl]: any level
    __shared__ double s_L[kWideMaxNl], s_dis[kWideMaxNl];  // (labour) levels and disutilities
    const int lane = threadIdx.x & 63;
    const int wave = readfirst(threadIdx.x >> 6);
    // every kernel argument the prologue and the bar read, in one batch of scalar loads (left to
    // itself the compiler fetches them in dependent rounds, a wait each, as each use is reached)
    asm volatile("" ::"s"(A.a), "s"(A.P), "s"(A.v_old), "s"(A.kf), "s"(A.hint), "s"(A.s),
                 "s"(A.w), "s"(A.beta), "s"(A.r), "s"(A.N), "s"(A.Na), "s"(A.Nl), "s"(A.sigma),
                 "s"(A.L), "s"(A.dis), "s"(A.trace), "s"(ntile), "s"(S), "s"(lsb), "s"(flags),
                 "s"(old_slots), "s"(A.fold), "s"(A.idx), "s"(A.pk), "s"(A.pc), "s"(A.v_new),
                 "s"(A.diff));
    // (instrumentation, aiy_ws_set_timing bit 2) wave 0's phase marks, one record per block
    const bool TR = A.trace != nullptr;
    long long tr_mark[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // (constant indices only: registers)
    const long long tr_wall0 = TR ? (long long)wall_clock64() : 0;
#define AIY_WMARK(q)                                                            \
    do {                                                                        \
        if (TR) tr_mark[q] = (long long)__builtin_amdgcn_s_memtime();           \
    } while (0)
    AIY_WMARK(0);
    // block → (tile item, split); the S splits of an item have equal blockIdx % 8 (one XCD under
    // round-robin placement: the partials' hand-off stays in one L2 — speed only)
    const int b = blockIdx.x;
    const int item = (b / (8 * S)) * 8 + (b & 7);
    const int sp = (b >> 3) % S;
    const int N = A.N, Na = A.Na, Nl = LAB ? A.Nl : 1;
    if (item >= N * ntile) return;  // block-uniform
    const int tile = item % ntile, i = item / ntile;
    const size_t nall = (size_t)N * Na;
    const double* __restrict__ a = A.a;
    // a wave holds SB = 2^lsb states (lane % SB) × Q = 64 / SB sub-slices of the candidates
    // (lane / SB): small grids get SB < 64 — more workgroups over the chip, no hand-off
    const int SB = 1 << lsb, Q = 64 >> lsb;
    const int ls = lane & (SB - 1), qs = lane >> lsb;
    const int j = tile * SB + ls;
    const bool okj = j < Na;
    const size_t t = (size_t)i * Na + (okj ? j : 0);

    // 0. every independent load at once: this lane's state (a_j, v_old, hint, the feasible
    // prefix of every level) and, by all threads, the row's expectation table
    constexpr int NLM = LAB ? kWideMaxNl : 1;
    int kfr[NLM];
#pragma unroll
    for (int l = 0; l < NLM; ++l) kfr[l] = (okj && l < Nl) ? A.kf[l * nall + t] : 0;
    const double aj = okj ? a[j] : 0.0;
    const double vo = (okj && wave == 0) ? A.v_old[t] : 0.0;
    const int h = (A.hint && okj) ? A.hint[t] : -1;
    const double y = A.w * A.s[i];
    // (labour) the levels and their disutilities, loaded with the rest (stored to LDS below: a
    // load issued after the table's would be a second dependent round trip)
    double lv_pre = 1.0, ds_pre = 0.0;
    if (LAB && threadIdx.x < Nl) {
        lv_pre = A.L[threadIdx.x];
        ds_pre = A.dis[threadIdx.x];
    }
    // 1. EV and D of the whole row into LDS (the table kernel's operations: bell_dev.hpp); no
    // dependence on this tile's feasible prefixes, so its loads leave with the ones above
    // and the maxima of D over aligned 8-candidate blocks (the screen's block bounds: DPP over
    // the eight lanes holding a block, as the table kernel's Dm8)
    double* s_ev = reinterpret_cast<double*>(s_tab + Na);
    double* s_dm8 = s_ev + Na;
    for (int k0 = 0; k0 < Na; k0 += 64 * NW) {  // (uniform trips: every lane in the DPP)
        const int k = k0 + (int)threadIdx.x;
        double D = -__builtin_inf();
        if (k < Na) {
            const double ak = a[k];  // (issued with the V column, not after the sum)
            const double ev = table_ev(N, Na, A.P, A.v_old, A.beta, i, k);
            D = table_D(ev, NP);
            s_tab[k] = make_double2(ak, D);
            s_ev[k] = ev;
        }
        double d8 = fmax(D, dpp_d<0xB1>(D));
        d8 = fmax(d8, dpp_d<0x4E>(d8));
        d8 = fmax(d8, dpp_d<0x104>(d8));
        if (k < Na && (k & 7) == 0) s_dm8[k >> 3] = d8;
    }
    AIY_WMARK(1);  // [1] table issued / written
    const double x = (1 + A.r) * aj;
    int kmx = 0, lwide = 0;
#pragma unroll
    for (int l = 0; l < NLM; ++l)
        if (kfr[l] > kmx) {
            kmx = kfr[l];
            lwide = l;
        }
    const bool anyfeas = kmx > 0;
    if (LAB && threadIdx.x < Nl) {
        s_L[threadIdx.x] = lv_pre;
        s_dis[threadIdx.x] = ds_pre;
    }
    // the tile's feasible range per level (a wave maximum: any sign of 1 + r), level l by wave
    // l mod NW and the widest by the last wave — spread out, not one wave doing all Nl + 1
    // reductions while the others wait at the barrier (≈ 4 k cycles at Nl = 10)
#pragma unroll
    for (int l = 0; l < NLM; ++l)
        if (l < Nl && l % NW == wave) {
            const int m = wave_max_i32_lane63(kfr[l]);
            if (lane == 63) s_kfl[l] = m;
        }
    if (wave == NW - 1) {
        const int km = wave_max_i32_lane63(kmx);
        if (lane == 63) s_kfl[Nl] = km;
    }
    int hl = lwide, hk = 0, kfh = kmx;
    if (h >= 0) {
        const int l = h % Nl;
        int kf = 0;
#pragma unroll
        for (int q = 0; q < NLM; ++q) kf = q == l ? kfr[q] : kf;
        if (kf > 0) {
            hl = l;
            hk = min(h / Nl, kf - 1);
            kfh = kf;
        }
    }
    __syncthreads();
    AIY_WMARK(2);  // [2] table complete (barrier)
    const int kmax = s_kfl[Nl];

    // 2. the bar: the hint (or a_1 at the widest level) and its two neighbours — exact values
    // from the LDS table, merged like any other candidate (a repeated candidate is a no-op
    // under the merge rule); with kWideClimb, then a climb in the improving direction.  Any
    // evaluated candidate is a valid bar: the result does not depend on it.
    double best = __builtin_nan("");
    int idx = -1;
    unsigned nhits = 0;
    if (okj && anyfeas) {
        const double coh = cash<LAB>(x, y, LAB ? s_L[hl] : 1.0);
        const double dis = LAB ? s_dis[hl] : 0.0;
        auto val_at = [&](int k) __attribute__((always_inline)) {
            return bell_val<NP, LAB>(coh - s_tab[k].x, s_ev[k], A.sigma, dis);
        };
        {
            const int k0 = max(hk - 1, 0), k2 = min(hk + 1, kfh - 1);
            const double v0 = val_at(k0), v1 = val_at(hk), v2 = val_at(k2);
            lexi_take(v1, hl + Nl * hk, best, idx);
            lexi_take(v0, hl + Nl * k0, best, idx);
            lexi_take(v2, hl + Nl * k2, best, idx);
            nhits += 3;
        }
        const int kb = idx / Nl;
        const int dir = !(flags & kWideClimb) ? 0 : (kb > hk ? 1 : (kb < hk ? -1 : 0));
        if (dir != 0) {
            int k = kb, step = 2;
            for (;;) {
                const int kn = min(max(k + dir * step, 0), kfh - 1);
                if (kn == k) break;
                ++nhits;
                if (!lexi_take(val_at(kn), hl + Nl * kn, best, idx)) break;
                k = kn;
                step <<= 1;
            }
            for (int s2 = step >> 1; s2 >= 1; s2 >>= 1) {
                const int c0 = idx / Nl;
                if (c0 + s2 < kfh) {
                    ++nhits;
                    lexi_take(val_at(c0 + s2), hl + Nl * (c0 + s2), best, idx);
                }
                if (c0 - s2 >= 0) {
                    ++nhits;
                    lexi_take(val_at(c0 - s2), hl + Nl * (c0 - s2), best, idx);
                }
            }
        }
    }
    AIY_WMARK(3);  // [3] bar

    // 3. the screen: the 8-candidate blocks of [0, kmax) dealt round-robin over the tile's
    // S·NW waves and each wave's Q slices (block g to slice g mod S·NW·Q: the blocks around
    // the tile's optima — the only ones with exact work — spread out), at every level.  First
    // the block's bound, (Dmax8 − B)·max(c_{k0}, 0)^n — c_k <= c_{k0} and D_k <= Dmax8 inside
    // the block, and fp subtraction and multiplication are monotone, so a block whose bound
    // fails holds no candidate that can reach the bar (the tree's 8-block level) — four
    // (level, block) pairs at a time; the candidates of a block only when some lane's bound
    // passes.
    const int gw0 = (sp * NW + wave) * Q, gstride = S * NW * Q;  // (the wave's first slice)
    const int gw = gw0 + qs;                                        // this lane's slice
    unsigned ntests = 0, nvotes = 0, nblk = 0, nrnd = 0;  // (instrumentation)
    // the eight candidates of the lane's block k0 at level l (every lane of the wave runs it)
    auto block = [&](int l, int k0, int kend, double coh, double dis)
                     __attribute__((always_inline)) {
        double B = okj ? screen_B(best, idx, dis, NP) : __builtin_nan("");
        double2 tk[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)  // (every read in range, then the selects: one LDS wait)
            tk[u] = s_tab[min(k0 + u, Na - 1)];
#pragma unroll
        for (int u = 0; u < 8; ++u)  // (past the range: a = +inf, c < 0, the test fails)
            tk[u] = k0 + u < kend ? tk[u] : make_double2(__builtin_inf(), 0.0);
        double cx[8], dd[8], tv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            cx[u] = coh - tk[u].x;
            dd[u] = tk[u].y - B;
        }
        AIY_SCHED_BARRIER();
        screen_t<NP, 8>(tv, cx, dd);
        // the current argmax itself is masked (its value is known)
        const int kidx = idx >= 0 ? idx / Nl : -1;
        const unsigned self = (idx >= 0 && idx - Nl * kidx == l && kidx >= k0 && kidx < k0 + 8)
                                  ? 1u << (kidx - k0) : 0u;
        bool pk[8], pall = false;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            pk[u] = tv[u] >= kThr && !((self >> u) & 1u);
            pall = pall || pk[u];
        }
        ntests += max(0, min(8, kend - k0));
        if (TR) ++nblk;
        if (!__any(pall)) return;
        unsigned vote = 0;
#pragma unroll
        for (int u = 0; u < 8; ++u) vote |= (__any(pk[u]) ? 1u : 0u) << u;
        nvotes += __builtin_popcount(vote);
        if ((flags & (kWideBatch | kWideBatch2)) &&
            __builtin_popcount(vote) >= ((flags & kWideBatch2) ? 2 : 4)) {
            // many voted: all eight exact values as independent chains, then the ordered
            // merges; a candidate outside the feasible prefix (c <= 0) is NaN, as in the
            // reference (any exactly evaluated candidate may be merged)
            double val[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const double c = cx[u] > 0 ? cx[u] : 1.0;
                const double v = bell_val<NP, LAB>(c, s_ev[min(k0 + u, Na - 1)], A.sigma, dis);
                val[u] = (okj && cx[u] > 0) ? v : __builtin_nan("");
            }
            AIY_SCHED_BARRIER();
#pragma unroll
            for (int u = 0; u < 8; ++u) lexi_take_sel(val[u], l + Nl * (k0 + u), best, idx);
            nhits += 8;
            return;
        }
        // the voted candidates one at a time (their exact paths are dependent chains, hidden
        // by the other waves of the SIMD); the bar may have risen since the vote
        while (vote) {
            const int u = __builtin_ctz(vote);
            vote &= vote - 1;
            const int k = min(k0 + u, Na - 1);
            const double2 tkk = s_tab[k];  // (both reads before any use)
            const double evk = s_ev[k];
            const double c = coh - tkk.x;
            const int lin = l + Nl * k;
            if (okj && pk[u] && lin != idx && c > 0 && (tkk.y - B) * aiy_ipow(c, NP) >= kThr) {
                ++nhits;
                const double val = bell_val<NP, LAB>(c, evk, A.sigma, dis);
                if (lexi_take(val, lin, best, idx)) B = screen_B(best, idx, dis, NP);
            }
        }
    };
    const int nbl = (kmax - 8 * gw0 + 8 * gstride - 1) / (8 * gstride);  // (wave-uniform)
    constexpr int VB = 4;
    if (LAB && nbl <= 2) {
        // few blocks per level (small labour grids): the lane's one or two blocks are the same
        // at every level, so their a_{k0} and Dmax8 are read once; per level only the cash and
        // the bar key change (computed once per level, not per (level, block) pair), and the
        // pairs of VL levels are bound-tested together — VL·nbl independent tests per round
        // (round 5: four pairs per round, every operand re-read and recomputed per pair,
        // ≈ 170 VALU per round; profiles/r05_wide_ab.txt)
        constexpr int VL = 5;
        double avb[2], dmb[2];
        int k0b[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            k0b[q] = 8 * (gw + q * gstride);
            const int kc = min(k0b[q], Na - 1);
            avb[q] = s_tab[kc].x;
            dmb[q] = s_dm8[kc >> 3];
        }
        for (int l0 = 0; l0 < Nl; l0 += VL) {
            double Lv[VL], dsv[VL], cohv[VL], Bv[VL], tb[2 * VL], cx[2 * VL], dd[2 * VL];
            int kev[VL];
#pragma unroll
            for (int v = 0; v < VL; ++v) {  // (reads first, clamped: one LDS wait)
                const int l = min(l0 + v, Nl - 1);
                Lv[v] = s_L[l];
                dsv[v] = s_dis[l];
                kev[v] = s_kfl[l];
            }
#pragma unroll
            for (int v = 0; v < VL; ++v) {
                cohv[v] = okj ? cash<LAB>(x, y, Lv[v]) : 0.0;
                Bv[v] = okj ? screen_B(best, idx, dsv[v], NP) : __builtin_nan("");
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const bool okb = l0 + v < Nl && q < nbl && k0b[q] < kev[v];
                    cx[2 * v + q] = okb ? cohv[v] - avb[q] : -1.0;
                    dd[2 * v + q] = okb ? dmb[q] - Bv[v] : __builtin_nan("");
                }
            }
            AIY_SCHED_BARRIER();
            screen_t<NP, 2 * VL>(tb, cx, dd);
            ntests += 2 * VL;  // (bound tests, counted per lane like the candidates)
            if (TR) ++nrnd;
#pragma unroll
            for (int v = 0; v < VL; ++v)
#pragma unroll
                for (int q = 0; q < 2; ++q)
                    if (__any(tb[2 * v + q] >= kThr))
                        block(l0 + v, k0b[q], kev[v], cohv[v], dsv[v]);
        }
    } else {
        // level by level, VB of the lane's blocks bound-tested at a time
        for (int l = 0; l < Nl; ++l) {
            const int kend = s_kfl[l];
            if (kend <= 8 * gw0) continue;
            const double coh = okj ? cash<LAB>(x, y, LAB ? s_L[l] : 1.0) : 0.0;
            const double dis = LAB ? s_dis[l] : 0.0;
            for (int kw = 8 * gw0; kw < kend; kw += VB * 8 * gstride) {  // (wave-uniform trips)
                const double B = okj ? screen_B(best, idx, dis, NP) : __builtin_nan("");
                double cx[VB], dd[VB], tb[VB], av[VB], dmv[VB];
                int k0v[VB];
#pragma unroll
                for (int v = 0; v < VB; ++v) {  // (reads first, clamped: one LDS wait)
                    k0v[v] = kw + v * 8 * gstride + 8 * qs;
                    const int kc = min(k0v[v], Na - 1);
                    av[v] = s_tab[kc].x;
                    dmv[v] = s_dm8[kc >> 3];
                }
#pragma unroll
                for (int v = 0; v < VB; ++v) {
                    const bool okb = k0v[v] < kend;
                    cx[v] = okb ? coh - av[v] : -1.0;
                    dd[v] = okb ? dmv[v] - B : __builtin_nan("");
                }
                AIY_SCHED_BARRIER();
                screen_t<NP, VB>(tb, cx, dd);
                ntests += VB;
                if (TR) ++nrnd;
#pragma unroll
                for (int v = 0; v < VB; ++v)
                    if (__any(tb[v] >= kThr)) block(l, k0v[v], kend, coh, dis);
            }
        }
    }
    AIY_WMARK(4);  // [4] screen (this wave)
    if (TR && lane == 0) {  // every wave's own bar and screen ends (64-word records)
        long long* tr = A.trace + 64 * (size_t)blockIdx.x;
        tr[16 + 2 * wave] = tr_mark[3] - tr_mark[0];
        tr[17 + 2 * wave] = tr_mark[4] - tr_mark[0];
        // its screen's work: bound-test rounds | entered 8-blocks << 16 | voted candidates << 32
        tr[48 + wave] = (long long)nrnd | ((long long)nblk << 16) | ((long long)nvotes << 32);
    }
    if (A.hitcount) {  // instrumentation (aiy_ws_set_timing bit 1): exact evaluations, tests
        unsigned long long* hc = A.hitcount + 4 * (blockIdx.x % kDiffSlots);
        unsigned hh = nhits, nt = ntests;
        for (int off = 32; off > 0; off >>= 1) {
            hh += __shfl_xor(hh, off);
            nt += __shfl_xor(nt, off);
        }
        if (lane == 0) {
            atomicAdd(hc, (unsigned long long)hh);
            atomicAdd(hc + 3, (unsigned long long)nt);
        }
    }

    // 4. the sub-slices' bests (butterfly: every lane of a state ends with the state's), the
    // waves' bests, then (S > 1) the tile's splits
    for (int m = SB; m < 64; m <<= 1) {
        const double ob = __shfl_xor(best, m);
        const int oi = __shfl_xor(idx, m);
        lexi_take(ob, oi, best, idx);
    }
    s_best[wave][lane] = best;
    s_idx[wave][lane] = idx;
    __syncthreads();
    // the previous sweep's slot set (not the one this sweep writes): folded and cleared by wave
    // 1 of block 0 while wave 0 writes the outputs (at the start it held block 0's table loads
    // back by a round trip)
    if (blockIdx.x == 0 && wave == 1 && old_slots) wide_fold_clear(old_slots, A.fold);
    if (wave != 0) return;
    AIY_WMARK(5);  // [5] every wave's screen (barrier)
#pragma unroll
    for (int w = 1; w < NW; ++w) lexi_take(s_best[w][lane], s_idx[w][lane], best, idx);
    auto trace_out = [&](int last) __attribute__((always_inline)) {
        if (!TR || lane != 0) return;
        long long* tr = A.trace + 64 * (size_t)blockIdx.x;
        tr[0] = tr_wall0;
        tr[1] = (long long)wall_clock64();
        tr[2] = (long long)(unsigned)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));
#pragma unroll
        for (int q = 1; q < 8; ++q) tr[2 + q] = tr_mark[q] ? tr_mark[q] - tr_mark[0] : -1;
        tr[10] = nhits;
        tr[11] = ntests;
        tr[12] = nvotes;
        tr[13] = last;
        tr[14] = item;
        tr[15] = (long long)__builtin_amdgcn_s_memtime() - tr_mark[0];
    };
    if (S > 1) {
        unsigned long long* pp = part + 2 * ((size_t)item * S * 64 + lane);
        __hip_atomic_store(pp + 2 * 64 * sp, __builtin_bit_cast(unsigned long long, best),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(pp + 2 * 64 * sp + 1, (unsigned long long)(long long)idx,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // the partials are published by a release RMW on the tile's counter (the
        // fence orders every lane's stores before lane 0's add) and the last arriver acquires
        // before it reads them back — the memory model's order, not the hardware's
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        unsigned prev = 0;
        if (lane == 0)
            prev = __hip_atomic_fetch_add(cnt + item, 1u, __ATOMIC_RELEASE,
                                          __HIP_MEMORY_SCOPE_AGENT);
        prev = (unsigned)readlane_i((int)prev, 0);
        AIY_WMARK(6);  // [6] partials published
        if (prev != (unsigned)(S - 1)) {  // not the last split of this tile
            trace_out(0);
            return;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // every split's partial visible
        if (lane == 0)  // re-armed for the next sweep (read after this launch's boundary)
            __hip_atomic_store(cnt + item, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // every split's partial (own included: a repeat merges as a no-op), all loads in
        // flight together, then the merges (lexi_take_sel: one basic block)
        unsigned long long vb[kWideMaxSplits], ib[kWideMaxSplits];
#pragma unroll
        for (int q = 0; q < kWideMaxSplits; ++q) {
            const int qq = min(q, S - 1);
            vb[q] = __hip_atomic_load(pp + 2 * 64 * qq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ib[q] = __hip_atomic_load(pp + 2 * 64 * qq + 1, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int q = 0; q < kWideMaxSplits; ++q)
            lexi_take_sel(__builtin_bit_cast(double, vb[q]), (int)(long long)ib[q], best, idx);
    }

    // 5. outputs (the merge kernel's rules: Aiyagari_VFI.m:79-81, Labor_VFI.m:85,106-109); a_k
    // comes from the LDS table (the table kernel stores the same a[k])
    bool okd = false;
    double dmax = 0.0;
    if (okj && qs == 0) {
        double bv = best;
        int q = idx;
        if (LAB && !anyfeas) {  // no feasible (l, a'): v_new keeps its value (Labor_VFI.m:85)
            bv = A.keep_incoming ? A.v_new[t] : vo;
        } else {
            if (q < 0) {  // all candidates NaN: max returns NaN at index 1
                q = 0;
                bv = __builtin_nan("");
            }
            const int l = q % Nl, k = q / Nl;
            const double kp = s_tab[k].x;
            A.idx[t] = q;
            if (A.pk) A.pk[t] = kp;
            if (A.pc) A.pc[t] = cash<LAB>(x, y, LAB ? s_L[l] : 1.0) - kp;
            if (LAB && A.pl) A.pl[t] = s_L[l];
        }
        A.v_new[t] = bv;
        const double d = fabs(bv - vo);
        okd = d == d;
        dmax = okd ? d : 0.0;
    }
    wave_max_to_slots(okd, dmax, A.diff);
    AIY_WMARK(7);  // [7] outputs
    trace_out(1);
#undef AIY_WMARK
}

// ------------------------------------------------------------------------------ launcher
template <int NP, bool LAB, int NW>
static void wide_geo(const BellArgs& A, int S, int lsb, unsigned long long* old_slots,
                     unsigned* cnt, unsigned long long* part, int flags, size_t min_lds,
                     hipStream_t st) {
    const int ntile = (A.Na + (1 << lsb) - 1) >> lsb;
    const int items = A.N * ntile;
    const int grid = ((items + 7) / 8) * 8 * S;
    const size_t lds = std::max(bell_wide_lds(A.Na, S, NW), min_lds);
    static bool big = false;  // dynamic LDS past 64 KiB needs the attribute (idempotent)
    if (!big && lds > 64 * 1024) {
        (void)hipFuncSetAttribute((const void*)bell_wide_kernel<NP, LAB, NW>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)kWideMaxLds);
        big = true;
    }
    launch_dispatch_timed(bell_wide_kernel<NP, LAB, NW>, dim3(grid), dim3(64 * NW), lds, st, A,
                          ntile, S, lsb, old_slots, cnt, part, flags);
}
template <int NP, bool LAB>
static void wide_w(const BellArgs& A, int S, int NW, int lsb, unsigned long long* old_slots,
                   unsigned* cnt, unsigned long long* part, int flags, size_t min_lds,
                   hipStream_t st) {
    switch (NW) {
        case 4: wide_geo<NP, LAB, 4>(A, S, lsb, old_slots, cnt, part, flags, min_lds, st); break;
        case 8: wide_geo<NP, LAB, 8>(A, S, lsb, old_slots, cnt, part, flags, min_lds, st); break;
        default: wide_geo<NP, LAB, 16>(A, S, lsb, old_slots, cnt, part, flags, min_lds, st); break;
    }
}

int launch_bell_wide(const BellArgs& A, int S, int NW, int SB, unsigned long long* old_slots,
                     unsigned* cnt, unsigned long long* part, int flags, size_t min_lds,
                     hipStream_t st) {
    if (A.np < 1 || A.np > 8) return fail(AIY_BAD_ARG, "wide sweep needs integer sigma in [2, 9]");
    if (A.C > 1) return fail(AIY_BAD_ARG, "wide sweep: one candidate rate");
    if (S < 1 || S > kWideMaxSplits || (NW != 4 && NW != 8 && NW != 16) ||
        (SB != 8 && SB != 16 && SB != 32 && SB != 64))
        return fail(AIY_BAD_ARG, "wide sweep: S in [1, %d], NW in {4, 8, 16}, SB in {8, ..., 64}",
                    kWideMaxSplits);
    const int lsb = 31 - __builtin_clz((unsigned)SB);
    if (bell_wide_lds(A.Na, S, NW) > kWideMaxLds)
        return fail(AIY_BAD_SHAPE, "wide sweep: the candidate slice does not fit in LDS");
#define AIY_WCASE(n)                                                               \
    case n:                                                                        \
        if (A.labor) wide_w<n, true>(A, S, NW, lsb, old_slots, cnt, part, flags, min_lds, st); \
        else wide_w<n, false>(A, S, NW, lsb, old_slots, cnt, part, flags, min_lds, st);        \
        break;
    switch (A.np) {
        AIY_WCASE(1) AIY_WCASE(2) AIY_WCASE(3) AIY_WCASE(4) AIY_WCASE(5) AIY_WCASE(6)
        AIY_WCASE(7) AIY_WCASE(8)
    }
#undef AIY_WCASE
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}

}  // namespace aiy
