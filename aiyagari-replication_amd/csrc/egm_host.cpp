// A4/A5 entry points: device tier (aiy_egm_step_dev) and MATLAB host tier (aiy_egm_*,
// aiy_labor_egm_*).  policy arrays are Na x N column-major == [N][Na]: no transposes.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <mutex>
#include <vector>

#include "aiy_common.hpp"
#include "egm.hpp"
#include "host_ctx.hpp"
#include "ws.hpp"

namespace aiy {

static int fail_nonmonotone() {
    return fail(AIY_BAD_ARG, "endogenous grid a_hat is not increasing: interp1 in the "
                             "reference would sort it or fail (Aiyagari_EGM.m:95)");
}

// the non-monotone flag of a step from host copies of its diff slots and flag word: bit 0 of
// the word (two-launch step) or bit 1 of a slot's second word (egm_fused_kernel)
static bool egm_nonmonotone(const unsigned long long* slots, unsigned flag_word) {
    if (flag_word & 1u) return true;
    for (int q = 0; q < kDiffSlots; ++q)
        if (slots[2 * q + 1] & 2ull) return true;
    return false;
}

static int ensure_egm(aiy_ws* ws) {
    size_t n = (size_t)ws->N * ws->Na;
    if (!ws->g0) AIY_HIP(hipMalloc((void**)&ws->g0, n * sizeof(double)));
    if (!ws->g1) AIY_HIP(hipMalloc((void**)&ws->g1, n * sizeof(double)));
    if (!ws->gi) AIY_HIP(hipMalloc((void**)&ws->gi, 16 * sizeof(int)));
    if (!ws->diff)
        AIY_HIP(hipMalloc((void**)&ws->diff, 2 * kDiffSlots * sizeof(unsigned long long)));
    if (!ws->hdiff)
        AIY_HIP(hipHostMalloc((void**)&ws->hdiff, (2 * kDiffSlots + 4) * sizeof(unsigned long long)));
    if (ws->tracing) {  // (instrumentation) one record per interp / chain wave: N·ntile
        const int64_t cap = (int64_t)ws->N * ((ws->Na + 15) / 16);
        if (ws->trace_cap < cap) {
            if (ws->trace) (void)hipFree(ws->trace);
            ws->trace = nullptr;
            ws->trace_cap = 0;
            AIY_HIP(hipMalloc((void**)&ws->trace, 16 * (size_t)cap * sizeof(long long)));
            AIY_HIP(hipMemset(ws->trace, 0, 16 * (size_t)cap * sizeof(long long)));
            ws->trace_cap = cap;
        }
    }
    if (!ws->egm_seg) {
        AIY_HIP(hipMalloc((void**)&ws->egm_seg, n * sizeof(int)));
        AIY_HIP(hipMemset(ws->egm_seg, 0xff, n * sizeof(int)));  // -1: no hint yet
    }
    return AIY_OK;
}

static EgmArgs egm_args(aiy_ws* ws, const double* c, const double* a, const double* s,
                        const double* P, double r, double w, double beta, double sigma,
                        double amin, bool labor, double phi, double theta, double* cout,
                        double* pk, double* pl) {
    EgmArgs A{};
    A.N = (int)ws->N;
    A.Na = (int)ws->Na;
    A.labor = labor;
    A.ns = is_int_ge(sigma, 1.0) ? (int)sigma : 0;
    A.r = r; A.w = w; A.beta = beta; A.sigma = sigma; A.amin = amin; A.phi = phi;
    A.theta = theta;
    A.c = c; A.a = a; A.s = s; A.P = P;
    A.ahat = ws->g0; A.cnext = ws->g1; A.cout = cout; A.pk = pk; A.pl = pl;
    A.diff = ws->diff;
    A.flags = (unsigned*)ws->gi;
    A.trace = ws->tracing ? ws->trace : nullptr;  // (instrumentation; see ensure_egm)
    // interp1 segment hints (verified in the kernel; kEgmNoHints turns them off, A/B only)
    A.seg = egm_knob(ws, kEgmNoHints) ? nullptr : ws->egm_seg;
    // small grids: one launch per step (egm_fused_kernel) unless kEgmTwoLaunch; large grids:
    // the two-launch step (the solve loop chains it, egm_solve_spec).  (A one-pass scatter step
    // was measured slower — 35.6 vs 12.1 us at Na = 20,000, DESIGN.md §5 — and removed.)
    A.fused = !egm_knob(ws, kEgmTwoLaunch);
    return A;
}

int egm_step_dev(aiy_ws* ws, const double* c, const double* a, const double* s, const double* P,
                 double r, double w, double beta, double sigma, double amin, bool labor,
                 double phi, double theta, double* cout, double* pk, double* pl, double* diff_out,
                 hipStream_t st) {
    if (!ws || !c || !a || !s || !P || !cout || !pk) return fail(AIY_BAD_ARG, "NULL argument");
    if (labor && !(phi == phi && theta == theta)) return fail(AIY_NON_FINITE, "phi/theta");
    AIY_TRY(ensure_egm(ws));
    EgmArgs A = egm_args(ws, c, a, s, P, r, w, beta, sigma, amin, labor, phi, theta, cout, pk, pl);
    // the two-launch and small-grid steps clear ws->diff and the flag word themselves
    AIY_TRY(ws_timing_begin(ws, st));
    AIY_TRY(launch_egm_step(A, st));
    AIY_TRY(ws_timing_end(ws, st));
    if (diff_out) AIY_TRY(launch_reduce_slots(ws->diff, diff_out, st));
    return AIY_OK;
}

// dist of the last step + the non-monotone-grid flag (synchronises)
static int read_egm(aiy_ws* ws, hipStream_t st, double* d) {
    unsigned long long* h = ws->hdiff;
    AIY_HIP(hipMemcpyAsync(h, ws->diff, 2 * kDiffSlots * sizeof(unsigned long long),
                           hipMemcpyDeviceToHost, st));
    AIY_HIP(hipMemcpyAsync(h + 2 * kDiffSlots, ws->gi, sizeof(int), hipMemcpyDeviceToHost, st));
    AIY_HIP(hipStreamSynchronize(st));
    *d = fold_slots_host(h);
    if (egm_nonmonotone(h, (unsigned)h[2 * kDiffSlots])) return fail_nonmonotone();
    return AIY_OK;
}

// The solve loop (Aiyagari_EGM.m:74-108, labour :67-105) with speculative batches, as the VFI
// solve (capi.cpp, bell_solve_spec): steps are deterministic, so batches of m steps are
// enqueued between reads — step g reads ring slot (g−1) mod R and writes slot g mod R, its
// dist lands in slot set g mod R with its flag word (a chained step zeroes set (g+1) mod R for
// the next step; the other steps clear their own) — and each batch ends with
// one D2H copy of the slot sets and an event.  Two batches are in flight: the host reads batch
// k's dists while batch k+1 runs, so the device never idles at a read; with R = 2M + 1 slots
// the stopping step's policy_c survives the next batch's writes.  Its policy_k (and policy_l)
// were overwritten by later speculative steps, so the stopping step is re-run from its input
// (identical values).  Iteration count, dist and outputs equal the one-read-per-step loop's.
static int egm_solve_spec(aiy_ws* ws, const EgmArgs& A0, double* c0, double tol,
                          int64_t max_iter, double** cur_out, double* dist, int64_t* iters,
                          hipStream_t st) {
    const int M = ws->spec_max, R = 2 * M + 1;
    const size_t n = (size_t)ws->N * ws->Na, nb = n * sizeof(double);
    const int SW = kEgmSlotWords;  // per step: {max bits, any} slots, then the flag word
    const size_t SB = (size_t)R * SW * sizeof(unsigned long long);
    if (ws->egm_spec_n != n || ws->egm_spec_m != M) {
        ws->free_egm_spec();
        AIY_HIP(hipMalloc((void**)&ws->egm_ring, (size_t)R * nb));
        AIY_HIP(hipMalloc((void**)&ws->egm_slots, SB));
        AIY_HIP(hipHostMalloc((void**)&ws->egm_hslots, 2 * SB));
        for (int b = 0; b < 2; ++b)
            AIY_HIP(hipEventCreateWithFlags(&ws->egm_ev[b], hipEventDisableTiming));
        ws->egm_spec_n = n;
        ws->egm_spec_m = M;
    }
    auto slot = [&](int64_t g) { return ws->egm_ring + (size_t)(g % R) * n; };
    auto sset = [&](int64_t g) { return ws->egm_slots + (size_t)(g % R) * SW; };
    AIY_HIP(hipMemcpyAsync(slot(0), c0, nb, hipMemcpyDeviceToDevice, st));
    // chained steps (the default for Na > 1,024): the RHS of step 1 here, then one launch per
    // step — interp1 of step g on â/c̃ pair (g−1) & 1, the RHS of step g+1 into pair g & 1
    const bool chain = !(A0.fused && A0.Na <= kEgmFusedMaxNa) && !egm_knob(ws, kEgmNoChain);
    if (chain) {
        if (!ws->egm_x2) AIY_HIP(hipMalloc((void**)&ws->egm_x2, nb));
        if (!ws->egm_y2) AIY_HIP(hipMalloc((void**)&ws->egm_y2, nb));
    }
    double* xs[2] = {ws->g0, ws->egm_x2};
    double* ys[2] = {ws->g1, ws->egm_y2};
    auto step = [&](int64_t g) {
        EgmArgs A = A0;
        A.c = slot(g - 1);
        A.cout = slot(g);
        A.diff = sset(g);
        A.flags = (unsigned*)(sset(g) + 2 * kDiffSlots);
        A.diff_clear = nullptr;
        if (!chain) return launch_egm_step(A, st);
        A.ahat = xs[(g - 1) & 1];
        A.cnext = ys[(g - 1) & 1];
        A.ahat_next = xs[g & 1];
        A.cnext_next = ys[g & 1];
        A.diff_clear = sset(g + 1);
        AIY_TRY(ws_dispatch_arm(ws));  // (timing) the chained launch's own duration
        const int rc = launch_egm_chain(A, st);
        ws_dispatch_commit(ws);
        return rc;
    };
    if (chain) {  // step 1's RHS from slot 0; it clears step 1's slot set and flag word
        EgmArgs A = A0;
        A.c = slot(0);
        A.ahat = xs[0];
        A.cnext = ys[0];
        A.diff = sset(1);
        A.flags = (unsigned*)(sset(1) + 2 * kDiffSlots);
        AIY_TRY(launch_egm_rhs(A, st));
    }
    struct Batch {
        int64_t s0, m;  // steps s0 + 1 .. s0 + m
        int hb;         // host half holding its slot sets
    };
    Batch q[2];
    int nq = 0, hb_next = 0;
    int64_t enq = 0, stop = 0;
    double d_prev = NAN, d_last = NAN, d_stop = 1.0;
    auto enqueue = [&]() -> int {
        int64_t m = M;
        if (d_last == d_last && d_prev == d_prev && d_last < d_prev && d_last > 0) {
            // steps the observed geometric decay still needs, counted from the last read
            const double need = std::ceil(std::log(tol / d_last) / std::log(d_last / d_prev));
            int64_t ahead = 0;  // steps in flight, not yet read
            for (int b = 0; b < nq; ++b) ahead += q[b].m;
            if (need >= 1 && need - (double)ahead < (double)m)
                m = (int64_t)std::max(1.0, need - (double)ahead);
        }
        m = std::min<int64_t>(std::max<int64_t>(m, 1), max_iter - enq);
        for (int64_t t = 0; t < m; ++t) AIY_TRY(step(enq + 1 + t));
        unsigned long long* h = ws->egm_hslots + (size_t)hb_next * R * SW;
        AIY_HIP(hipMemcpyAsync(h, ws->egm_slots, SB, hipMemcpyDeviceToHost, st));
        AIY_HIP(hipEventRecord(ws->egm_ev[hb_next], st));
        q[nq++] = Batch{enq, m, hb_next};
        hb_next ^= 1;
        enq += m;
        return AIY_OK;
    };
    if (max_iter > 0) AIY_TRY(enqueue());
    while (nq > 0) {
        if (nq < 2 && enq < max_iter) AIY_TRY(enqueue());  // keep the device busy while reading
        const Batch b = q[0];
        AIY_TRY(wait_event(ws->egm_ev[b.hb]));
        const unsigned long long* hs = ws->egm_hslots + (size_t)b.hb * R * SW;
        for (int64_t t = 0; t < b.m; ++t) {
            const unsigned long long* h = hs + (size_t)((b.s0 + 1 + t) % R) * SW;
            if (egm_nonmonotone(h, (unsigned)h[2 * kDiffSlots])) {
                AIY_HIP(hipStreamSynchronize(st));
                return fail_nonmonotone();
            }
            const double d = fold_slots_host(h);
            d_prev = d_last;
            d_last = d;
            d_stop = d;
            if (!(d > tol)) {  // Aiyagari_EGM.m:74 `while dist > tol`
                stop = b.s0 + 1 + t;
                break;
            }
        }
        q[0] = q[1];
        --nq;
        if (stop) break;
    }
    AIY_HIP(hipStreamSynchronize(st));  // (a speculative batch may still be running)
    const int64_t g = stop ? stop : enq;
    if (g > 0 && g != enq) {  // policy_k/l of the stopping step (its slots are not read
                              // again): the two-launch step from its input
        EgmArgs A = A0;
        A.c = slot(g - 1);
        A.cout = slot(g);
        A.diff = sset(g);
        A.flags = (unsigned*)(sset(g) + 2 * kDiffSlots);
        A.diff_clear = nullptr;
        AIY_TRY(launch_egm_step(A, st));
    }
    *cur_out = g > 0 ? slot(g) : slot(0);
    *dist = d_stop;
    *iters = g;
    return AIY_OK;
}

static int egm_host(double* pc, const double* a, const double* s, const double* P, int64_t N,
                    int64_t Na, double r, double w, double beta, double sigma, double amin,
                    bool labor, double phi, double theta, bool solve, double tol,
                    int64_t max_iter, double* pcn_out, double* pk_out, double* pl_out,
                    double* dist, int64_t* iters) {
    if (!pc || !s || !P || !pk_out || !dist) return fail(AIY_BAD_ARG, "NULL argument");
    if (N < 1 || Na < 2) return fail(AIY_BAD_SHAPE, "need N >= 1 and Na >= 2");
    AIY_TRY(check_grid(a, Na));
    std::lock_guard<std::mutex> lk(host_mutex());
    HostCtx* c;
    AIY_TRY(get_ctx(N, Na, 1, &c));
    double *da, *ds, *dP, *dc0, *dc1, *dpk, *dpl;
    AIY_TRY(stage_common(c, a, s, P, N, Na, &da, &ds, &dP));
    size_t nb = sizeof(double) * N * Na;
    AIY_TRY(c->buf("egm_c0", nb, (void**)&dc0));
    AIY_TRY(c->buf("egm_c1", nb, (void**)&dc1));
    AIY_TRY(c->buf("pk", nb, (void**)&dpk));
    AIY_TRY(c->buf("pl", nb, (void**)&dpl));
    AIY_HIP(hipMemcpyAsync(dc0, pc, nb, hipMemcpyHostToDevice, c->st));
    double d = 1.0;
    int64_t it = 0;
    double* cur = dc0;
    double* nxt = dc1;
    if (!solve) {
        AIY_TRY(egm_step_dev(c->ws, cur, da, ds, dP, r, w, beta, sigma, amin, labor, phi, theta,
                             nxt, dpk, labor ? dpl : nullptr, nullptr, c->st));
        AIY_TRY(read_egm(c->ws, c->st, &d));
        cur = nxt;
        it = 1;
    } else if (c->ws->spec_max > 1 && max_iter > 0 && d > tol) {  // :74 tests dist = 1 first
        AIY_TRY(ensure_egm(c->ws));
        const EgmArgs A = egm_args(c->ws, cur, da, ds, dP, r, w, beta, sigma, amin, labor, phi,
                                   theta, nxt, dpk, labor ? dpl : nullptr);
        AIY_TRY(egm_solve_spec(c->ws, A, cur, tol, max_iter, &cur, &d, &it, c->st));
    } else {
        while (d > tol && it < max_iter) {  // Aiyagari_EGM.m:74
            ++it;
            AIY_TRY(egm_step_dev(c->ws, cur, da, ds, dP, r, w, beta, sigma, amin, labor, phi,
                                 theta, nxt, dpk, labor ? dpl : nullptr, nullptr, c->st));
            AIY_TRY(read_egm(c->ws, c->st, &d));
            std::swap(cur, nxt);  // :107 policy_c = policy_c_next
        }
    }
    double* dst = solve ? pc : pcn_out;
    if (dst) AIY_HIP(hipMemcpyAsync(dst, cur, nb, hipMemcpyDeviceToHost, c->st));
    AIY_HIP(hipMemcpyAsync(pk_out, dpk, nb, hipMemcpyDeviceToHost, c->st));
    if (labor && pl_out) AIY_HIP(hipMemcpyAsync(pl_out, dpl, nb, hipMemcpyDeviceToHost, c->st));
    AIY_HIP(hipStreamSynchronize(c->st));
    *dist = d;
    if (iters) *iters = it;
    return AIY_OK;
}

}  // namespace aiy

using namespace aiy;

extern "C" {

int aiy_egm_step(const double* policy_c, const double* a_grid, const double* s,
                 const double* P, int64_t N, int64_t Na, double r, double w, double beta,
                 double sigma, double amin, double* policy_c_next, double* policy_k,
                 double* dist) {
    if (!policy_c_next) return fail(AIY_BAD_ARG, "NULL policy_c_next");
    return egm_host(const_cast<double*>(policy_c), a_grid, s, P, N, Na, r, w, beta, sigma, amin,
                    false, 1, 1, false, 0, 1, policy_c_next, policy_k, nullptr, dist, nullptr);
}

int aiy_egm_solve(double* policy_c, const double* a_grid, const double* s, const double* P,
                  int64_t N, int64_t Na, double r, double w, double beta, double sigma,
                  double amin, double tol, int64_t max_iter, double* policy_k, double* dist,
                  int64_t* iters) {
    return egm_host(policy_c, a_grid, s, P, N, Na, r, w, beta, sigma, amin, false, 1, 1, true,
                    tol, max_iter, nullptr, policy_k, nullptr, dist, iters);
}

int aiy_labor_egm_step(const double* policy_c, const double* a_grid, const double* s,
                       const double* P, int64_t N, int64_t Na, double r, double w, double beta,
                       double sigma, double phi, double theta, double amin,
                       double* policy_c_next, double* policy_k, double* policy_l,
                       double* dist) {
    if (!policy_c_next || !policy_l) return fail(AIY_BAD_ARG, "NULL output");
    return egm_host(const_cast<double*>(policy_c), a_grid, s, P, N, Na, r, w, beta, sigma, amin,
                    true, phi, theta, false, 0, 1, policy_c_next, policy_k, policy_l, dist,
                    nullptr);
}

int aiy_labor_egm_solve(double* policy_c, const double* a_grid, const double* s,
                        const double* P, int64_t N, int64_t Na, double r, double w,
                        double beta, double sigma, double phi, double theta, double amin,
                        double tol, int64_t max_iter, double* policy_k, double* policy_l,
                        double* dist, int64_t* iters) {
    if (!policy_l) return fail(AIY_BAD_ARG, "NULL policy_l");
    return egm_host(policy_c, a_grid, s, P, N, Na, r, w, beta, sigma, amin, true, phi, theta,
                    true, tol, max_iter, nullptr, policy_k, policy_l, dist, iters);
}

int aiy_egm_solve_dev(aiy_ws* ws, double* policy_c, const double* a_grid, const double* s,
                      const double* P, double r, double w, double beta, double sigma,
                      double amin, int labor, double phi, double theta, double tol,
                      int64_t max_iter, double* policy_k, double* policy_l, int64_t* iters,
                      double* dist, void* stream) {
    if (!ws || !policy_c || !a_grid || !s || !P || !policy_k || !iters || !dist)
        return fail(AIY_BAD_ARG, "NULL argument");
    if (labor && !(phi == phi && theta == theta)) return fail(AIY_NON_FINITE, "phi/theta");
    if (max_iter < 0) return fail(AIY_BAD_ARG, "max_iter must be >= 0");
    hipStream_t st = (hipStream_t)stream;
    AIY_TRY(ensure_egm(ws));
    const size_t nb = sizeof(double) * ws->N * ws->Na;
    double d = 1.0;
    int64_t it = 0;
    if (max_iter > 0 && d > tol) {  // Aiyagari_EGM.m:74 tests dist = 1 first
        if (ws->spec_max > 1) {
            const EgmArgs A = egm_args(ws, policy_c, a_grid, s, P, r, w, beta, sigma, amin,
                                       labor != 0, phi, theta, nullptr, policy_k,
                                       labor ? policy_l : nullptr);
            double* cur = nullptr;
            AIY_TRY(egm_solve_spec(ws, A, policy_c, tol, max_iter, &cur, &d, &it, st));
            AIY_HIP(hipMemcpyAsync(policy_c, cur, nb, hipMemcpyDeviceToDevice, st));
        } else {
            double* nxt = ws->g2;
            if (!nxt) {
                AIY_HIP(hipMalloc((void**)&ws->g2, nb));
                nxt = ws->g2;
            }
            while (d > tol && it < max_iter) {  // :74 (one read per step)
                ++it;
                AIY_TRY(egm_step_dev(ws, policy_c, a_grid, s, P, r, w, beta, sigma, amin,
                                     labor != 0, phi, theta, nxt, policy_k,
                                     labor ? policy_l : nullptr, nullptr, st));
                AIY_TRY(read_egm(ws, st, &d));
                AIY_HIP(hipMemcpyAsync(policy_c, nxt, nb, hipMemcpyDeviceToDevice, st));
            }
        }
    }
    AIY_HIP(hipStreamSynchronize(st));
    *iters = it;
    *dist = d;
    return AIY_OK;
}

int aiy_egm_step_dev(aiy_ws* ws, const double* policy_c, const double* a_grid,
                     const double* s, const double* P, double r, double w, double beta,
                     double sigma, double amin, int labor, double phi, double theta,
                     double* policy_c_next, double* policy_k, double* policy_l, double* diff,
                     void* stream) {
    return egm_step_dev(ws, policy_c, a_grid, s, P, r, w, beta, sigma, amin, labor != 0, phi,
                        theta, policy_c_next, policy_k, policy_l, diff, (hipStream_t)stream);
}

}  // extern "C"
