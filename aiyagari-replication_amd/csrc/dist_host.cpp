// A10 entry points: aiy_dist_update_dev (one histogram push on device),
// aiy_dist_stationary_dev (iterate to the fixed point on device) and aiy_dist_stationary
// (MATLAB layouts, K = Σ λ·a).
//
// The policy is fixed across the fixed-point iteration, so its plan (keys, lottery weights,
// run offsets, the monotonicity flag) is built ONCE per call and read back once; every push is
// then one launch (dist_push_kernel).  The iteration runs in speculative batches as the VFI
// and EGM solves do: m pushes are enqueued per batch — push g reads ring slot (g−1) mod R
// and writes slot g mod R, its max|Δλ| lands in its own slot set — and the host reads one
// batch's slot sets while the next batch runs, to find the first push with max|Δλ| < tol.  Pushes are deterministic, so the iteration count,
// the returned λ and dist are exactly the one-read-per-push loop's.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <vector>

#include "aiy_common.hpp"
#include "dist.hpp"
#include "host_ctx.hpp"
#include "ws.hpp"

namespace aiy {

constexpr int kDistSpecMax = 32;  // pushes per batch (two batches in flight)

static int ensure_dist(aiy_ws* ws) {
    const size_t n = (size_t)ws->N * ws->Na;
    if (!ws->d_key) AIY_HIP(hipMalloc((void**)&ws->d_key, n * sizeof(int)));
    if (!ws->d_off) AIY_HIP(hipMalloc((void**)&ws->d_off, (n + ws->N) * sizeof(int)));
    if (!ws->d_wr) AIY_HIP(hipMalloc((void**)&ws->d_wr, n * sizeof(double)));
    if (!ws->d_mass) AIY_HIP(hipMalloc((void**)&ws->d_mass, n * sizeof(double)));
    if (!ws->d_part) AIY_HIP(hipMalloc((void**)&ws->d_part, 260 * sizeof(double)));
    if (!ws->gi) AIY_HIP(hipMalloc((void**)&ws->gi, 16 * sizeof(int)));
    if (!ws->diff)
        AIY_HIP(hipMalloc((void**)&ws->diff, 2 * kDiffSlots * sizeof(unsigned long long)));
    if (!ws->hdiff)
        AIY_HIP(hipHostMalloc((void**)&ws->hdiff, (2 * kDiffSlots + 4) * sizeof(unsigned long long)));
    return AIY_OK;
}

// the policy's plan; *fallback = the policy is not monotone (ordered-scan gather).
// Synchronises once to read the flags.
static int dist_plan(aiy_ws* ws, const int* idx, const double* kp, const double* a,
                     const double* P, DistArgs* A, bool* fallback, hipStream_t st) {
    if (!ws || !a || !P || (!idx && !kp))
        return fail(AIY_BAD_ARG, "NULL argument (need policy_idx or policy_k)");
    AIY_TRY(ensure_dist(ws));
    *A = DistArgs{};
    A->N = (int)ws->N; A->Na = (int)ws->Na; A->lottery = (idx == nullptr);
    A->idx = idx; A->kp = kp; A->a = a; A->P = P;
    A->key = ws->d_key; A->off = ws->d_off; A->wr = ws->d_wr; A->mass = ws->d_mass;
    A->diff = ws->diff; A->flags = (unsigned*)ws->gi;
    A->trace = nullptr;
    if (ws->tracing) {  // (instrumentation) one record per push wave: ceil(Na/64)·N <= cap
        const int64_t cap = (int64_t)ws->N * ((ws->Na + 15) / 16);
        if (ws->trace_cap < cap) {
            if (ws->trace) (void)hipFree(ws->trace);
            ws->trace = nullptr;
            ws->trace_cap = 0;
            AIY_HIP(hipMalloc((void**)&ws->trace, 16 * (size_t)cap * sizeof(long long)));
            ws->trace_cap = cap;
        }
        AIY_HIP(hipMemsetAsync(ws->trace, 0, 16 * (size_t)cap * sizeof(long long), st));
        A->trace = ws->trace;
    }
    AIY_HIP(hipMemsetAsync(ws->gi, 0, sizeof(int), st));
    AIY_TRY(launch_dist_prepare(*A, st));
    AIY_HIP(hipMemcpyAsync(&ws->hdiff[2 * kDiffSlots], ws->gi, sizeof(int), hipMemcpyDeviceToHost, st));
    AIY_HIP(hipStreamSynchronize(st));
    const unsigned flags = (unsigned)ws->hdiff[2 * kDiffSlots];
    if (flags & 2u) return fail(AIY_BAD_ARG, "policy index outside [1, Na]");
    *fallback = (flags & 1u) != 0;
    return AIY_OK;
}

// one push λ → λ'; *d_host = max|λ'−λ| (synchronising) when d_host != nullptr
int dist_update_dev(aiy_ws* ws, const double* lam, const int* idx, const double* kp,
                    const double* a, const double* P, double* out, double* diff_dev,
                    double* d_host, hipStream_t st) {
    if (!lam || !out) return fail(AIY_BAD_ARG, "NULL argument");
    DistArgs A;
    bool fb = false;
    AIY_TRY(dist_plan(ws, idx, kp, a, P, &A, &fb, st));
    A.lam = lam;
    A.out = out;
    AIY_HIP(hipMemsetAsync(ws->diff, 0, 2 * kDiffSlots * sizeof(unsigned long long), st));
    AIY_TRY(ws_timing_begin(ws, st));
    AIY_TRY(launch_dist_push(A, fb, st));
    AIY_TRY(ws_timing_end(ws, st));
    if (diff_dev) AIY_TRY(launch_reduce_slots(ws->diff, diff_dev, st));
    if (d_host) {
        AIY_HIP(hipMemcpyAsync(ws->hdiff, ws->diff, 2 * kDiffSlots * sizeof(unsigned long long),
                               hipMemcpyDeviceToHost, st));
        AIY_HIP(hipStreamSynchronize(st));
        *d_host = fold_slots_host(ws->hdiff);
    }
    return AIY_OK;
}

// the fixed-point loop of aiy_dist_stationary on device:  for it = 1..max_iter: push; stop
// when max|Δλ| < tol.  lam_out receives the last push; k_dev (nullable) = Σ λ·a.  Batches of
// pushes with one D2H copy of their diff slots and an event each; two batches in flight (the
// host reads batch k while batch k+1 runs), a ring of 2M + 1 λ buffers so that the stopping
// push's λ survives the next batch.
int dist_stationary_dev(aiy_ws* ws, const double* lam0, const int* idx, const double* kp,
                        const double* a, const double* P, double tol, int64_t max_iter,
                        double* lam_out, double* k_dev, int64_t* iters, double* dist,
                        hipStream_t st) {
    if (!lam0 || !lam_out || !iters || !dist) return fail(AIY_BAD_ARG, "NULL argument");
    if (max_iter < 1) return fail(AIY_BAD_ARG, "max_iter must be >= 1");
    DistArgs A0;
    bool fb = false;
    AIY_TRY(dist_plan(ws, idx, kp, a, P, &A0, &fb, st));
    const bool two_launch = fb || ws->N > kDistPushMaxN;  // (no diff_clear in those kernels)
    const int M = kDistSpecMax, R = 2 * M + 1;
    const size_t n = (size_t)ws->N * ws->Na, nb = n * sizeof(double);
    const int SW = 2 * kDiffSlots;
    const size_t SB = (size_t)R * SW * sizeof(unsigned long long);
    if (ws->dist_n != n || ws->dist_m != M) {
        ws->free_dist_spec();
        AIY_HIP(hipMalloc((void**)&ws->dist_ring, (size_t)R * nb));
        AIY_HIP(hipMalloc((void**)&ws->dist_slots, SB));
        AIY_HIP(hipHostMalloc((void**)&ws->dist_hslots, 2 * SB));
        for (int b = 0; b < 2; ++b)
            AIY_HIP(hipEventCreateWithFlags(&ws->dist_ev[b], hipEventDisableTiming));
        ws->dist_n = n;
        ws->dist_m = M;
    }
    auto slot = [&](int64_t g) { return ws->dist_ring + (size_t)(g % R) * n; };
    auto sset = [&](int64_t g) { return ws->dist_slots + (size_t)(g % R) * SW; };
    AIY_HIP(hipMemcpyAsync(slot(0), lam0, nb, hipMemcpyDeviceToDevice, st));
    AIY_HIP(hipMemsetAsync(sset(1), 0, SW * sizeof(unsigned long long), st));
    struct Batch {
        int64_t s0, m;  // pushes s0 + 1 .. s0 + m
        int hb;
    };
    Batch q[2];
    int nq = 0, hb_next = 0;
    int64_t enq = 0, stop = 0;
    double d_prev = NAN, d_last = NAN, d_stop = NAN;
    auto enqueue = [&]() -> int {
        int64_t m = M;
        if (d_last == d_last && d_prev == d_prev && d_last < d_prev && d_last > 0 && tol > 0) {
            const double need = std::ceil(std::log(tol / d_last) / std::log(d_last / d_prev));
            int64_t ahead = 0;  // pushes in flight, not yet read
            for (int b = 0; b < nq; ++b) ahead += q[b].m;
            if (need >= 1 && need - (double)ahead < (double)m)
                m = (int64_t)std::max(1.0, need - (double)ahead);
        }
        m = std::min<int64_t>(std::max<int64_t>(m, 1), max_iter - enq);
        for (int64_t t = 0; t < m; ++t) {
            const int64_t g = enq + 1 + t;
            DistArgs A = A0;
            A.lam = slot(g - 1);
            A.out = slot(g);
            A.diff = sset(g);
            // push g's set was zeroed by push g−1 (one-launch push) or is zeroed here
            if (two_launch) AIY_HIP(hipMemsetAsync(sset(g), 0, SW * sizeof(unsigned long long), st));
            else A.diff_clear = sset(g + 1);
            AIY_TRY(ws_dispatch_arm(ws));  // the push's own duration (one-launch push)
            const int rc = launch_dist_push(A, fb, st);
            ws_dispatch_commit(ws);
            AIY_TRY(rc);
        }
        unsigned long long* h = ws->dist_hslots + (size_t)hb_next * R * SW;
        AIY_HIP(hipMemcpyAsync(h, ws->dist_slots, SB, hipMemcpyDeviceToHost, st));
        AIY_HIP(hipEventRecord(ws->dist_ev[hb_next], st));
        q[nq++] = Batch{enq, m, hb_next};
        hb_next ^= 1;
        enq += m;
        return AIY_OK;
    };
    AIY_TRY(enqueue());
    while (nq > 0) {
        if (nq < 2 && enq < max_iter) AIY_TRY(enqueue());  // keep the device busy while reading
        const Batch b = q[0];
        AIY_TRY(wait_event(ws->dist_ev[b.hb]));
        const unsigned long long* hs = ws->dist_hslots + (size_t)b.hb * R * SW;
        for (int64_t t = 0; t < b.m; ++t) {
            const double d = fold_slots_host(hs + (size_t)((b.s0 + 1 + t) % R) * SW);
            d_prev = d_last;
            d_last = d;
            d_stop = d;
            if (d < tol) {
                stop = b.s0 + 1 + t;
                break;
            }
        }
        q[0] = q[1];
        --nq;
        if (stop) break;
    }
    const int64_t g = stop ? stop : enq;
    AIY_HIP(hipMemcpyAsync(lam_out, slot(g), nb, hipMemcpyDeviceToDevice, st));
    if (k_dev)
        AIY_TRY(launch_dist_capital(lam_out, a, (int)ws->N, (int)ws->Na, ws->d_part, k_dev, st));
    AIY_HIP(hipStreamSynchronize(st));  // (a speculative batch may still be running)
    *iters = g;
    *dist = d_stop;
    return AIY_OK;
}

}  // namespace aiy

using namespace aiy;

extern "C" {

int aiy_dist_update_dev(aiy_ws* ws, const double* lambda, const int32_t* policy_idx,
                        const double* policy_k, const double* a_grid, const double* P,
                        double* lambda_out, double* diff, void* stream) {
    return dist_update_dev(ws, lambda, policy_idx, policy_k, a_grid, P, lambda_out, diff,
                           nullptr, (hipStream_t)stream);
}

int aiy_dist_stationary_dev(aiy_ws* ws, const double* lambda, const int32_t* policy_idx,
                            const double* policy_k, const double* a_grid, const double* P,
                            double tol, int64_t max_iter, double* lambda_out,
                            double* k_supply, int64_t* iters, double* dist, void* stream) {
    return dist_stationary_dev(ws, lambda, policy_idx, policy_k, a_grid, P, tol, max_iter,
                               lambda_out, k_supply, iters, dist, (hipStream_t)stream);
}

int aiy_dist_stationary(const int32_t* policy_idx, const double* policy_k, int vfi_layout,
                        const double* a_grid, const double* P, int64_t N, int64_t Na,
                        double tol, int64_t max_iter, double* lambda, double* k_supply,
                        int64_t* iters, double* dist) {
    if ((!policy_idx && !policy_k) || !P || !lambda || !k_supply || !iters || !dist)
        return fail(AIY_BAD_ARG, "NULL argument");
    if (N < 1 || Na < 2) return fail(AIY_BAD_SHAPE, "need N >= 1 and Na >= 2");
    if (max_iter < 1) return fail(AIY_BAD_ARG, "max_iter must be >= 1");
    // the lottery divides by a(k+1) - a(k): repeated nodes are rejected (interp1 would error)
    AIY_TRY(policy_k ? check_grid_strict(a_grid, Na) : check_grid(a_grid, Na));
    std::lock_guard<std::mutex> lk(host_mutex());
    HostCtx* c;
    AIY_TRY(get_ctx(N, Na, 1, &c));
    std::vector<double> s1(N, 1.0);
    double *da, *ds, *dP, *dl0, *dl1, *dkp = nullptr, *dK;
    int* didx = nullptr;
    AIY_TRY(stage_common(c, a_grid, s1.data(), P, N, Na, &da, &ds, &dP));
    size_t n = (size_t)N * Na, nb = n * sizeof(double);
    AIY_TRY(c->buf("dist_l0", nb, (void**)&dl0));
    AIY_TRY(c->buf("dist_l1", nb, (void**)&dl1));
    AIY_TRY(c->buf("dist_K", 16, (void**)&dK));
    // layouts: vfi_layout → N x Na column-major; else Na x N column-major (== [N][Na])
    std::vector<double> rows(n);
    auto to_rows = [&](const double* src) {
        if (vfi_layout) cm_to_rows(src, N, Na, rows.data());
        else memcpy(rows.data(), src, nb);
    };
    if (policy_idx) {
        std::vector<int> ib(n);
        for (int64_t i = 0; i < N; ++i)
            for (int64_t j = 0; j < Na; ++j)
                ib[i * Na + j] = (vfi_layout ? policy_idx[i + j * N] : policy_idx[j + i * Na]) - 1;
        AIY_TRY(c->buf("dist_idx", n * sizeof(int), (void**)&didx));
        AIY_HIP(hipMemcpyAsync(didx, ib.data(), n * sizeof(int), hipMemcpyHostToDevice, c->st));
        AIY_HIP(hipStreamSynchronize(c->st));
    } else {
        AIY_TRY(c->buf("dist_kp", nb, (void**)&dkp));
        to_rows(policy_k);
        AIY_HIP(hipMemcpyAsync(dkp, rows.data(), nb, hipMemcpyHostToDevice, c->st));
        AIY_HIP(hipStreamSynchronize(c->st));
    }
    to_rows(lambda);
    AIY_HIP(hipMemcpyAsync(dl0, rows.data(), nb, hipMemcpyHostToDevice, c->st));
    double d = NAN;
    int64_t it = 0;
    AIY_TRY(dist_stationary_dev(c->ws, dl0, didx, dkp, da, dP, tol, max_iter, dl1, dK, &it, &d,
                                c->st));
    AIY_HIP(hipMemcpyAsync(rows.data(), dl1, nb, hipMemcpyDeviceToHost, c->st));
    AIY_HIP(hipMemcpyAsync(k_supply, dK, sizeof(double), hipMemcpyDeviceToHost, c->st));
    AIY_HIP(hipStreamSynchronize(c->st));
    if (vfi_layout) rows_to_cm(rows.data(), N, Na, lambda);
    else memcpy(lambda, rows.data(), nb);
    *iters = it;
    *dist = d;
    return AIY_OK;
}

}  // extern "C"
