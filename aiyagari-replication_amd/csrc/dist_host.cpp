// A10 entry points: aiy_dist_update_dev (one histogram push on device) and
// aiy_dist_stationary (MATLAB layouts, iterate to the fixed point, K = Σ λ·a).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <mutex>
#include <vector>

#include "aiy_common.hpp"
#include "dist.hpp"
#include "host_ctx.hpp"
#include "ws.hpp"

namespace aiy {

static int ensure_dist(aiy_ws* ws) {
    size_t n = (size_t)ws->N * ws->Na;
    if (!ws->d_key) AIY_HIP(hipMalloc((void**)&ws->d_key, n * sizeof(int)));
    if (!ws->d_head) AIY_HIP(hipMalloc((void**)&ws->d_head, n * sizeof(int)));
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

// one push λ → λ'; *d_out = max|λ'−λ| (host, synchronising) when d_out != nullptr
int dist_update_dev(aiy_ws* ws, const double* lam, const int* idx, const double* kp,
                    const double* a, const double* P, double* out, double* diff_dev,
                    double* d_host, hipStream_t st) {
    if (!ws || !lam || !a || !P || !out || (!idx && !kp))
        return fail(AIY_BAD_ARG, "NULL argument (need policy_idx or policy_k)");
    AIY_TRY(ensure_dist(ws));
    DistArgs A{};
    A.N = (int)ws->N; A.Na = (int)ws->Na; A.lottery = (idx == nullptr);
    A.idx = idx; A.kp = kp; A.a = a; A.P = P; A.lam = lam; A.out = out;
    A.key = ws->d_key; A.head = ws->d_head; A.wr = ws->d_wr; A.mass = ws->d_mass;
    A.diff = ws->diff; A.flags = (unsigned*)ws->gi;
    AIY_HIP(hipMemsetAsync(ws->diff, 0, 2 * kDiffSlots * sizeof(unsigned long long), st));
    AIY_HIP(hipMemsetAsync(ws->gi, 0, sizeof(int), st));
    AIY_TRY(ws_timing_begin(ws, st));
    AIY_TRY(launch_dist_update(A, false, st));
    AIY_TRY(ws_timing_end(ws, st));
    // flags decide whether the exact fallback must run: read them (synchronises)
    unsigned flags = 0;
    AIY_HIP(hipMemcpyAsync(&ws->hdiff[2 * kDiffSlots], ws->gi, sizeof(int), hipMemcpyDeviceToHost, st));
    AIY_HIP(hipStreamSynchronize(st));
    flags = (unsigned)ws->hdiff[2 * kDiffSlots];
    if (flags & 2u) return fail(AIY_BAD_ARG, "policy index outside [1, Na]");
    if (flags & 1u) {  // non-monotone policy: redo the gather by exhaustive ordered scans
        AIY_HIP(hipMemsetAsync(ws->diff, 0, 2 * kDiffSlots * sizeof(unsigned long long), st));
        AIY_TRY(launch_dist_update(A, true, st));
    }
    if (diff_dev) AIY_TRY(launch_reduce_slots(ws->diff, diff_dev, st));
    if (d_host) {
        AIY_HIP(hipMemcpyAsync(ws->hdiff, ws->diff, 2 * kDiffSlots * sizeof(unsigned long long),
                               hipMemcpyDeviceToHost, st));
        AIY_HIP(hipStreamSynchronize(st));
        *d_host = fold_slots_host(ws->hdiff);
    }
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
    int64_t it;
    double* cur = dl0;
    double* nxt = dl1;
    for (it = 1; it <= max_iter; ++it) {
        AIY_TRY(dist_update_dev(c->ws, cur, didx, dkp, da, dP, nxt, nullptr, &d, c->st));
        std::swap(cur, nxt);
        if (d < tol) break;
    }
    if (it > max_iter) it = max_iter;
    AIY_TRY(ensure_dist(c->ws));
    AIY_TRY(launch_dist_capital(cur, da, (int)N, (int)Na, c->ws->d_part, dK, c->st));
    AIY_HIP(hipMemcpyAsync(rows.data(), cur, nb, hipMemcpyDeviceToHost, c->st));
    AIY_HIP(hipMemcpyAsync(k_supply, dK, sizeof(double), hipMemcpyDeviceToHost, c->st));
    AIY_HIP(hipStreamSynchronize(c->st));
    if (vfi_layout) rows_to_cm(rows.data(), N, Na, lambda);
    else memcpy(lambda, rows.data(), nb);
    *iters = it;
    *dist = d;
    return AIY_OK;
}

}  // extern "C"
