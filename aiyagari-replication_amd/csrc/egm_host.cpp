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

static int ensure_egm(aiy_ws* ws) {
    size_t n = (size_t)ws->N * ws->Na;
    if (!ws->g0) AIY_HIP(hipMalloc((void**)&ws->g0, n * sizeof(double)));
    if (!ws->g1) AIY_HIP(hipMalloc((void**)&ws->g1, n * sizeof(double)));
    if (!ws->gi) AIY_HIP(hipMalloc((void**)&ws->gi, 16 * sizeof(int)));
    if (!ws->diff)
        AIY_HIP(hipMalloc((void**)&ws->diff, 2 * kDiffSlots * sizeof(unsigned long long)));
    if (!ws->hdiff)
        AIY_HIP(hipHostMalloc((void**)&ws->hdiff, (2 * kDiffSlots + 4) * sizeof(unsigned long long)));
    return AIY_OK;
}

int egm_step_dev(aiy_ws* ws, const double* c, const double* a, const double* s, const double* P,
                 double r, double w, double beta, double sigma, double amin, bool labor,
                 double phi, double theta, double* cout, double* pk, double* pl, double* diff_out,
                 hipStream_t st) {
    if (!ws || !c || !a || !s || !P || !cout || !pk) return fail(AIY_BAD_ARG, "NULL argument");
    if (labor && !(phi == phi && theta == theta)) return fail(AIY_NON_FINITE, "phi/theta");
    AIY_TRY(ensure_egm(ws));
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
    AIY_HIP(hipMemsetAsync(ws->diff, 0, 2 * kDiffSlots * sizeof(unsigned long long), st));
    AIY_HIP(hipMemsetAsync(ws->gi, 0, sizeof(int), st));
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
    if ((unsigned)h[2 * kDiffSlots] & 1u)
        return fail(AIY_BAD_ARG, "endogenous grid a_hat is not increasing: interp1 in the "
                                 "reference would sort it or fail (Aiyagari_EGM.m:95)");
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

int aiy_egm_step_dev(aiy_ws* ws, const double* policy_c, const double* a_grid,
                     const double* s, const double* P, double r, double w, double beta,
                     double sigma, double amin, int labor, double phi, double theta,
                     double* policy_c_next, double* policy_k, double* policy_l, double* diff,
                     void* stream) {
    return egm_step_dev(ws, policy_c, a_grid, s, P, r, w, beta, sigma, amin, labor != 0, phi,
                        theta, policy_c_next, policy_k, policy_l, diff, (hipStream_t)stream);
}

}  // extern "C"
