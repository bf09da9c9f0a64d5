// A8 entry point (Krusell_Smith_EGM.m:129-209): k_opt is k x K x S column-major exactly as
// in the script; P is MATLAB's 4 x 4; params = the 13-double KS block {beta, alpha, delta,
// k_min, k_max, ug, ub, l_bar, mu, z_grid(1:2), eps_grid(1:2)} (mu unused by the EGM script).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <mutex>
#include <vector>

#include "aiy_common.hpp"
#include "host_ctx.hpp"
#include "ks_egm.hpp"
#include "ws.hpp"

#include <algorithm>

namespace aiy {

// per-pair scalars in the script's order with libm (:101-112 tables, :139-175)
static void ks_egm_pairs(const double* prm, const double* K_grid, const double* B, int nK,
                         std::vector<KsEgmPair>& out) {
    const double alpha = prm[1], delta = prm[2], ug = prm[5], ub = prm[6], lb = prm[7];
    const double zg[2] = {prm[9], prm[10]}, eg[2] = {prm[11], prm[12]};
    out.resize(4 * nK);
    auto labour = [&](double z) {
        return lb * (1 - ug * (double)(z == zg[0]) - ub * (double)(z == zg[1]));
    };
    auto alm = [&](double z, double K) {
        return (z == zg[0]) ? exp(B[0] + B[1] * log(K)) : exp(B[2] + B[3] * log(K));
    };
    for (int s_i = 0; s_i < 4; ++s_i) {
        const double z = zg[s_i < 2 ? 0 : 1], e = eg[s_i % 2];  // s_grid = [Z(:), Eps(:)] (:18-19)
        for (int K_i = 0; K_i < nK; ++K_i) {
            KsEgmPair q{};
            const double K = K_grid[K_i];
            const double L = labour(z);
            const double r = alpha * z * pow(K, alpha - 1) * pow(L, 1 - alpha);  // r_table (:110)
            const double w = (1 - alpha) * z * pow(K, alpha) * pow(L, -alpha);   // w_table (:109)
            const double Kp = alm(z, K);                                         // :140-145
            for (int s_j = 0; s_j < 4; ++s_j) {
                const double zn = zg[s_j < 2 ? 0 : 1], en = eg[s_j % 2];
                const double Kd = alm(zn, Kp);                                   // :164-169
                int idx = 0;
                double bd = fabs(K_grid[0] - Kd);
                for (int m = 1; m < nK; ++m) {  // min(abs(K_grid - K_dprime)): first on ties
                    const double dd = fabs(K_grid[m] - Kd);
                    if (dd < bd) {
                        bd = dd;
                        idx = m;
                    }
                }
                const double Ln = labour(zn);
                const double rn = alpha * zn * pow(Kd, alpha - 1) * pow(Ln, 1 - alpha);  // :174
                const double wn = (1 - alpha) * zn * pow(Kd, alpha) * pow(Ln, -alpha);   // :175
                q.kd[s_j] = idx;
                q.Rn[s_j] = (1 + rn) - delta;
                q.Wn[s_j] = (wn * en) * lb;
            }
            q.R = (1 + r) - delta;
            q.We = (w * e) * lb;
            out[s_i * nK + K_i] = q;
        }
    }
}

}  // namespace aiy

using namespace aiy;

extern "C" {

int ks_egm_solve(double* k_opt, const double* k_grid, const double* K_grid, const double* B,
                 const double* P, const double* params, int64_t nk, int64_t nK, double tol,
                 int64_t max_iter, int64_t* iters, double* diff) {
    if (!k_opt || !k_grid || !K_grid || !B || !P || !params || !iters || !diff)
        return fail(AIY_BAD_ARG, "NULL argument");
    if (nk < 3 || nK < 1 || nk > (1 << 20))
        return fail(AIY_BAD_SHAPE, "need k_size >= 3 and K_size >= 1");
    if (max_iter < 1 || max_iter > 2147483647) return fail(AIY_BAD_ARG, "max_iter in [1, 2^31)");
    if (!ks_egm_fits((int)nk, (int)nK))
        return fail(AIY_BAD_SHAPE, "k_size x K_size too large for the one-workgroup EGM solve");
    AIY_TRY(check_grid(k_grid, nk));
    for (int64_t q = 0; q < nK; ++q)
        if (!(K_grid[q] > 0) || !std::isfinite(K_grid[q]))
            return fail(AIY_NON_FINITE, "K_grid must be positive and finite");
    std::lock_guard<std::mutex> lk(host_mutex());
    HostCtx* c;
    AIY_TRY(get_ctx(4 * nK, nk, 1, &c));
    std::vector<KsEgmPair> pairs;
    ks_egm_pairs(params, K_grid, B, (int)nK, pairs);
    double Pr[16];
    for (int i = 0; i < 4; ++i)
        for (int m = 0; m < 4; ++m) Pr[i * 4 + m] = P[i + m * 4];
    const size_t n = (size_t)nk * nK * 4;
    double *dkg, *dP, *dk;
    KsEgmPair* dpairs;
    KsEgmOut* dout;
    AIY_TRY(c->buf("egm_kg", nk * sizeof(double), (void**)&dkg));
    AIY_TRY(c->buf("egm_P", sizeof Pr, (void**)&dP));
    AIY_TRY(c->buf("egm_k", n * sizeof(double), (void**)&dk));
    AIY_TRY(c->buf("egm_pairs", pairs.size() * sizeof(KsEgmPair), (void**)&dpairs));
    AIY_TRY(c->buf("egm_out", sizeof(KsEgmOut), (void**)&dout));
    AIY_HIP(hipMemcpyAsync(dkg, k_grid, nk * sizeof(double), hipMemcpyHostToDevice, c->st));
    AIY_HIP(hipMemcpyAsync(dP, Pr, sizeof Pr, hipMemcpyHostToDevice, c->st));
    AIY_HIP(hipMemcpyAsync(dk, k_opt, n * sizeof(double), hipMemcpyHostToDevice, c->st));
    AIY_HIP(hipMemcpyAsync(dpairs, pairs.data(), pairs.size() * sizeof(KsEgmPair),
                           hipMemcpyHostToDevice, c->st));
    KsEgmArgs A{};
    A.nk = (int)nk;
    A.nK = (int)nK;
    A.max_iter = (int)max_iter;
    A.k_grid = dkg;
    A.P = dP;
    A.pairs = dpairs;
    A.beta = params[0];
    A.k_min = params[3];
    A.k_max = params[4];
    A.tol = tol;
    AIY_TRY(launch_ks_egm_solve(A, dk, dout, c->st));
    KsEgmOut o;
    AIY_HIP(hipMemcpyAsync(&o, dout, sizeof o, hipMemcpyDeviceToHost, c->st));
    AIY_HIP(hipMemcpyAsync(k_opt, dk, n * sizeof(double), hipMemcpyDeviceToHost, c->st));
    AIY_HIP(hipStreamSynchronize(c->st));
    *iters = o.iters;
    *diff = o.diff;
    if (o.status)
        return fail(AIY_NON_FINITE, "an (s, K) pair had fewer than 2 valid EGM points "
                                    "(griddedInterpolant needs two; Krusell_Smith_EGM.m:196)");
    return AIY_OK;
}

// F1 — the Jacobi variant of the KS EGM iteration: every (s, K) pair of a sweep reads the
// previous sweep's k_opt, all pairs of a sweep in one launch.  NOT the reference's result (the
// script is Gauss-Seidel, Krusell_Smith_EGM.m:199); same stop rule (:204-207).  Sweeps are
// enqueued in batches with one diff-slot set each and read back once per batch.
int ks_egm_solve_jacobi(double* k_opt, const double* k_grid, const double* K_grid,
                        const double* B, const double* P, const double* params, int64_t nk,
                        int64_t nK, double tol, int64_t max_iter, int64_t* iters, double* diff) {
    if (!k_opt || !k_grid || !K_grid || !B || !P || !params || !iters || !diff)
        return fail(AIY_BAD_ARG, "NULL argument");
    if (nk < 3 || nK < 1) return fail(AIY_BAD_SHAPE, "need k_size >= 3 and K_size >= 1");
    if (ks_egm_jacobi_lds_bytes((int)nk) > 150 * 1024)
        return fail(AIY_BAD_SHAPE, "k_size too large for one workgroup per (s, K) pair");
    if (max_iter < 1 || max_iter > 2147483647) return fail(AIY_BAD_ARG, "max_iter in [1, 2^31)");
    AIY_TRY(check_grid(k_grid, nk));
    for (int64_t q = 0; q < nK; ++q)
        if (!(K_grid[q] > 0) || !std::isfinite(K_grid[q]))
            return fail(AIY_NON_FINITE, "K_grid must be positive and finite");
    std::lock_guard<std::mutex> lk(host_mutex());
    HostCtx* c;
    AIY_TRY(get_ctx(4 * nK, nk, 1, &c));
    std::vector<KsEgmPair> pairs;
    ks_egm_pairs(params, K_grid, B, (int)nK, pairs);
    double Pr[16];
    for (int i = 0; i < 4; ++i)
        for (int m = 0; m < 4; ++m) Pr[i * 4 + m] = P[i + m * 4];
    const size_t n = (size_t)nk * nK * 4;
    constexpr int kBatch = 16;
    // ring of kBatch + 1 policy buffers: sweep g reads slot (g-1) % R and writes slot g % R, so
    // the sweeps a batch runs past the stopping sweep never overwrite its output
    constexpr int R = kBatch + 1;
    double *dkg, *dP, *ring;
    KsEgmPair* dpairs;
    unsigned long long* dslots;
    int* dstatus;
    AIY_TRY(c->buf("egmj_kg", nk * sizeof(double), (void**)&dkg));
    AIY_TRY(c->buf("egmj_P", sizeof Pr, (void**)&dP));
    AIY_TRY(c->buf("egmj_ring", (size_t)R * n * sizeof(double), (void**)&ring));
    AIY_TRY(c->buf("egmj_pairs", pairs.size() * sizeof(KsEgmPair), (void**)&dpairs));
    AIY_TRY(c->buf("egmj_slots", kBatch * 2 * kDiffSlots * sizeof(unsigned long long), (void**)&dslots));
    AIY_TRY(c->buf("egmj_status", sizeof(int), (void**)&dstatus));
    AIY_HIP(hipMemcpyAsync(dkg, k_grid, nk * sizeof(double), hipMemcpyHostToDevice, c->st));
    AIY_HIP(hipMemcpyAsync(dP, Pr, sizeof Pr, hipMemcpyHostToDevice, c->st));
    AIY_HIP(hipMemcpyAsync(ring, k_opt, n * sizeof(double), hipMemcpyHostToDevice, c->st));
    AIY_HIP(hipMemcpyAsync(dpairs, pairs.data(), pairs.size() * sizeof(KsEgmPair),
                           hipMemcpyHostToDevice, c->st));
    AIY_HIP(hipMemsetAsync(dstatus, 0, sizeof(int), c->st));
    KsEgmArgs A{};
    A.nk = (int)nk; A.nK = (int)nK; A.max_iter = (int)max_iter; A.k_grid = dkg; A.P = dP;
    A.pairs = dpairs; A.beta = params[0]; A.k_min = params[3]; A.k_max = params[4]; A.tol = tol;
    auto slot = [&](int64_t g) { return ring + (size_t)(g % R) * n; };
    std::vector<unsigned long long> hs(kBatch * 2 * kDiffSlots);
    int64_t done = 0, stop = 0;
    double d_last = NAN;
    int status = 0;
    while (!stop && done < max_iter) {
        const int64_t m = std::min<int64_t>(kBatch, max_iter - done);
        AIY_HIP(hipMemsetAsync(dslots, 0, m * 2 * kDiffSlots * sizeof(unsigned long long), c->st));
        for (int64_t t = 0; t < m; ++t) {
            const int64_t g = done + 1 + t;
            AIY_TRY(launch_ks_egm_jacobi(A, slot(g - 1), slot(g),
                                         dslots + t * 2 * kDiffSlots, dstatus, c->st));
        }
        AIY_HIP(hipMemcpyAsync(hs.data(), dslots, m * 2 * kDiffSlots * sizeof(unsigned long long),
                               hipMemcpyDeviceToHost, c->st));
        AIY_HIP(hipMemcpyAsync(&status, dstatus, sizeof(int), hipMemcpyDeviceToHost, c->st));
        AIY_HIP(hipStreamSynchronize(c->st));
        if (status) break;
        for (int64_t t = 0; t < m; ++t) {
            d_last = fold_slots_host(hs.data() + t * 2 * kDiffSlots);
            if (d_last < tol) {
                stop = done + 1 + t;
                break;
            }
        }
        if (!stop) done += m;
    }
    if (status)
        return fail(AIY_NON_FINITE, "an (s, K) pair had fewer than 2 valid EGM points "
                                    "(griddedInterpolant needs two; Krusell_Smith_EGM.m:196)");
    const int64_t g = stop ? stop : max_iter;
    AIY_HIP(hipMemcpyAsync(k_opt, slot(g), n * sizeof(double), hipMemcpyDeviceToHost, c->st));
    AIY_HIP(hipStreamSynchronize(c->st));
    *iters = g;
    *diff = d_last;
    return AIY_OK;
}

}  // extern "C"
