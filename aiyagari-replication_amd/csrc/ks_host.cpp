// A6/A7 entry points (Krusell_Smith_VFI.m:143-204).  value / k_opt are k x K x S
// column-major, exactly as in the script; P is MATLAB's 4 x 4; params = 13 doubles
// {beta, alpha, delta, k_min, k_max, ug, ub, l_bar, mu, z_grid(1:2), eps_grid(1:2)}.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <mutex>
#include <vector>

#include "aiy_common.hpp"
#include "host_ctx.hpp"
#include "ks.hpp"
#include "ws.hpp"

namespace aiy {

// per-slice constants, in the script's own operation order (libm pow/exp/log on the host)
void ks_slices(const KsParams& p, const double* B, const double* K_grid, int nK,
                      std::vector<KsSlice>& out) {
    out.resize(4 * nK);
    const double zg[2] = {p.z1, p.z2}, eg[2] = {p.e1, p.e2};
    for (int si = 0; si < 4; ++si)
        for (int Ki = 0; Ki < nK; ++Ki) {
            KsSlice sl{};
            double K = K_grid[Ki];
            // bellman_value: current_z = z_grid((s_i <= 2) + 1)  (flipped, :332)
            double z = zg[(si + 1 <= 2) ? 1 : 0];
            double Kp;
            if (z == zg[0]) Kp = exp(B[0] + B[1] * log(fmax(K, 1e-8)));
            else Kp = exp(B[2] + B[3] * log(fmax(K, 1e-8)));
            Kp = fmax(fmin(Kp, K_grid[nK - 1]), K_grid[0]);
            int idx = 0;
            double bd = fabs(K_grid[0] - Kp);
            for (int q = 1; q < nK; ++q) {
                double dd = fabs(K_grid[q] - Kp);
                if (dd < bd) { bd = dd; idx = q; }
            }
            sl.kp_idx = idx;
            double L = p.l_bar * (1 - p.ug * (double)(z == zg[0]) - p.ub * (double)(z == zg[1]));
            double r_val = p.alpha * z * pow(K, p.alpha - 1) * pow(L, 1 - p.alpha);
            double w_val = (1 - p.alpha) * z * pow(K, p.alpha) * pow(L, -p.alpha);
            double eps = (si % 2 == 0) ? eg[0] : eg[1];  // s_grid(s_i, 2), :19-20
            sl.a1 = r_val + 1 - p.delta;
            sl.a2 = w_val * (eps * p.l_bar);
            // resources for fminbnd's upper bound use the table z (:107-115, :149-155)
            double zt = (si < 2) ? zg[0] : zg[1];
            double Lt = p.l_bar * (1 - p.ug * (double)(zt == zg[0]) - p.ub * (double)(zt == zg[1]));
            double wt = (1 - p.alpha) * zt * pow(K, p.alpha) * pow(Lt, -p.alpha);
            double rt = p.alpha * zt * pow(K, p.alpha - 1) * pow(Lt, 1 - p.alpha);
            sl.b1 = rt + 1 - p.delta;
            sl.b2 = wt * (eps * p.l_bar + (1 - eps) * p.mu);
            out[si * nK + Ki] = sl;
        }
}

struct KsDev {
    double *kg, *kgt, *P, *V, *V2, *dV, *dV2, *Vold, *kopt;
    int* nfev;
    int* seg;  // Howard segment hints (verified before use, so never initialised)
    KsSlice* sl;
    KsOut* out;
    unsigned long long* slots;
};

static int ks_stage(HostCtx* c, const double* value, const double* k_opt, const double* k_grid,
                    const double* K_grid, const double* B, const double* P, const double* params,
                    int64_t nk, int64_t nK, KsArgs& A, KsDev& D) {
    if (!value || !k_grid || !K_grid || !B || !P || !params)
        return fail(AIY_BAD_ARG, "NULL argument");
    if (nk < 3 || nK < 1) return fail(AIY_BAD_SHAPE, "need k_size >= 3 and K_size >= 1");
    AIY_TRY(check_grid(k_grid, nk));
    KsParams p;
    memcpy(&p, params, sizeof p);
    std::vector<KsSlice> sl;
    ks_slices(p, B, K_grid, (int)nK, sl);
    size_t n = (size_t)nk * nK * 4, nb = n * sizeof(double);
    AIY_TRY(c->buf("ks_kg", nk * sizeof(double), (void**)&D.kg));
    AIY_TRY(c->buf("ks_kgt", 3 * nk * sizeof(double), (void**)&D.kgt));
    AIY_TRY(c->buf("ks_P", 16 * sizeof(double), (void**)&D.P));
    AIY_TRY(c->buf("ks_V", nb, (void**)&D.V));
    AIY_TRY(c->buf("ks_V2", nb, (void**)&D.V2));
    AIY_TRY(c->buf("ks_dV", nb, (void**)&D.dV));
    AIY_TRY(c->buf("ks_dV2", nb, (void**)&D.dV2));
    AIY_TRY(c->buf("ks_Vold", nb, (void**)&D.Vold));
    AIY_TRY(c->buf("ks_kopt", nb, (void**)&D.kopt));
    AIY_TRY(c->buf("ks_nfev", n * sizeof(int), (void**)&D.nfev));
    AIY_TRY(c->buf("ks_seg", n * sizeof(int), (void**)&D.seg));
    AIY_TRY(c->buf("ks_sl", sl.size() * sizeof(KsSlice), (void**)&D.sl));
    AIY_TRY(c->buf("ks_out", sizeof(KsOut), (void**)&D.out));
    AIY_TRY(c->buf("ks_slots", 2 * kDiffSlots * sizeof(unsigned long long), (void**)&D.slots));
    double Pr[16];
    for (int i = 0; i < 4; ++i)
        for (int m = 0; m < 4; ++m) Pr[i * 4 + m] = P[i + m * 4];
    AIY_HIP(hipMemcpyAsync(D.kg, k_grid, nk * sizeof(double), hipMemcpyHostToDevice, c->st));
    AIY_TRY(launch_ks_grid_tables(D.kg, (int)nk, D.kgt, c->st));
    AIY_HIP(hipMemcpyAsync(D.P, Pr, sizeof Pr, hipMemcpyHostToDevice, c->st));
    AIY_HIP(hipMemcpyAsync(D.V, value, nb, hipMemcpyHostToDevice, c->st));
    if (k_opt) AIY_HIP(hipMemcpyAsync(D.kopt, k_opt, nb, hipMemcpyHostToDevice, c->st));
    AIY_HIP(hipMemcpyAsync(D.sl, sl.data(), sl.size() * sizeof(KsSlice), hipMemcpyHostToDevice, c->st));
    AIY_HIP(hipStreamSynchronize(c->st));
    A = KsArgs{};
    A.nk = (int)nk; A.nK = (int)nK; A.node0 = 0; A.n_local = (int)n;
    A.k_grid = D.kg; A.kg_tab = D.kgt; A.P = D.P; A.slice = D.sl;
    A.beta = p.beta; A.k_min = p.k_min; A.k_max = p.k_max;
    A.seg_hint = D.seg;
    return AIY_OK;
}

static int ks_read_slots(HostCtx* c, const unsigned long long* slots, double* d) {
    std::vector<unsigned long long> h(2 * kDiffSlots);
    AIY_HIP(hipMemcpyAsync(h.data(), slots, h.size() * sizeof(unsigned long long),
                           hipMemcpyDeviceToHost, c->st));
    AIY_HIP(hipStreamSynchronize(c->st));
    *d = fold_slots_host(h.data());
    return AIY_OK;
}

}  // namespace aiy

using namespace aiy;

extern "C" {

int ks_policy_improve(const double* value, const double* k_grid, const double* K_grid,
                      const double* B, const double* P, const double* params, int64_t nk,
                      int64_t nK, double* k_opt, int32_t* nfev) {
    if (!k_opt) return fail(AIY_BAD_ARG, "NULL k_opt");
    std::lock_guard<std::mutex> lk(host_mutex());
    HostCtx* c;
    AIY_TRY(get_ctx(4 * nK, nk, 1, &c));
    KsArgs A;
    KsDev D;
    AIY_TRY(ks_stage(c, value, nullptr, k_grid, K_grid, B, P, params, nk, nK, A, D));
    AIY_TRY(launch_ks_slopes(A, D.V, D.dV, c->st));
    AIY_TRY(launch_ks_improve(A, D.V, D.dV, D.kopt, D.nfev, c->st));
    size_t n = (size_t)nk * nK * 4;
    AIY_HIP(hipMemcpyAsync(k_opt, D.kopt, n * sizeof(double), hipMemcpyDeviceToHost, c->st));
    if (nfev) AIY_HIP(hipMemcpyAsync(nfev, D.nfev, n * sizeof(int), hipMemcpyDeviceToHost, c->st));
    AIY_HIP(hipStreamSynchronize(c->st));
    return AIY_OK;
}

int ks_howard(double* value, const double* k_opt, const double* k_grid, const double* K_grid,
              const double* B, const double* P, const double* params, int64_t nk, int64_t nK,
              int64_t steps) {
    if (!k_opt) return fail(AIY_BAD_ARG, "NULL k_opt");
    std::lock_guard<std::mutex> lk(host_mutex());
    HostCtx* c;
    AIY_TRY(get_ctx(4 * nK, nk, 1, &c));
    KsArgs A;
    KsDev D;
    AIY_TRY(ks_stage(c, value, k_opt, k_grid, K_grid, B, P, params, nk, nK, A, D));
    double* cur = D.V;
    double* nxt = D.V2;
    double *dcur = D.dV, *dnxt = D.dV2;
    if (steps > 0) AIY_TRY(launch_ks_slopes(A, cur, dcur, c->st));
    for (int64_t h = 0; h < steps; ++h) {  // one fused launch per sweep (value + next slopes)
        AIY_TRY(launch_ks_howard_slopes(A, cur, dcur, D.kopt, nxt, dnxt, c->st));
        std::swap(cur, nxt);
        std::swap(dcur, dnxt);
    }
    size_t n = (size_t)nk * nK * 4;
    AIY_HIP(hipMemcpyAsync(value, cur, n * sizeof(double), hipMemcpyDeviceToHost, c->st));
    AIY_HIP(hipStreamSynchronize(c->st));
    return AIY_OK;
}

int ks_vfi_solve(double* value, double* k_opt, const double* k_grid, const double* K_grid,
                 const double* B, const double* P, const double* params, int64_t nk,
                 int64_t nK, int64_t howard_steps, double tol, int64_t max_vfi, int n_devices,
                 int64_t* iters, double* rel_diff) {
    if (!k_opt || !iters || !rel_diff) return fail(AIY_BAD_ARG, "NULL argument");
    if (max_vfi < 1 || howard_steps < 0) return fail(AIY_BAD_ARG, "max_vfi >= 1, howard_steps >= 0");
    // the checks ks_stage makes, before the multi-device branch (which does not stage)
    if (!value || !k_grid || !K_grid || !B || !P || !params) return fail(AIY_BAD_ARG, "NULL argument");
    if (nk < 3 || nK < 1) return fail(AIY_BAD_SHAPE, "need k_size >= 3 and K_size >= 1");
    // several devices: (K, Z) slices, 4 Howard sweeps per exchange (ks_multi_host.cpp)
    if (n_devices > 1) return ks_vfi_solve_sharded(value, k_opt, k_grid, K_grid, B, P, params, nk,
                                                   nK, howard_steps, tol, max_vfi, n_devices, 4,
                                                   iters, rel_diff);
    std::lock_guard<std::mutex> lk(host_mutex());
    HostCtx* c;
    AIY_TRY(get_ctx(4 * nK, nk, 1, &c));
    KsArgs A;
    KsDev D;
    AIY_TRY(ks_stage(c, value, k_opt, k_grid, K_grid, B, P, params, nk, nK, A, D));
    A.howard = (int)howard_steps;
    A.max_vfi = (int)max_vfi;
    A.tol = tol;
    size_t n = (size_t)nk * nK * 4;
    if (ks_fused_fits((int)nk, (int)nK)) {
        AIY_TRY(launch_ks_fused(A, D.V, D.kopt, nullptr, D.out, c->st));
        KsOut o;
        AIY_HIP(hipMemcpyAsync(&o, D.out, sizeof o, hipMemcpyDeviceToHost, c->st));
        AIY_HIP(hipMemcpyAsync(value, D.V, n * sizeof(double), hipMemcpyDeviceToHost, c->st));
        AIY_HIP(hipMemcpyAsync(k_opt, D.kopt, n * sizeof(double), hipMemcpyDeviceToHost, c->st));
        AIY_HIP(hipStreamSynchronize(c->st));
        *iters = o.iters;
        *rel_diff = o.rel;
        return AIY_OK;
    }
    double* cur = D.V;
    double* nxt = D.V2;
    double rel = NAN;
    int64_t it;
    for (it = 1; it <= max_vfi; ++it) {
        AIY_HIP(hipMemcpyAsync(D.Vold, cur, n * sizeof(double), hipMemcpyDeviceToDevice, c->st));
        if ((it - 1) % 5 == 0) {
            AIY_TRY(launch_ks_slopes(A, cur, D.dV, c->st));
            AIY_TRY(launch_ks_improve(A, cur, D.dV, D.kopt, nullptr, c->st));
        }
        // improve left the slopes of cur in D.dV only on improvement iterations: rebuild once,
        // then one fused launch per sweep (value + the next sweep's slopes)
        double *dcur = D.dV, *dnxt = D.dV2;
        if (howard_steps > 0) AIY_TRY(launch_ks_slopes(A, cur, dcur, c->st));
        for (int64_t h = 0; h < howard_steps; ++h) {
            AIY_TRY(launch_ks_howard_slopes(A, cur, dcur, D.kopt, nxt, dnxt, c->st));
            std::swap(cur, nxt);
            std::swap(dcur, dnxt);
        }
        AIY_HIP(hipMemsetAsync(D.slots, 0, 2 * kDiffSlots * sizeof(unsigned long long), c->st));
        AIY_TRY(launch_ks_reldiff(A, cur, D.Vold, D.slots, c->st));
        AIY_TRY(ks_read_slots(c, D.slots, &rel));
        if (rel < tol) break;
    }
    if (it > max_vfi) it = max_vfi;
    AIY_HIP(hipMemcpyAsync(value, cur, n * sizeof(double), hipMemcpyDeviceToHost, c->st));
    AIY_HIP(hipMemcpyAsync(k_opt, D.kopt, n * sizeof(double), hipMemcpyDeviceToHost, c->st));
    AIY_HIP(hipStreamSynchronize(c->st));
    *iters = it;
    *rel_diff = rel;
    return AIY_OK;
}

}  // extern "C"
