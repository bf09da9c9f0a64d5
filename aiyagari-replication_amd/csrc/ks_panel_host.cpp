// F3 / F2 entry points: ks_shocks, ks_simulate_capital (MATLAB layouts, synchronous) and
// their device tiers ks_shocks_dev, ks_simulate_capital_dev.
#include <hip/hip_runtime.h>

#include <cmath>
#include <mutex>
#include <vector>

#include "aiy_common.hpp"
#include "host_ctx.hpp"
#include "ks_panel.hpp"

namespace aiy {

// Krusell_Smith_VFI.m:24-45, the same expressions in the same order as the script (the
// durations 8, 1.5, 2.5 and the ratios 1.25, 0.75 are literals there, not parameters).
static void shock_probs(double ug, double ub, ShockArgs& A) {
    const double pgg = 1 - 1 / 8.0, pbb = 1 - 1 / 8.0;
    const double p00_gg = 1 - 1 / 1.5, p00_bb = 1 - 1 / 2.5;
    const double p00_gb = 1.25 * p00_bb, p00_bg = 0.75 * p00_gg;
    const double p01_gg = 1 - p00_gg, p01_bb = 1 - p00_bb;
    const double p01_gb = 1 - p00_gb, p01_bg = 1 - p00_bg;
    const double p10_gg = (ug - ug * p00_gg) / (1 - ug);
    const double p10_bb = (ub - ub * p00_bb) / (1 - ub);
    const double p10_gb = (ub - ug * p00_gb) / (1 - ug);
    const double p10_bg = (ug - ub * p00_bg) / (1 - ub);
    const double p11_gg = 1 - p10_gg, p11_bb = 1 - p10_bb;
    const double p11_gb = 1 - p10_gb, p11_bg = 1 - p10_bg;
    A.pgg = pgg;
    A.pbb = pbb;
    A.ug = ug;
    // [cur_z][prev_z][prev_e]; (0,0) gg, (0,1) bg, (1,0) gb, (1,1) bb (:78-86)
    const double p11[4] = {p11_gg, p11_bg, p11_gb, p11_bb};
    const double p01[4] = {p01_gg, p01_bg, p01_gb, p01_bb};
    for (int q = 0; q < 4; ++q) {
        A.thr[q * 2 + 0] = p11[q];
        A.thr[q * 2 + 1] = p01[q];
    }
}

static int check_panel_shape(int64_t T, int64_t pop) {
    if (T < 1 || T > (1ll << 30)) return fail(AIY_BAD_SHAPE, "T must be in [1, 2^30]");
    if (pop < 1 || pop > (1ll << 31) - 1) return fail(AIY_BAD_SHAPE, "population must be in [1, 2^31)");
    return AIY_OK;
}

int shocks_dev(int64_t T, int64_t pop, const double* U, const double* params, int8_t* zi,
               int8_t* eps, int64_t ts, int64_t is, hipStream_t st) {
    if (!U || !params || !zi || !eps) return fail(AIY_BAD_ARG, "NULL argument");
    AIY_TRY(check_panel_shape(T, pop));
    const double ug = params[5], ub = params[6];
    if (!(ug > 0 && ug < 1 && ub > 0 && ub < 1))
        return fail(AIY_BAD_ARG, "ug and ub must lie in (0, 1)");
    ShockArgs A{};
    A.T = (int)T;
    A.pop = (int)pop;
    shock_probs(ug, ub, A);
    A.U = U;
    A.zi = zi;
    A.eps = eps;
    A.ts = ts;
    A.is = is;
    return launch_ks_shocks(A, st);
}

int panel_dev(int64_t nk, int64_t nK, const double* k_grid, const double* K_grid,
              const double* k_opt, int64_t T, int64_t pop, const int8_t* zi, const int8_t* eps,
              int64_t ts, int64_t is, double* k_pop, double* K_ts, double* scratch,
              hipStream_t st) {
    if (!k_grid || !K_grid || !k_opt || !zi || !eps || !k_pop || !K_ts || !scratch)
        return fail(AIY_BAD_ARG, "NULL argument");
    if (nk < 2 || nK < 2 || nk > (1 << 24) || nK > (1 << 24))
        return fail(AIY_BAD_SHAPE, "need 2 <= k_size, K_size <= 2^24");
    AIY_TRY(check_panel_shape(T, pop));
    PanelArgs A{};
    A.nk = (int)nk;
    A.nK = (int)nK;
    A.T = (int)T;
    A.pop = (int)pop;
    A.G = panel_blocks(pop);
    A.k_grid = k_grid;
    A.K_grid = K_grid;
    A.k_opt = k_opt;
    A.zi = zi;
    A.eps = eps;
    A.ts = ts;
    A.is = is;
    A.k_pop = k_pop;
    A.K_ts = K_ts;
    A.part = scratch;
    return launch_ks_panel(A, st);
}

}  // namespace aiy

using namespace aiy;

extern "C" {

int64_t ks_shock_draws(int64_t T, int64_t population) {
    return (T - 1) + population + (T - 1) * population;
}

int64_t ks_panel_scratch_bytes(int64_t population) {
    return (int64_t)(2 * sizeof(double)) * panel_blocks(population);
}

int ks_shocks_dev(int64_t T, int64_t population, const double* uniforms, const double* params,
                  int8_t* zi, int8_t* eps, void* stream) {
    return shocks_dev(T, population, uniforms, params, zi, eps, population, 1,
                      (hipStream_t)stream);
}

int ks_simulate_capital_dev(int64_t nk, int64_t nK, const double* k_grid, const double* K_grid,
                            const double* k_opt, int64_t T, int64_t population,
                            const int8_t* zi, const int8_t* eps, double* k_population,
                            double* K_ts, void* scratch, void* stream) {
    return panel_dev(nk, nK, k_grid, K_grid, k_opt, T, population, zi, eps, population, 1,
                     k_population, K_ts, (double*)scratch, (hipStream_t)stream);
}

int ks_shocks(int64_t T, int64_t population, const double* uniforms, const double* params,
              double* zi_shock, double* epsi_shock) {
    if (!uniforms || !params || !zi_shock || !epsi_shock) return fail(AIY_BAD_ARG, "NULL argument");
    AIY_TRY(check_panel_shape(T, population));
    std::lock_guard<std::mutex> lk(host_mutex());
    HostCtx* c;
    AIY_TRY(get_ctx(1, 2, 1, &c));
    const int64_t nU = ks_shock_draws(T, population);
    double* dU;
    int8_t *dz, *de;
    AIY_TRY(c->buf("ksp_U", sizeof(double) * nU, (void**)&dU));
    AIY_TRY(c->buf("ksp_zi", (size_t)T, (void**)&dz));
    AIY_TRY(c->buf("ksp_eps", (size_t)T * population, (void**)&de));
    AIY_HIP(hipMemcpyAsync(dU, uniforms, sizeof(double) * nU, hipMemcpyHostToDevice, c->st));
    // MATLAB epsi_shock is T x population column-major: (t, i) at t + T*i
    AIY_TRY(shocks_dev(T, population, dU, params, dz, de, 1, T, c->st));
    std::vector<int8_t> hz(T), he((size_t)T * population);
    AIY_HIP(hipMemcpyAsync(hz.data(), dz, (size_t)T, hipMemcpyDeviceToHost, c->st));
    AIY_HIP(hipMemcpyAsync(he.data(), de, he.size(), hipMemcpyDeviceToHost, c->st));
    AIY_HIP(hipStreamSynchronize(c->st));
    for (int64_t t = 0; t < T; ++t) zi_shock[t] = hz[t];           // after :68 (0 good)
    for (size_t q = 0; q < he.size(); ++q) epsi_shock[q] = he[q] + 1;  // 1 employed, 2 not
    return AIY_OK;
}

int ks_simulate_capital(const double* k_opt, const double* k_grid, const double* K_grid,
                        int64_t nk, int64_t nK, const double* zi_shock,
                        const double* epsi_shock, int64_t T, int64_t population,
                        double* k_population, double* K_ts) {
    if (!k_opt || !zi_shock || !epsi_shock || !k_population || !K_ts)
        return fail(AIY_BAD_ARG, "NULL argument");
    AIY_TRY(check_panel_shape(T, population));
    if (nk < 2 || nK < 2) return fail(AIY_BAD_SHAPE, "need k_size, K_size >= 2");
    AIY_TRY(check_grid_strict(k_grid, nk));  // griddedInterpolant rejects repeated points
    AIY_TRY(check_grid_strict(K_grid, nK));
    // MATLAB's lookup (:227-231) maps only z in z_grid and eps in eps_grid; other codes error
    std::vector<int8_t> hz(T), he((size_t)T * population);
    for (int64_t t = 0; t < T; ++t) {
        if (zi_shock[t] != 0 && zi_shock[t] != 1)
            return fail(AIY_BAD_ARG, "zi_shock must hold 0 (good) or 1 (bad)");
        hz[t] = (int8_t)zi_shock[t];
    }
    for (size_t q = 0; q < he.size(); ++q) {
        if (epsi_shock[q] != 1 && epsi_shock[q] != 2)
            return fail(AIY_BAD_ARG, "epsi_shock must hold 1 (employed) or 2 (unemployed)");
        he[q] = (int8_t)(epsi_shock[q] - 1);
    }
    for (int64_t i = 0; i < population; ++i)
        if (!std::isfinite(k_population[i])) return fail(AIY_NON_FINITE, "non-finite k_population");
    std::lock_guard<std::mutex> lk(host_mutex());
    HostCtx* c;
    AIY_TRY(get_ctx(4 * nK, nk, 1, &c));
    const size_t nko = (size_t)nk * nK * 4;
    double *dko, *dkg, *dKg, *dkp, *dKts, *dpart;
    int8_t *dz, *de;
    AIY_TRY(c->buf("ksp_kopt", sizeof(double) * nko, (void**)&dko));
    AIY_TRY(c->buf("ksp_kg", sizeof(double) * nk, (void**)&dkg));
    AIY_TRY(c->buf("ksp_Kg", sizeof(double) * nK, (void**)&dKg));
    AIY_TRY(c->buf("ksp_kpop", sizeof(double) * population, (void**)&dkp));
    AIY_TRY(c->buf("ksp_Kts", sizeof(double) * T, (void**)&dKts));
    AIY_TRY(c->buf("ksp_part", (size_t)ks_panel_scratch_bytes(population), (void**)&dpart));
    AIY_TRY(c->buf("ksp_zi", (size_t)T, (void**)&dz));
    AIY_TRY(c->buf("ksp_eps", he.size(), (void**)&de));
    AIY_HIP(hipMemcpyAsync(dko, k_opt, sizeof(double) * nko, hipMemcpyHostToDevice, c->st));
    AIY_HIP(hipMemcpyAsync(dkg, k_grid, sizeof(double) * nk, hipMemcpyHostToDevice, c->st));
    AIY_HIP(hipMemcpyAsync(dKg, K_grid, sizeof(double) * nK, hipMemcpyHostToDevice, c->st));
    AIY_HIP(hipMemcpyAsync(dkp, k_population, sizeof(double) * population, hipMemcpyHostToDevice, c->st));
    AIY_HIP(hipMemcpyAsync(dz, hz.data(), (size_t)T, hipMemcpyHostToDevice, c->st));
    AIY_HIP(hipMemcpyAsync(de, he.data(), he.size(), hipMemcpyHostToDevice, c->st));
    AIY_TRY(panel_dev(nk, nK, dkg, dKg, dko, T, population, dz, de, 1, T, dkp, dKts, dpart, c->st));
    AIY_HIP(hipMemcpyAsync(k_population, dkp, sizeof(double) * population, hipMemcpyDeviceToHost, c->st));
    AIY_HIP(hipMemcpyAsync(K_ts, dKts, sizeof(double) * T, hipMemcpyDeviceToHost, c->st));
    AIY_HIP(hipStreamSynchronize(c->st));
    return AIY_OK;
}

}  // extern "C"
