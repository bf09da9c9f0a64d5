// Config 4 host tier (BASELINE configs[3], SURVEY §8(b) B2 `ge_batch`): excess demand at C
// candidate interest rates in one call — for each candidate the body of one GE step of
// Aiyagari_VFI.m:147-195 (VFI from a common v_old, Monte-Carlo capital supply with the
// candidate's own block of MATLAB's rand stream, K_d = labor·(α/(r+δ))^(1/(1−α))).  The
// candidates are spread over n_devices GPUs of this process, each device solving its share as
// one batched solve (aiy_vfi_solve_batch_dev) and one batched launch of the chains.  The bracket
// logic stays with the caller (the MATLAB script or ge_batch.py), exactly as in the reference.
#include <hip/hip_runtime.h>

#include <cmath>
#include <string>
#include <thread>
#include <vector>

#include "aiy_common.hpp"
#include "host_ctx.hpp"
#include "sim.hpp"
#include "ws.hpp"

namespace aiy {

namespace {
struct GeShare {
    int dev = 0;
    int64_t c0 = 0, cn = 0;  // candidates [c0, c0 + cn)
    HostCtx* ctx = nullptr;
    int rc = AIY_OK;
    std::string err;
};
}  // namespace

// one device's share: stage, batched solve, batched chains, outputs back
static int ge_share(GeShare& sh, const double* r, const double* v_rows, const double* a,
                    const double* s, const double* P, int64_t N, int64_t Na, double alpha,
                    double delta, double beta, double sigma, double tol, int64_t max_iter,
                    int64_t z1, double k1, int64_t T, const double* uniforms, double* k_supply,
                    int64_t* iters) {
    AIY_HIP(hipSetDevice(sh.dev));
    HostCtx* c = sh.ctx;
    const int64_t C = sh.cn;
    const size_t n = (size_t)N * Na, nb = n * sizeof(double);
    double *da, *ds, *dP, *va, *vb, *pk, *dU, *dout;
    int *idx, *dst;
    AIY_TRY(stage_common(c, a, s, P, N, Na, &da, &ds, &dP));
    AIY_TRY(c->buf("ge_va", nb * C, (void**)&va));
    AIY_TRY(c->buf("ge_vb", nb * C, (void**)&vb));
    AIY_TRY(c->buf("ge_pk", nb * C, (void**)&pk));
    AIY_TRY(c->buf("ge_idx", sizeof(int) * n * C, (void**)&idx));
    AIY_TRY(c->buf("ge_U", sizeof(double) * std::max<int64_t>(T - 1, 1) * C, (void**)&dU));
    AIY_TRY(c->buf("ge_out", sizeof(double) * C, (void**)&dout));
    AIY_TRY(c->buf("ge_st", sizeof(int) * C, (void**)&dst));
    // every candidate starts from the same v_old (the caller's warm start)
    AIY_HIP(hipMemcpyAsync(va, v_rows, nb, hipMemcpyHostToDevice, c->st));
    for (int64_t q = 1; q < C; ++q)
        AIY_HIP(hipMemcpyAsync(va + q * n, va, nb, hipMemcpyDeviceToDevice, c->st));
    if (T > 1)
        AIY_HIP(hipMemcpyAsync(dU, uniforms + sh.c0 * (T - 1), sizeof(double) * (T - 1) * C,
                               hipMemcpyHostToDevice, c->st));
    std::vector<double> w(C);
    for (int64_t q = 0; q < C; ++q)  // Aiyagari_VFI.m:149 (w at the candidate r)
        w[q] = (1 - alpha) * std::pow(alpha / (r[sh.c0 + q] + delta), alpha / (1 - alpha));
    std::vector<int> which(C);
    AIY_TRY(bell_solve_batch_dev(c->ws, C, r + sh.c0, w.data(), va, vb, da, ds, dP, beta, sigma,
                                 tol, max_iter, 0, idx, pk, nullptr, iters + sh.c0, which.data(),
                                 c->st));
    SimArgs S{};
    S.N = (int)N; S.Na = (int)Na; S.T = (int)T; S.z1 = (int)(z1 - 1); S.k1 = k1;
    S.pol = pk; S.zs = (size_t)Na; S.as = 1; S.a = da; S.P = dP; S.U = dU;
    S.out = dout; S.status = dst;
    S.C = (int)C; S.pcs = n; S.ucs = (size_t)std::max<int64_t>(T - 1, 0);
    S.par = c->ws->sim_par;
    if (S.par != 0)  // the speculative-segment chains' scratch (paths, state paths, flags)
        AIY_TRY(c->buf("ge_kscr", sim_par_scratch_bytes(T, C), (void**)&S.kscr));
    AIY_TRY(launch_sim_capital(S, c->st));
    std::vector<int> status(C);
    AIY_HIP(hipMemcpyAsync(k_supply + sh.c0, dout, sizeof(double) * C, hipMemcpyDeviceToHost, c->st));
    AIY_HIP(hipMemcpyAsync(status.data(), dst, sizeof(int) * C, hipMemcpyDeviceToHost, c->st));
    AIY_HIP(hipStreamSynchronize(c->st));
    for (int64_t q = 0; q < C; ++q)
        if (status[q]) return fail(AIY_FIND_EMPTY, "candidate %lld: find(rand < cumsum(P(z,:))) empty",
                                   (long long)(sh.c0 + q + 1));
    return AIY_OK;
}

}  // namespace aiy

using namespace aiy;

extern "C" {

int aiy_ge_batch(const double* r, int64_t C, const double* v_start, const double* a_grid,
                 const double* s, const double* P, int64_t N, int64_t Na, double alpha,
                 double delta, double beta, double sigma, double labor, double tol,
                 int64_t max_iter, int64_t z1, double k1, int64_t T, const double* uniforms,
                 int n_devices, double* k_supply, double* k_demand, int64_t* iters) {
    if (!r || !v_start || !s || !P || !k_supply || !k_demand || !iters || (T > 1 && !uniforms))
        return fail(AIY_BAD_ARG, "NULL argument");
    if (C < 1 || N < 1 || Na < 2) return fail(AIY_BAD_SHAPE, "need C >= 1, N >= 1, Na >= 2");
    if (T < 1 || T > (1ll << 31) - 1) return fail(AIY_BAD_SHAPE, "T must be in [1, 2^31)");
    if (z1 < 1 || z1 > N) return fail(AIY_BAD_ARG, "z1 (1-based) out of range");
    if (max_iter < 1) return fail(AIY_BAD_ARG, "max_iter must be >= 1");
    AIY_TRY(check_grid_strict(a_grid, Na));
    for (int64_t q = 0; q < C; ++q)
        if (!std::isfinite(r[q]) || r[q] + delta <= 0)
            return fail(AIY_BAD_ARG, "candidate %lld: r must be finite with r + delta > 0", (long long)q + 1);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1)
        return fail(AIY_NO_DEVICE, "no HIP device visible");
    const int nd = (int)std::min<int64_t>(std::max(n_devices, 1), std::min<int64_t>(ndev, C));
    std::vector<double> rows((size_t)N * Na);
    cm_to_rows(v_start, N, Na, rows.data());
    std::lock_guard<std::mutex> lk(host_mutex());
    int cur = 0;
    (void)hipGetDevice(&cur);
    std::vector<GeShare> sh(nd);
    for (int d = 0; d < nd; ++d) {  // contiguous shares, the first C % nd one larger
        sh[d].dev = (cur + d) % ndev;
        sh[d].c0 = d * (C / nd) + std::min<int64_t>(d, C % nd);
        sh[d].cn = C / nd + (d < C % nd ? 1 : 0);
        (void)hipSetDevice(sh[d].dev);
        int rc = get_ctx(N, Na, 1, &sh[d].ctx);
        if (rc != AIY_OK) {
            (void)hipSetDevice(cur);
            return rc;
        }
    }
    auto run = [&](GeShare& g) {
        g.rc = ge_share(g, r, rows.data(), a_grid, s, P, N, Na, alpha, delta, beta, sigma, tol,
                        max_iter, z1, k1, T, uniforms, k_supply, iters);
        if (g.rc != AIY_OK) g.err = aiy_last_error();
    };
    if (nd == 1) {
        run(sh[0]);
    } else {  // one host thread per device: the shares run concurrently
        std::vector<std::thread> th;
        for (auto& g : sh) th.emplace_back(run, std::ref(g));
        for (auto& t : th) t.join();
    }
    (void)hipSetDevice(cur);
    for (auto& g : sh)
        if (g.rc != AIY_OK) return fail(g.rc, "%s", g.err.c_str());
    for (int64_t q = 0; q < C; ++q)  // Aiyagari_VFI.m:195
        k_demand[q] = labor * std::pow(alpha / (r[q] + delta), 1 / (1 - alpha));
    return AIY_OK;
}

}  // extern "C"
