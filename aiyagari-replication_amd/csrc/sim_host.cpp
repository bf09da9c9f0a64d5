// A9 entry points: aiy_sim_capital (MATLAB layouts, synchronous) and aiy_sim_capital_dev.
#include <hip/hip_runtime.h>

#include <cstring>
#include <mutex>
#include <vector>

#include "aiy_common.hpp"
#include "host_ctx.hpp"
#include "sim.hpp"
#include "ws.hpp"

namespace aiy {

int sim_capital_dev(const double* pol, size_t zs, size_t as, const double* a, const double* P,
                    int64_t N, int64_t Na, int64_t z1, double k1, int64_t T, const double* U,
                    double* out, double* sim_k, int* sim_z, int* status, hipStream_t st,
                    bool exclusive = false, double* kscr = nullptr, int par = -1) {
    if (!pol || !a || !P || !out || !status || (T > 1 && !U))
        return fail(AIY_BAD_ARG, "NULL argument");
    if (T < 1 || T > (1ll << 31) - 1) return fail(AIY_BAD_SHAPE, "T must be in [1, 2^31)");
    if (z1 < 0 || z1 >= N) return fail(AIY_BAD_ARG, "z1 out of range");
    SimArgs A{};
    A.N = (int)N; A.Na = (int)Na; A.T = (int)T; A.z1 = (int)z1; A.k1 = k1;
    A.pol = pol; A.zs = zs; A.as = as; A.a = a; A.P = P; A.U = U;
    A.out = out; A.sim_k = sim_k; A.sim_z = sim_z; A.status = status;
    A.exclusive = exclusive;
    A.kscr = kscr;
    A.par = par;
    return launch_sim_capital(A, st);
}

}  // namespace aiy

using namespace aiy;

extern "C" {

int aiy_sim_capital(const double* policy_k, int vfi_layout, const double* a_grid,
                    const double* P, int64_t N, int64_t Na, int64_t z1, double k1, int64_t T,
                    const double* uniforms, double* k_supply, double* sim_k, int32_t* sim_z) {
    if (!policy_k || !P || !k_supply) return fail(AIY_BAD_ARG, "NULL argument");
    if (N < 1 || Na < 2) return fail(AIY_BAD_SHAPE, "need N >= 1 and Na >= 2");
    AIY_TRY(check_grid_strict(a_grid, Na));  // interp1 (:113) rejects repeated points
    std::lock_guard<std::mutex> lk(host_mutex());
    HostCtx* c;
    AIY_TRY(get_ctx(N, Na, 1, &c));
    double *da, *dP, *dpol, *dU, *dout, *dk = nullptr;
    int *dst, *dz = nullptr;
    // P rows: reuse stage_common with a dummy s (only a and P are used here)
    std::vector<double> s1(N, 1.0);
    double* ds;
    AIY_TRY(stage_common(c, a_grid, s1.data(), P, N, Na, &da, &ds, &dP));
    size_t nb = sizeof(double) * N * Na;
    AIY_TRY(c->buf("sim_pol", nb, (void**)&dpol));
    AIY_TRY(c->buf("sim_U", sizeof(double) * (T > 1 ? T - 1 : 1), (void**)&dU));
    AIY_TRY(c->buf("sim_out", sizeof(double) + 16, (void**)&dout));
    AIY_TRY(c->buf("sim_status", sizeof(int) * 4, (void**)&dst));
    if (sim_k) AIY_TRY(c->buf("sim_k", sizeof(double) * T, (void**)&dk));
    if (sim_z) AIY_TRY(c->buf("sim_z", sizeof(int) * T, (void**)&dz));
    AIY_HIP(hipMemcpyAsync(dpol, policy_k, nb, hipMemcpyHostToDevice, c->st));
    if (T > 1)
        AIY_HIP(hipMemcpyAsync(dU, uniforms, sizeof(double) * (T - 1), hipMemcpyHostToDevice, c->st));
    // MATLAB layouts: VFI policy_k is N x Na (z stride 1, a stride N); EGM is Na x N.
    size_t zs = vfi_layout ? 1 : (size_t)Na, as = vfi_layout ? (size_t)N : 1;
    double* dks = nullptr;  // the speculative-segment chain's path scratch
    AIY_TRY(c->buf("sim_kscr", sim_par_scratch_bytes(T, 1), (void**)&dks));
    AIY_TRY(sim_capital_dev(dpol, zs, as, da, dP, N, Na, z1 - 1, k1, T, dU, dout, dk, dz, dst,
                            c->st, false, dks, c->ws ? c->ws->sim_par : -1));
    double out;
    int status;
    AIY_HIP(hipMemcpyAsync(&out, dout, sizeof(double), hipMemcpyDeviceToHost, c->st));
    AIY_HIP(hipMemcpyAsync(&status, dst, sizeof(int), hipMemcpyDeviceToHost, c->st));
    if (sim_k) AIY_HIP(hipMemcpyAsync(sim_k, dk, sizeof(double) * T, hipMemcpyDeviceToHost, c->st));
    std::vector<int> zb;
    if (sim_z) {
        zb.resize(T);
        AIY_HIP(hipMemcpyAsync(zb.data(), dz, sizeof(int) * T, hipMemcpyDeviceToHost, c->st));
    }
    AIY_HIP(hipStreamSynchronize(c->st));
    if (status != 0)
        return fail(AIY_FIND_EMPTY, "rand >= cumsum(P(z,:)) for every column: MATLAB's "
                                    "find(...,1) is empty and the assignment at "
                                    "Aiyagari_VFI.m:106 errors");
    if (sim_z)
        for (int64_t t = 0; t < T; ++t) sim_z[t] = zb[t] + 1;
    *k_supply = out;
    return AIY_OK;
}

int aiy_sim_capital_dev(aiy_ws* ws, const double* policy_rows, const double* a_grid,
                        const double* P, int64_t z1, double k1, int64_t T,
                        const double* uniforms, double* k_supply, double* sim_k,
                        int32_t* sim_z, int32_t* status, void* stream) {
    if (!ws) return fail(AIY_BAD_ARG, "NULL workspace");
    const size_t kb = sim_par_scratch_bytes(T, 1);
    if (T >= 2 && ws->sim_par != 0 && ws->sim_kcap < kb) {  // the chain's scratch (per workspace)
        if (ws->sim_kbuf) AIY_HIP(hipFree(ws->sim_kbuf));
        ws->sim_kbuf = nullptr;
        ws->sim_kcap = 0;
        AIY_HIP(hipMalloc((void**)&ws->sim_kbuf, kb));
        ws->sim_kcap = kb;
    }
    return sim_capital_dev(policy_rows, (size_t)ws->Na, 1, a_grid, P, ws->N, ws->Na, z1, k1, T,
                           uniforms, k_supply, sim_k, sim_z, status, (hipStream_t)stream,
                           ws->cu_exclusive, ws->sim_par != 0 ? ws->sim_kbuf : nullptr,
                           ws->sim_par);
}

int aiy_ws_set_sim(aiy_ws* ws, int mode) {
    if (!ws) return fail(AIY_BAD_ARG, "NULL workspace");
    if (mode < -1 || mode > 2) return fail(AIY_BAD_ARG, "mode: -1 (by size), 0, 1 or 2");
    ws->sim_par = mode;
    return AIY_OK;
}

}  // extern "C"
