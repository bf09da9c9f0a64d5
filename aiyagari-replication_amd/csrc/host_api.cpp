// Host tier of the C ABI: MATLAB column-major arrays in and out, synchronous.  Each call
// stages its inputs into library-owned device buffers (cached per shape), runs the device
// tier and copies the outputs back in the layout of the variables the call replaces.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <tuple>
#include <vector>

#include "aiy_common.hpp"
#include "host_ctx.hpp"
#include "ws.hpp"

namespace aiy {

static std::mutex g_mu;
static std::map<std::tuple<int, int64_t, int64_t, int64_t>, std::unique_ptr<HostCtx>> g_ctx;

HostCtx::~HostCtx() {
    for (auto& kv : bufs) (void)hipFree(kv.second.first);
    if (ws) aiy_ws_destroy(ws);
    if (st) (void)hipStreamDestroy(st);
}

int HostCtx::buf(const char* name, size_t bytes, void** out) {
    auto it = bufs.find(name);
    if (it != bufs.end() && it->second.second >= bytes) {
        *out = it->second.first;
        return AIY_OK;
    }
    if (it != bufs.end()) {
        (void)hipFree(it->second.first);
        bufs.erase(it);
    }
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, bytes ? bytes : 8);
    if (e != hipSuccess) return fail(AIY_NO_MEMORY, "hipMalloc(%zu) failed", bytes);
    bufs[name] = {p, bytes};
    *out = p;
    return AIY_OK;
}

int get_ctx(int64_t N, int64_t Na, int64_t Nl, HostCtx** out) {
    int dev = 0;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1)
        return fail(AIY_NO_DEVICE, "no HIP device visible");
    (void)hipGetDevice(&dev);
    auto key = std::make_tuple(dev, N, Na, Nl);
    auto it = g_ctx.find(key);
    if (it != g_ctx.end()) {
        *out = it->second.get();
        return AIY_OK;
    }
    auto ctx = std::make_unique<HostCtx>();
    AIY_TRY(aiy_ws_create(N, Na, Nl, &ctx->ws));
    AIY_HIP(hipStreamCreateWithFlags(&ctx->st, hipStreamNonBlocking));
    *out = ctx.get();
    g_ctx[key] = std::move(ctx);
    return AIY_OK;
}

std::mutex& host_mutex() { return g_mu; }

// MATLAB N x Na column-major -> [N][Na] row-major
void cm_to_rows(const double* cm, int64_t N, int64_t Na, double* rows) {
    for (int64_t j = 0; j < Na; ++j)
        for (int64_t i = 0; i < N; ++i) rows[i * Na + j] = cm[i + j * N];
}
void rows_to_cm(const double* rows, int64_t N, int64_t Na, double* cm) {
    for (int64_t j = 0; j < Na; ++j)
        for (int64_t i = 0; i < N; ++i) cm[i + j * N] = rows[i * Na + j];
}

int check_grid(const double* a, int64_t Na) {
    if (!a) return fail(AIY_BAD_ARG, "a_grid is NULL");
    for (int64_t k = 0; k < Na; ++k)
        if (!std::isfinite(a[k])) return fail(AIY_NON_FINITE, "a_grid(%lld) is not finite", (long long)k + 1);
    for (int64_t k = 1; k < Na; ++k)
        if (a[k] < a[k - 1])
            return fail(AIY_BAD_ARG, "a_grid must be non-decreasing (a_grid(%lld) < a_grid(%lld))",
                        (long long)k + 1, (long long)k);
    return AIY_OK;
}

// interp1 and griddedInterpolant reject repeated grid points: the interpolating entry points
// (simulation, histogram lottery, KS panel) need a strictly increasing grid, else they would
// divide by a[k+1] - a[k] = 0 (MATLAB raises an error there)
int check_grid_strict(const double* a, int64_t Na) {
    AIY_TRY(check_grid(a, Na));
    for (int64_t k = 1; k < Na; ++k)
        if (!(a[k] > a[k - 1]))
            return fail(AIY_BAD_ARG, "grid must be strictly increasing (point %lld repeats point %lld)",
                        (long long)k + 1, (long long)k);
    return AIY_OK;
}

// stage the common Aiyagari inputs (a_grid, s, P) on the device; P transposed to row-major
int stage_common(HostCtx* c, const double* a, const double* s, const double* P, int64_t N,
                 int64_t Na, double** da, double** ds, double** dP) {
    AIY_TRY(c->buf("a", sizeof(double) * Na, (void**)da));
    AIY_TRY(c->buf("s", sizeof(double) * N, (void**)ds));
    AIY_TRY(c->buf("P", sizeof(double) * N * N, (void**)dP));
    std::vector<double> Pr(N * N);
    for (int64_t i = 0; i < N; ++i)
        for (int64_t m = 0; m < N; ++m) Pr[i * N + m] = P[i + m * N];
    AIY_HIP(hipMemcpyAsync(*da, a, sizeof(double) * Na, hipMemcpyHostToDevice, c->st));
    AIY_HIP(hipMemcpyAsync(*ds, s, sizeof(double) * N, hipMemcpyHostToDevice, c->st));
    AIY_HIP(hipMemcpyAsync(*dP, Pr.data(), sizeof(double) * N * N, hipMemcpyHostToDevice, c->st));
    AIY_HIP(hipStreamSynchronize(c->st));
    aiy_ws_invalidate(c->ws);  // the staged a/s contents may differ from the last call
    return AIY_OK;
}

static int vfi_host(const double* v_old_cm, const double* a, const double* s, const double* P,
                    int64_t N, int64_t Na, double r, double w, double beta, double sigma,
                    bool solve, double tol, int64_t max_iter, double* v_old_out_cm,
                    double* v_new_cm, double* pk_cm, double* pc_cm, int32_t* idx_cm,
                    int64_t* iters) {
    if (!v_old_cm || !s || !P || !v_new_cm || !pk_cm || !pc_cm)
        return fail(AIY_BAD_ARG, "NULL argument");
    if (N < 1 || Na < 2) return fail(AIY_BAD_SHAPE, "need N >= 1 and Na >= 2");
    AIY_TRY(check_grid(a, Na));
    std::lock_guard<std::mutex> lk(g_mu);
    HostCtx* c;
    AIY_TRY(get_ctx(N, Na, 1, &c));
    double *da, *ds, *dP, *dva, *dvb, *dpk, *dpc;
    int* didx;
    AIY_TRY(stage_common(c, a, s, P, N, Na, &da, &ds, &dP));
    size_t nb = sizeof(double) * N * Na;
    AIY_TRY(c->buf("va", nb, (void**)&dva));
    AIY_TRY(c->buf("vb", nb, (void**)&dvb));
    AIY_TRY(c->buf("pk", nb, (void**)&dpk));
    AIY_TRY(c->buf("pc", nb, (void**)&dpc));
    AIY_TRY(c->buf("idx", sizeof(int) * N * Na, (void**)&didx));
    std::vector<double> rows(N * Na), tmp(N * Na);
    cm_to_rows(v_old_cm, N, Na, rows.data());
    AIY_HIP(hipMemcpyAsync(dva, rows.data(), nb, hipMemcpyHostToDevice, c->st));
    int out_new = 1;
    BellCall bc{};
    bc.a = da; bc.s = ds; bc.P = dP; bc.r = r; bc.w = w; bc.beta = beta; bc.sigma = sigma;
    bc.idx = didx; bc.pk = dpk; bc.pc = dpc;
    if (solve) {
        AIY_TRY(bell_solve_dev(c->ws, bc, dva, dvb, tol, max_iter, iters, &out_new, c->st));
    } else {
        bc.v_old = dva;
        bc.v_new = dvb;
        AIY_TRY(bell_sweep_dev(c->ws, bc, c->st));
    }
    double* dnew = out_new ? dvb : dva;
    double* dold = out_new ? dva : dvb;
    auto back = [&](const double* d, double* cm) -> int {
        AIY_HIP(hipMemcpyAsync(tmp.data(), d, nb, hipMemcpyDeviceToHost, c->st));
        AIY_HIP(hipStreamSynchronize(c->st));
        rows_to_cm(tmp.data(), N, Na, cm);
        return AIY_OK;
    };
    AIY_TRY(back(dnew, v_new_cm));
    AIY_TRY(back(dpk, pk_cm));
    AIY_TRY(back(dpc, pc_cm));
    if (solve && v_old_out_cm) AIY_TRY(back(dold, v_old_out_cm));
    if (idx_cm) {
        std::vector<int> ib(N * Na);
        AIY_HIP(hipMemcpyAsync(ib.data(), didx, sizeof(int) * N * Na, hipMemcpyDeviceToHost, c->st));
        AIY_HIP(hipStreamSynchronize(c->st));
        for (int64_t j = 0; j < Na; ++j)
            for (int64_t i = 0; i < N; ++i) idx_cm[i + j * N] = ib[i * Na + j] + 1;
    }
    return AIY_OK;
}

// A3 host tier: VFI arrays N x Na column-major; v_new and policies in/out.
static int labor_host(const double* v_old_cm, const double* a, const double* s, const double* P,
                      const double* L, int64_t N, int64_t Na, int64_t Nl, double r, double w,
                      double beta, double sigma, double psi, double eta, bool solve, double tol,
                      int64_t max_iter, double* v_old_out_cm, double* v_new_cm, double* pk_cm,
                      double* pl_cm, double* pc_cm, int32_t* lin_cm, int64_t* iters) {
    if (!v_old_cm || !s || !P || !L || !v_new_cm || !pk_cm || !pl_cm || !pc_cm)
        return fail(AIY_BAD_ARG, "NULL argument");
    if (N < 1 || Na < 2 || Nl < 1) return fail(AIY_BAD_SHAPE, "need N >= 1, Na >= 2, Nl >= 1");
    AIY_TRY(check_grid(a, Na));
    std::lock_guard<std::mutex> lk(g_mu);
    HostCtx* c;
    AIY_TRY(get_ctx(N, Na, Nl, &c));
    double *da, *ds, *dP, *dva, *dvb, *dpk, *dpc, *dpl, *dL;
    int* dlin;
    AIY_TRY(stage_common(c, a, s, P, N, Na, &da, &ds, &dP));
    size_t nb = sizeof(double) * N * Na;
    AIY_TRY(c->buf("va", nb, (void**)&dva));
    AIY_TRY(c->buf("vb", nb, (void**)&dvb));
    AIY_TRY(c->buf("pk", nb, (void**)&dpk));
    AIY_TRY(c->buf("pc", nb, (void**)&dpc));
    AIY_TRY(c->buf("pl", nb, (void**)&dpl));
    AIY_TRY(c->buf("L", sizeof(double) * Nl, (void**)&dL));
    AIY_TRY(c->buf("idx", sizeof(int) * N * Na, (void**)&dlin));
    std::vector<double> rows(N * Na), tmp(N * Na);
    std::vector<int> ib(N * Na);
    auto up = [&](const double* cm, double* d) -> int {
        cm_to_rows(cm, N, Na, rows.data());
        AIY_HIP(hipMemcpyAsync(d, rows.data(), nb, hipMemcpyHostToDevice, c->st));
        AIY_HIP(hipStreamSynchronize(c->st));
        return AIY_OK;
    };
    AIY_TRY(up(v_old_cm, dva));
    AIY_TRY(up(v_new_cm, dvb));  // in/out: states without a feasible choice keep these
    AIY_TRY(up(pk_cm, dpk));
    AIY_TRY(up(pl_cm, dpl));
    AIY_TRY(up(pc_cm, dpc));
    for (int64_t j = 0; j < Na; ++j)
        for (int64_t i = 0; i < N; ++i) ib[i * Na + j] = lin_cm ? lin_cm[i + j * N] - 1 : 0;
    AIY_HIP(hipMemcpyAsync(dlin, ib.data(), sizeof(int) * N * Na, hipMemcpyHostToDevice, c->st));
    AIY_HIP(hipMemcpyAsync(dL, L, sizeof(double) * Nl, hipMemcpyHostToDevice, c->st));
    int out_new = 1;
    BellCall bc{};
    bc.labor = true; bc.Nl = Nl; bc.L = dL; bc.psi = psi; bc.eta = eta;
    bc.a = da; bc.s = ds; bc.P = dP; bc.r = r; bc.w = w; bc.beta = beta; bc.sigma = sigma;
    bc.idx = dlin; bc.pk = dpk; bc.pl = dpl; bc.pc = dpc;
    if (solve) {
        // the MATLAB loop keeps v_new across sweeps; at sweep 1 the ping-pong partner of
        // v_old must hold the incoming v_new, which merge copies from v_old where needed
        AIY_TRY(bell_solve_dev(c->ws, bc, dva, dvb, tol, max_iter, iters, &out_new, c->st));
    } else {
        bc.v_old = dva;
        bc.v_new = dvb;
        AIY_TRY(bell_sweep_dev(c->ws, bc, c->st));
    }
    double* dnew = out_new ? dvb : dva;
    double* dold = out_new ? dva : dvb;
    auto back = [&](const double* d, double* cm) -> int {
        AIY_HIP(hipMemcpyAsync(tmp.data(), d, nb, hipMemcpyDeviceToHost, c->st));
        AIY_HIP(hipStreamSynchronize(c->st));
        rows_to_cm(tmp.data(), N, Na, cm);
        return AIY_OK;
    };
    AIY_TRY(back(dnew, v_new_cm));
    AIY_TRY(back(dpk, pk_cm));
    AIY_TRY(back(dpl, pl_cm));
    AIY_TRY(back(dpc, pc_cm));
    if (solve && v_old_out_cm) AIY_TRY(back(dold, v_old_out_cm));
    if (lin_cm) {
        AIY_HIP(hipMemcpyAsync(ib.data(), dlin, sizeof(int) * N * Na, hipMemcpyDeviceToHost, c->st));
        AIY_HIP(hipStreamSynchronize(c->st));
        for (int64_t j = 0; j < Na; ++j)
            for (int64_t i = 0; i < N; ++i) lin_cm[i + j * N] = ib[i * Na + j] + 1;
    }
    return AIY_OK;
}

}  // namespace aiy

using namespace aiy;

extern "C" {

int aiy_release_all(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (auto& kv : g_ctx) {  // each context's buffers live on its own device
        (void)hipSetDevice(std::get<0>(kv.first));
        kv.second.reset();
    }
    g_ctx.clear();
    (void)hipSetDevice(cur);
    return AIY_OK;
}

int64_t aiy_host_cache_bytes(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    int64_t b = 0;
    for (auto& kv : g_ctx)
        for (auto& q : kv.second->bufs) b += (int64_t)q.second.second;
    return b;
}

int aiy_vfi_sweep(const double* v_old, const double* a_grid, const double* s, const double* P,
                  int64_t N, int64_t Na, double r, double w, double beta, double sigma,
                  double* v_new, double* policy_k, double* policy_c, int32_t* policy_idx) {
    return vfi_host(v_old, a_grid, s, P, N, Na, r, w, beta, sigma, false, 0, 1, nullptr, v_new,
                    policy_k, policy_c, policy_idx, nullptr);
}

int aiy_vfi_solve(double* v_old, const double* a_grid, const double* s, const double* P,
                  int64_t N, int64_t Na, double r, double w, double beta, double sigma,
                  double tol, int64_t max_iter, double* v_new, double* policy_k,
                  double* policy_c, int32_t* policy_idx, int64_t* iters) {
    if (!iters) return fail(AIY_BAD_ARG, "NULL iters");
    return vfi_host(v_old, a_grid, s, P, N, Na, r, w, beta, sigma, true, tol, max_iter, v_old,
                    v_new, policy_k, policy_c, policy_idx, iters);
}

int aiy_labor_vfi_sweep(const double* v_old, const double* a_grid, const double* s,
                        const double* P, const double* labor_choice, int64_t N, int64_t Na,
                        int64_t Nl, double r, double w, double beta, double sigma, double psi,
                        double eta, double* v_new, double* policy_k, double* policy_l,
                        double* policy_c, int32_t* policy_lin) {
    return labor_host(v_old, a_grid, s, P, labor_choice, N, Na, Nl, r, w, beta, sigma, psi, eta,
                      false, 0, 1, nullptr, v_new, policy_k, policy_l, policy_c, policy_lin,
                      nullptr);
}

int aiy_labor_vfi_solve(double* v_old, const double* a_grid, const double* s, const double* P,
                        const double* labor_choice, int64_t N, int64_t Na, int64_t Nl, double r,
                        double w, double beta, double sigma, double psi, double eta, double tol,
                        int64_t max_iter, double* v_new, double* policy_k, double* policy_l,
                        double* policy_c, int32_t* policy_lin, int64_t* iters) {
    if (!iters) return fail(AIY_BAD_ARG, "NULL iters");
    return labor_host(v_old, a_grid, s, P, labor_choice, N, Na, Nl, r, w, beta, sigma, psi, eta,
                      true, tol, max_iter, v_old, v_new, policy_k, policy_l, policy_c,
                      policy_lin, iters);
}

}  // extern "C"
