// Launch-chain timing through the C ABI from C++ (no Python between launches), to separate the
// kernels' own cost from host issue: EGM steps (aiy_egm_step_dev), headline
// sweeps (aiy_vfi_sweep_dev, hint = previous argmax) and histogram pushes
// (aiy_dist_stationary_dev, tol = 0) at Na = 20,000, N = 7, chained on one stream and timed
// with hipEvents.  Synthetic calibration of the benched shape (quadratic grid on [0, 50],
// tridiagonal P, r = 0.04, sigma = 5).
//   g++ -O2 -std=c++17 -I../../include -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ chain_bench.cpp \
//       -L../../aiyagari-replication_amd -laiyagari_hip -L/opt/rocm/lib -lamdhip64 \
//       -Wl,-rpath,'$ORIGIN/../../aiyagari-replication_amd' -o chain_bench
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "aiyagari_hip.h"

#define CK(x)                                                                          \
    do {                                                                               \
        int e_ = (int)(x);                                                             \
        if (e_ != 0) {                                                                 \
            printf("error %d at %s:%d: %s\n", e_, __FILE__, __LINE__, aiy_last_error()); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

int main() {
    const int N = 7, Na = 20000;
    const size_t n = (size_t)N * Na;
    std::vector<double> a(Na), s(N), P(N * N, 0.0), c0(n), v0(n, 0.0), lam(n, 1.0 / n);
    for (int k = 0; k < Na; ++k) a[k] = 50.0 * std::pow(k / (Na - 1.0), 2.0);
    for (int i = 0; i < N; ++i) s[i] = std::exp(-0.6 + 0.2 * i);
    for (int i = 0; i < N; ++i) {
        P[i * N + i] = 0.8;
        P[i * N + (i > 0 ? i - 1 : i + 1)] += 0.1;
        P[i * N + (i < N - 1 ? i + 1 : i - 1)] += 0.1;
    }
    const double r = 0.04, w = 1.2, beta = 0.96, sigma = 5.0;
    for (int i = 0; i < N; ++i)
        for (int k = 0; k < Na; ++k) c0[(size_t)i * Na + k] = (1 + r) * a[k] + w * s[i];
    double *da, *ds, *dP, *dc[2], *dpk, *dv[2], *dpc, *dl[2];
    int* idx;
    hipMalloc(&da, Na * 8); hipMalloc(&ds, N * 8); hipMalloc(&dP, N * N * 8);
    hipMalloc(&dc[0], n * 8); hipMalloc(&dc[1], n * 8); hipMalloc(&dpk, n * 8);
    hipMalloc(&dv[0], n * 8); hipMalloc(&dv[1], n * 8); hipMalloc(&dpc, n * 8);
    hipMalloc(&dl[0], n * 8); hipMalloc(&dl[1], n * 8); hipMalloc(&idx, n * 4);
    hipMemcpy(da, a.data(), Na * 8, hipMemcpyHostToDevice);
    hipMemcpy(ds, s.data(), N * 8, hipMemcpyHostToDevice);
    hipMemcpy(dP, P.data(), N * N * 8, hipMemcpyHostToDevice);
    hipMemcpy(dv[0], v0.data(), n * 8, hipMemcpyHostToDevice);
    hipMemcpy(dl[0], lam.data(), n * 8, hipMemcpyHostToDevice);
    hipStream_t st;
    hipStreamCreate(&st);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    aiy_ws* ws;
    CK(aiy_ws_create(N, Na, 1, &ws));
    auto span = [&](auto&& body, int reps) -> double {
        hipEventRecord(e0, st);
        for (int q = 0; q < reps; ++q)
            if (body(q)) return -1.0;
        hipEventRecord(e1, st);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        return ms * 1e3 / reps;
    };
    for (int variant : {-1, 4096}) {  // EGM: two launches (default), one-pass scatter
        CK(aiy_ws_set_variant(ws, variant));
        hipMemcpy(dc[0], c0.data(), n * 8, hipMemcpyHostToDevice);
        auto step = [&](int q) {
            return aiy_egm_step_dev(ws, dc[q & 1], da, ds, dP, r, w, beta, sigma, 0.0, 0, 1.0, 1.0,
                                    dc[1 - (q & 1)], dpk, nullptr, nullptr, st);
        };
        span(step, 20);
        printf("{\"egm_step_variant\": %d, \"us_per_step\": %.3f}\n", variant, span(step, 200));
    }
    for (int variant : {-1, 8192}) {  // the device-tier EGM solve: chained steps (default), two
        CK(aiy_ws_set_variant(ws, variant));  // launches per step (bit 13); 200 steps at tol = 0
        int64_t itn;
        double dd;
        auto solve = [&](int) {
            hipMemcpyAsync(dc[0], c0.data(), n * 8, hipMemcpyHostToDevice, st);
            return aiy_egm_solve_dev(ws, dc[0], da, ds, dP, r, w, beta, sigma, 0.0, 0, 1.0, 1.0,
                                     0.0, 200, dpk, nullptr, &itn, &dd, st);
        };
        solve(0);
        printf("{\"egm_solve_dev_variant\": %d, \"us_per_step\": %.3f}\n", variant,
               span(solve, 3) / 200);
    }
    CK(aiy_ws_set_variant(ws, -1));
    int cur = 0;
    auto sweep = [&](int q) {  // headline sweeps from v = 0, hint = the previous argmax
        int rc = aiy_vfi_sweep_dev(ws, dv[cur], da, ds, dP, r, w, beta, sigma, q ? idx : nullptr,
                                   0, dv[1 - cur], idx, dpk, dpc, nullptr, st);
        cur = 1 - cur;
        return rc;
    };
    span(sweep, 5);
    printf("{\"vfi_sweeps\": \"6-25\", \"us_per_sweep\": %.3f}\n", span(sweep, 20));
    printf("{\"vfi_sweeps\": \"26-125\", \"us_per_sweep\": %.3f}\n", span(sweep, 100));
    int64_t it;
    double d;
    hipStreamSynchronize(st);
    auto pushes = [&](int) {
        return aiy_dist_stationary_dev(ws, dl[0], idx, nullptr, da, dP, 0.0, 320, dl[1], nullptr,
                                       &it, &d, st);
    };
    pushes(0);
    printf("{\"dist_pushes\": 320, \"us_per_push\": %.3f}\n", span(pushes, 3) / 320);
    aiy_ws_destroy(ws);
    return 0;
}
