// Floor of a dependent launch at the EGM/histogram grid shape: 313
// workgroups x 448 threads (N = 7 waves per workgroup, 64 nodes each, Na = 20,000), chains of
// 200 launches on one stream, each reading what the previous one wrote.  Variants:
//   0 empty kernel                          1 one load + one store per thread (1.1 MB each way)
//   2 as 1 + LDS exchange + __syncthreads   3 as 2 + aiy_pow per thread (the EGM RHS's pow)
//   4 as 3 + a 64-ary wave search of a 20,000-point grid (3 dependent rounds, the interp kernel)
//   5 the EGM RHS body (egm_rhs_kernel's arithmetic: u'(c) = 1/c^5, the Euler sum from LDS,
//     c~ = RHS^(-1/5) by aiy_pow, the endogenous grid; two stores)   6 as 5 with P from memory
//   7 as 5 with a plain division instead of aiy_pow (cost of the software pow)
//   8 as 5 with sigma a kernel argument (runtime aiy_ipow(c, ns), aiy_pow(acc, -1/sigma)) as
//     in egm_rhs_kernel
// Prints us per launch (hipEvent over the chain) for each variant.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I../../aiyagari-replication_amd/csrc \
//         kernel_floor.hip -o kernel_floor
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "aiy_math.h"

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) {                                                      \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            return 1;                                                               \
        }                                                                           \
    } while (0)

constexpr int kNa = 20000, kN = 7;

__device__ __forceinline__ double ipow5(double c) {
    double r = c * c;
    r = r * r;
    return r * c;
}

template <int V>
__global__ __launch_bounds__(1024) void floor_kernel(const double* __restrict__ x,
                                                     double* __restrict__ y,
                                                     const double* __restrict__ grid,
                                                     double sigma, int ns) {
    __shared__ double s[16][64];
    if (V == 0) return;
    const int lane = threadIdx.x & 63, m = threadIdx.x >> 6;
    const int k = blockIdx.x * 64 + lane;
    const bool ok = k < kNa;
    double v = ok ? x[(size_t)m * kNa + k] : 1.0;
    if (V >= 5) {  // egm_rhs_kernel's body
        const int j = __builtin_amdgcn_readfirstlane(m);
        s[m][lane] = ok ? 1.0 / (V == 8 ? aiy_ipow(v + 1.0, ns) : ipow5(v + 1.0)) : 0.0;
        __syncthreads();
        if (!ok) return;
        double acc = 0.0;
        for (int q = 0; q < kN; ++q) {
            const double pq = V == 6 ? grid[q * 7 + j] * 1e-5 : 0.13;
            acc = acc + (0.9 * pq) * s[q][lane];
        }
        const double cn = V == 7 ? 1.0 / acc : aiy_pow(acc, V == 8 ? -1.0 / sigma : -0.2);
        const double ag = grid[k];
        const double ah = ((cn + ag) - 0.7 * (1 + j)) / 1.04;
        y[(size_t)m * kNa + k] = ah;
        y[(size_t)((m + 1) % kN) * kNa + k] = cn;  // (a second 1.1 MB stream, as ahat + cnext)
        return;
    }
    if (V >= 2) {
        s[m][lane] = v;
        __syncthreads();
        double acc = 0.0;
        for (int q = 0; q < kN; ++q) acc = acc + 0.1 * s[q][lane];
        v = acc;
    }
    if (V >= 3) v = aiy_pow(v + 1.5, -0.2);
    if (V >= 4) {
        int lo = 0, hi = kNa;
        const double q0 = __shfl(v, 0);
        while (lo < hi) {
            const int st = max((hi - lo + 63) >> 6, 1);
            const int kk = lo + (lane + 1) * st - 1;
            const bool vv = kk < hi;
            const double g = vv ? grid[kk] : 0.0;
            const int c = __popcll(__ballot(vv && g <= q0));
            const int nh = lo + (c + 1) * st - 1;
            lo += c * st;
            hi = nh < hi ? nh : hi;
        }
        v = v + (double)lo;
    }
    if (ok) y[(size_t)m * kNa + k] = v;
}

template <int V>
int run(double* a, double* b, const double* g, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
    const int nb = (kNa + 63) / 64;
    for (int w = 0; w < 20; ++w) floor_kernel<V><<<nb, 64 * kN, 0, st>>>(a, b, g, 5.0, 5);
    CK(hipEventRecord(e0, st));
    for (int it = 0; it < 200; ++it) {
        floor_kernel<V><<<nb, 64 * kN, 0, st>>>(it & 1 ? b : a, it & 1 ? a : b, g, 5.0, 5);
    }
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"variant\": %d, \"us_per_launch\": %.3f}\n", V, ms * 1e3 / 200);
    return 0;
}

int main() {
    double *a, *b, *g;
    CK(hipMalloc(&a, sizeof(double) * kN * kNa));
    CK(hipMalloc(&b, sizeof(double) * kN * kNa));
    CK(hipMalloc(&g, sizeof(double) * kNa));
    std::vector<double> h(kN * kNa, 1.0), hg(kNa);
    for (int i = 0; i < kNa; ++i) hg[i] = 50.0 * (i / (kNa - 1.0)) * (i / (kNa - 1.0));
    CK(hipMemcpy(a, h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(b, h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(g, hg.data(), sizeof(double) * kNa, hipMemcpyHostToDevice));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int rep = 0; rep < 2; ++rep) {
        if (run<0>(a, b, g, st, e0, e1) || run<1>(a, b, g, st, e0, e1) ||
            run<2>(a, b, g, st, e0, e1) || run<3>(a, b, g, st, e0, e1) ||
            run<4>(a, b, g, st, e0, e1) || run<5>(a, b, g, st, e0, e1) ||
            run<6>(a, b, g, st, e0, e1) || run<7>(a, b, g, st, e0, e1) ||
            run<8>(a, b, g, st, e0, e1))
            return 1;
    }
    return 0;
}
