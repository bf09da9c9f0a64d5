// Microbenchmark: dependent vs independent fp64 VALU issue on gfx950 (one wave).  Tuning aid.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CH>
__global__ void chain_mul(double* out, double y, int iters, long long* cyc) {
    double x[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = threadIdx.x * 1e-3 + c;
    long long t0 = clock64();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CH; ++c) x[c] = x[c] * y;
#pragma unroll
        for (int c = 0; c < CH; ++c) x[c] = x[c] - y;
    }
    long long t1 = clock64();
    double s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += x[c];
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

template <int CH>
__global__ void chain_max(double* out, double y, int iters, long long* cyc) {
    double x[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = threadIdx.x * 1e-3 + c;
    long long t0 = clock64();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CH; ++c) x[c] = fmax(x[c] * y, y);
    }
    long long t1 = clock64();
    double s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += x[c];
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

template <class K>
void run(const char* name, K k, int ops_per_iter, int waves) {
    double* out;
    long long* cyc;
    hipMalloc(&out, 64 * waves * sizeof(double));
    hipMalloc(&cyc, sizeof(long long));
    const int iters = 4096;
    hipLaunchKernelGGL(k, dim3(1), dim3(64 * waves), 0, 0, out, 1.0000001, iters, cyc);
    hipLaunchKernelGGL(k, dim3(1), dim3(64 * waves), 0, 0, out, 1.0000001, iters, cyc);
    long long c = 0;
    hipMemcpy(&c, cyc, sizeof c, hipMemcpyDeviceToHost);
    printf("%-28s waves/block %d: %.2f cycles per wave-instruction (clock64)\n", name, waves,
           (double)c / ((double)iters * ops_per_iter));
    hipFree(out);
    hipFree(cyc);
}

int main() {
    for (int w : {1, 4, 8}) {
        run("mul/sub chain x1", chain_mul<1>, 2, w);
        run("mul/sub chains x2", chain_mul<2>, 4, w);
        run("mul/sub chains x4", chain_mul<4>, 8, w);
        run("mul/sub chains x8", chain_mul<8>, 16, w);
        run("mul+max chain x1", chain_max<1>, 2, w);
        run("mul+max chains x8", chain_max<8>, 16, w);
    }
    return 0;
}
