// Does code size cost time at kernel start?  The same dependent chains of T fp64 FMAs per
// lane, run as a U-fold unrolled loop (U = 16: a few hundred bytes of code) or straight-line
// (U = T: 8 bytes per FMA, up to 64 KB), in back-to-back dependent launches on one stream.
// Any time the straight-line kernel takes beyond the looped one is instruction fetch.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 icache_probe.hip -o icache_probe && ./icache_probe
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);   \
            return 1;                                                          \
        }                                                                      \
    } while (0)

template <int T, int U>
__global__ __launch_bounds__(256) void chain(double* out, double y, double z) {
    double x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;
    for (int it = 0; it < T / U; ++it) {
#pragma unroll
        for (int u = 0; u < U; u += 4) {
            asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x0) : "v"(y), "v"(z));
            asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x1) : "v"(y), "v"(z));
            asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x2) : "v"(y), "v"(z));
            asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x3) : "v"(y), "v"(z));
        }
    }
    const double s = x0 + x1 + x2 + x3;
    if (s == 12345.0) out[blockIdx.x] = s;  // (never: keeps the chains live)
}

template <int T, int U>
static int run(const char* name, int grid, int block, double* out, hipStream_t st) {
    const int reps = 200;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int w = 0; w < 20; ++w) chain<T, U><<<grid, block, 0, st>>>(out, 1.0000001, 1e-9);
    CK(hipEventRecord(e0, st));
    for (int r = 0; r < reps; ++r) chain<T, U><<<grid, block, 0, st>>>(out, 1.0000001, 1e-9);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-10s T=%5d U=%5d grid=%5d block=%4d code~%6d B  %8.3f us/launch\n", name, T, U, grid,
           block, U * 8, ms * 1e3 / reps);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return 0;
}

int main() {
    double* out;
    CK(hipMalloc(&out, 1 << 20));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    const int geo[][2] = {{256, 64}, {256, 512}, {2048, 256}};
    for (auto& g : geo) {
        if (run<1024, 16>("loop", g[0], g[1], out, st)) return 1;
        if (run<1024, 1024>("straight", g[0], g[1], out, st)) return 1;
        if (run<2048, 16>("loop", g[0], g[1], out, st)) return 1;
        if (run<2048, 2048>("straight", g[0], g[1], out, st)) return 1;
        if (run<4096, 16>("loop", g[0], g[1], out, st)) return 1;
        if (run<4096, 4096>("straight", g[0], g[1], out, st)) return 1;
        if (run<8192, 16>("loop", g[0], g[1], out, st)) return 1;
        if (run<8192, 8192>("straight", g[0], g[1], out, st)) return 1;
    }
    CK(hipFree(out));
    return 0;
}
