// Microbenchmark: dependent global-load latency (pointer chase, one wave) on gfx950 for
// working sets in L2, in the MALL and in HBM.  Tuning aid.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void chase(const unsigned* __restrict__ next, int steps, unsigned* out, long long* cyc) {
    unsigned p = threadIdx.x * 16;  // 64 lanes, distinct cache lines
    long long t0 = clock64();
    for (int i = 0; i < steps; ++i) p = next[p];
    long long t1 = clock64();
    out[threadIdx.x] = p;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    for (size_t bytes : {size_t(1) << 16, size_t(1) << 21, size_t(1) << 26, size_t(1) << 30}) {
        size_t n = bytes / 4;
        std::vector<unsigned> h(n);
        // stride of 4 KiB + 64 B through the array, wrapping: defeats simple prefetch
        size_t stride = (4096 + 64) / 4;
        for (size_t i = 0; i < n; ++i) h[i] = (unsigned)((i + stride) % n);
        unsigned* d;
        unsigned* out;
        long long* cyc;
        (void)hipMalloc(&d, bytes);
        (void)hipMalloc(&out, 256);
        (void)hipMalloc(&cyc, 8);
        (void)hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice);
        const int steps = 2000;
        hipLaunchKernelGGL(chase, dim3(1), dim3(64), 0, 0, d, steps, out, cyc);  // warm
        hipLaunchKernelGGL(chase, dim3(1), dim3(64), 0, 0, d, steps, out, cyc);
        long long c = 0;
        (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("working set %10zu B: %.0f cycles per dependent load (clock64)\n", bytes,
               (double)c / steps);
        (void)hipFree(d);
        (void)hipFree(out);
        (void)hipFree(cyc);
    }
    return 0;
}
