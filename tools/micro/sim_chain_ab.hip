// A/B of the A9 chain step (GE inner loop, Aiyagari_VFI.m:174-193): the round-4 window kernel
// and the two-wave pipe kernel (both from csrc/sim_kernels.hip) on a synthetic Na = 400 /
// N = 7 policy and T = 10,000 uniforms — their paths must agree bit for bit — plus timing-only
// diagnostics (exp0-3: one cost removed each; their paths are not kept).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math \
//         -I../../include sim_chain_ab.hip -o sim_chain_ab && ./sim_chain_ab [Na] [T] [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../aiyagari-replication_amd/csrc/sim_kernels.hip"

namespace aiy {
int fail(int code, const char*, ...) { return code; }
}  // namespace aiy


namespace exp {
using namespace aiy;
// MODE 0: baseline step; 1: division replaced by a multiply (timing only); 2: no readlane (lane
// 0's candidate; timing only); 3: window loads from registers fixed at w0 = 0 (timing only);
template <int MODE>
__global__ __launch_bounds__(256) void chain_exp(SimArgs A) {
    extern __shared__ double lds[];
    __shared__ unsigned long long F[kSimChunk];
    __shared__ double cs[16 * 16];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int N = A.N, Na = A.Na;
    const int S = Na + 64;
    double* a = lds;            // [S]
    double* pol = lds + S;      // [N][S]
    for (int k = tid; k < S; k += 256) a[k] = A.a[min(k, Na - 1)];
    for (int q = tid; q < N * S; q += 256) {
        int zz = q / S, kk = q - zz * S;
        pol[q] = kk < Na ? A.pol[(size_t)zz * A.zs + (size_t)kk * A.as] : 0.0;
    }
    __syncthreads();
    if (tid == 0) {
        for (int z = 0; z < N; ++z) {
            double acc = 0.0;
            for (int m = 0; m < N; ++m) {
                acc = acc + A.P[z * N + m];
                cs[z * N + m] = acc;
            }
        }
    }
    __syncthreads();
    const int wmax = Na > 64 ? Na - 64 : 0;
    int z = A.z1;
    double k = A.k1;
    double sum = k;
    int w0 = 0;
    double rx0 = a[lane], rx1 = a[lane + 1], ry0 = pol[lane], ry1 = pol[lane + 1];
    for (int c0 = 1; c0 < A.T; c0 += kSimChunk) {
        const int cn = min(kSimChunk, A.T - c0);
        for (int q = tid; q < cn; q += 256) {
            const double u = A.U[c0 + q - 1];
            unsigned long long f = 0;
            for (int zz = 0; zz < N; ++zz) {
                int m = 15;
                for (int mm = N - 1; mm >= 0; --mm)
                    if (u < cs[zz * N + mm]) m = mm;
                f |= (unsigned long long)m << (4 * zz);
            }
            F[q] = f;
        }
        __syncthreads();
        if (wave == 0) {
            unsigned long long Fv = 0;
            for (int i = 0; i < cn; ++i) {
                if ((i & 63) == 0) Fv = (i + lane < cn) ? F[i + lane] : 0ull;
                const unsigned long long f = readlane_u64(Fv, i & 63);
                const int zn = (int)((f >> (4 * z)) & 15ull);
                if (zn == 15) break;
                z = zn;
                const double* y = pol + (size_t)z * S;
                const int p = w0 + lane;
                double x0, x1, y0, y1;
                if (MODE == 3) { x0 = rx0; x1 = rx1; y0 = ry0; y1 = ry1; }
                else { x0 = a[p]; x1 = a[p + 1]; y0 = y[p]; y1 = y[p + 1]; }
                const int cnt = __popcll(__ballot(p < Na && x0 <= k));
                double kn;
                if (MODE == 1) kn = y0 + (k - x0) * (x1 - x0) * (y1 - y0);
 else kn = y0 + (k - x0) / (x1 - x0) * (y1 - y0);
                int seg = w0 + cnt - 1;
                seg = seg < 0 ? 0 : (seg > Na - 2 ? Na - 2 : seg);
                const int sl = min(max(seg - w0, 0), 63);
                k = MODE == 2 ? __shfl(kn, 0) : readlane_d(kn, sl);
                if (MODE != 3) {
                    w0 = seg - 31;
                    w0 = w0 < 0 ? 0 : (w0 > wmax ? wmax : w0);
                }
                sum += k;
            }
        }
        __syncthreads();
    }
    if (tid == 0) { A.out[0] = sum / (double)A.T; A.status[0] = 0; }
}
template <int MODE>
int launch_exp(const SimArgs& A) {
    const size_t S = A.Na + 64;
    const size_t bytes = 8 * (S * (A.N + 1));
    (void)hipFuncSetAttribute((const void*)chain_exp<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    chain_exp<MODE><<<1, 256, bytes, 0>>>(A);
    return hipGetLastError() != hipSuccess;
}

int launch_exp_mode(int m, const SimArgs& A) {
    switch (m) {
        case 0: return launch_exp<0>(A);
        case 1: return launch_exp<1>(A);
        case 2: return launch_exp<2>(A);
        default: return launch_exp<3>(A);
    }
}
}  // namespace exp

#define CK(x)                                                          \
    do {                                                               \
        hipError_t e_ = (x);                                           \
        if (e_ != hipSuccess) {                                        \
            printf("hip error %s at %d\n", hipGetErrorString(e_), __LINE__); \
            return 1;                                                  \
        }                                                              \
    } while (0)

int main(int argc, char** argv) {
    const int Na = argc > 1 ? atoi(argv[1]) : 400;
    const int T = argc > 2 ? atoi(argv[2]) : 10000;
    const int reps = argc > 3 ? atoi(argv[3]) : 15;
    const int N = 7;
    std::vector<double> a(Na), pol((size_t)N * Na), P(N * N, 0.0), U(T);
    const double amax = 60.0, amin = 0.0;
    for (int i = 0; i < Na; ++i) a[i] = amin + (amax - amin) * std::pow(i / (Na - 1.0), 2.0);
    for (int z = 0; z < N; ++z) {
        const double s = std::exp(-0.9 + 0.3 * z);
        for (int i = 0; i < Na; ++i) {  // a policy on the grid, mean-reverting around ~8
            double kp = 0.93 * a[i] + 0.6 * s;
            int j = (int)(std::lower_bound(a.begin(), a.end(), kp) - a.begin());
            pol[(size_t)z * Na + i] = a[std::min(j, Na - 1)];
        }
    }
    for (int i = 0; i < N; ++i) {
        P[i * N + i] = 0.7;
        P[i * N + (i > 0 ? i - 1 : i + 1)] += 0.15;
        P[i * N + (i < N - 1 ? i + 1 : i - 1)] += 0.15;
    }
    unsigned long long st = 88172645463325252ull;
    for (int t = 0; t < T; ++t) {
        st ^= st << 13; st ^= st >> 7; st ^= st << 17;
        U[t] = ((st >> 11) + 0.5) * (1.0 / 9007199254740992.0);
    }
    double *da, *dpol, *dP, *dU, *dout, *dk;
    int *dstat, *dz;
    CK(hipMalloc(&da, Na * 8)); CK(hipMalloc(&dpol, pol.size() * 8)); CK(hipMalloc(&dP, N * N * 8));
    CK(hipMalloc(&dU, T * 8)); CK(hipMalloc(&dout, 8)); CK(hipMalloc(&dk, T * 8));
    CK(hipMalloc(&dstat, 4)); CK(hipMalloc(&dz, T * 4));
    CK(hipMemcpy(da, a.data(), Na * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dpol, pol.data(), pol.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dP, P.data(), N * N * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dU, U.data(), T * 8, hipMemcpyHostToDevice));
    aiy::SimArgs A{};
    A.N = N; A.Na = Na; A.T = T; A.z1 = 3; A.k1 = a[Na / 4];
    A.pol = dpol; A.zs = Na; A.as = 1; A.a = da; A.P = dP; A.U = dU; A.out = dout;
    A.status = dstat; A.C = 1;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<double> ref_k;
    double ref_mean = 0;
    const char* names[] = {"window chain", "pipe chain", "exp0 base", "exp1 mul", "exp2 noreadlane", "exp3 regwin"};
    for (int v = 0; v < 6; ++v) {
        auto launch = [&](bool path) {
            aiy::SimArgs B = A;
            B.sim_k = path ? dk : nullptr;
            B.sim_z = path ? dz : nullptr;
            if (v == 0) {  // the round-4 window kernel (LDS rows), launched directly
                const size_t bytes = 8 * (size_t)(B.Na + 64) * (B.N + 1);
                if (path) aiy::sim_chain_kernel<true, true><<<1, 256, bytes, 0>>>(B);
                else aiy::sim_chain_kernel<true, false><<<1, 256, bytes, 0>>>(B);
                return (int)(hipGetLastError() != hipSuccess);
            }
            if (v == 1) return aiy::launch_sim_chain_pipe(B, 0);
            return exp::launch_exp_mode(v - 2, B);
        };
        CK(hipMemset(dk, 0, T * 8));
        if (launch(true) != 0) { printf("%s: launch refused\n", names[v]); continue; }
        CK(hipDeviceSynchronize());
        std::vector<double> k(T);
        double mean;
        int stat;
        CK(hipMemcpy(k.data(), dk, T * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&mean, dout, 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&stat, dstat, 4, hipMemcpyDeviceToHost));
        if (v == 0) { ref_k = k; ref_mean = mean; }
        int diff = 0;
        for (int t = 0; t < T; ++t) diff += memcmp(&k[t], &ref_k[t], 8) != 0;
        std::vector<float> ms;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0, 0));
            launch(false);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float x;
            CK(hipEventElapsedTime(&x, e0, e1));
            ms.push_back(x);
        }
        std::sort(ms.begin(), ms.end());
        double mean2;
        CK(hipMemcpy(&mean2, dout, 8, hipMemcpyDeviceToHost));
        printf("%-18s Na=%d T=%d  median %.3f ms  min %.3f  (%.1f ns/step)  path diffs %d  mean %s  "
               "status %d  k range [%g, %g]\n", names[v], Na, T, ms[ms.size() / 2], ms[0],
               ms[ms.size() / 2] * 1e6 / T, diff,
               (memcmp(&mean, &ref_mean, 8) == 0 && memcmp(&mean2, &ref_mean, 8) == 0) ? "same" : "DIFF",
               stat, *std::min_element(k.begin(), k.end()), *std::max_element(k.begin(), k.end()));
    }
    return 0;
}
