// F3 / F2 — the Krusell-Smith shock panel (Krusell_Smith_VFI.m:57-94) and the capital-path
// simulation of the agent panel (:206-248).
//
// Shock panel: the aggregate chain zi is serial (T-1 draws) and runs on one lane; the
// idiosyncratic chains are independent per agent, so one lane owns one agent and walks t.
// The uniforms are laid out in the order MATLAB draws them (t outer, agent inner), so at
// every t the lanes of a wave read 64 consecutive doubles: coalesced, HBM-bound.  The loads
// do not depend on the recurrence, so the t loop is unrolled to keep several in flight.
//
// Panel simulation: per period every agent moves by a 2-D linear interpolation of k_opt(:,:,s)
// at (k, K_ts(t)) (griddedInterpolant default 'linear', linear extrapolation), and
// K_ts(t+1) = mean(k_population) couples all agents.  One launch per period: the launch for
// period t first folds the previous launch's block partials in block order (every block, the
// same sequence of additions, so every block holds the same K_ts(t) — no grid barrier, no
// atomics), then moves its agents and writes its own partial.  The order of the mean is fixed
// (lane-strided sums, pairwise fold per block, block order) and restated by
// np_oracle.ks_panel_simulate; MATLAB's own summation order is unpinned.
#include "aiy_common.hpp"
#include "ks_panel.hpp"

namespace aiy {

constexpr int kPanelLdsGrid = 8192;  // k_grid staged in LDS up to this many points

__global__ __launch_bounds__(64) void ks_zi_kernel(ShockArgs A) {
    if (threadIdx.x != 0) return;
    int z = 1;                                   // :60 zi_shock(1) = 1 (1-based good)
    A.zi[0] = 0;
    for (int t = 1; t < A.T; ++t) {              // :61-67
        const double u = A.U[t - 1];
        z = 1 + (u > (z == 1 ? A.pgg : A.pbb) ? 1 : 0);
        A.zi[t] = (int8_t)(z - 1);               // :68
    }
}

__global__ __launch_bounds__(256) void ks_eps_kernel(ShockArgs A) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A.pop) return;
    const int64_t pop = A.pop;
    const double* __restrict__ U = A.U + (A.T - 1);
    int e = U[i] > A.ug ? 1 : 0;                 // :71 (rand > ug) + 1, stored minus 1
    A.eps[i * A.is] = (int8_t)e;
    U += pop;
    const int8_t* __restrict__ zi = A.zi;
    int zp = zi[0];
    constexpr int UN = 8;
    int t = 1;
    for (; t + UN <= A.T; t += UN) {
        double u[UN];
#pragma unroll
        for (int q = 0; q < UN; ++q) u[q] = __builtin_nontemporal_load(U + (int64_t)(t - 1 + q) * pop + i);
#pragma unroll
        for (int q = 0; q < UN; ++q) {
            const int zc = zi[t + q];
            e = u[q] > A.thr[(zc * 2 + zp) * 2 + e] ? 1 : 0;   // :88-92
            A.eps[(int64_t)(t + q) * A.ts + i * A.is] = (int8_t)e;
            zp = zc;
        }
    }
    for (; t < A.T; ++t) {
        const double u = U[(int64_t)(t - 1) * pop + i];
        const int zc = zi[t];
        e = u > A.thr[(zc * 2 + zp) * 2 + e] ? 1 : 0;
        A.eps[(int64_t)t * A.ts + i * A.is] = (int8_t)e;
        zp = zc;
    }
}

int launch_ks_shocks(const ShockArgs& A, hipStream_t st) {
    ks_zi_kernel<<<1, 64, 0, st>>>(A);
    AIY_HIP(hipGetLastError());
    ks_eps_kernel<<<(A.pop + 255) / 256, 256, 0, st>>>(A);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}

// ------------------------------------------------------------------ panel simulation

// block fold of the 256 lane sums (pairwise, h = 128 ... 1: s[l] + s[l+h]); thread 0 returns it
__device__ __forceinline__ double block_fold(double acc, double* red) {
    const int tid = threadIdx.x;
    red[tid] = acc;
    __syncthreads();
    if (tid < 128) red[tid] = red[tid] + red[tid + 128];
    __syncthreads();
    double x = 0.0;
    if (tid < 64) {
        x = red[tid] + red[tid + 64];
#pragma unroll
        for (int h = 32; h >= 1; h >>= 1) {
            const double o = __shfl_down(x, h);
            x = x + o;   // lanes l < h hold s[l] + s[l+h]
        }
    }
    return x;
}

// sum of the G block partials in block order, divided by the population (thread 0)
__device__ __forceinline__ double fold_partials(const double* __restrict__ part, int G, int pop) {
    double acc = 0.0;
    for (int b = 0; b < G; ++b) acc = acc + part[b];
    return acc / (double)pop;
}

__device__ __forceinline__ int seg_lds(const double* x, int n, double q) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (x[mid] <= q) lo = mid + 1;
        else hi = mid;
    }
    int i = lo - 1;
    i = i < 0 ? 0 : i;
    return i > n - 2 ? n - 2 : i;
}

// partial sums of the initial population (K_ts(1) = mean(k_population), :208)
__global__ __launch_bounds__(256) void ks_panel_sum_kernel(PanelArgs A) {
    __shared__ double red[256];
    const int64_t L = (int64_t)A.G * 256;
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < A.pop; i += L)
        acc = acc + A.k_pop[i];
    const double s = block_fold(acc, red);
    if (threadIdx.x == 0) A.part[blockIdx.x] = s;
}

template <bool LDS>
__global__ __launch_bounds__(256) void ks_panel_step_kernel(PanelArgs A, int t) {
    __shared__ double red[256];
    __shared__ double sK;
    extern __shared__ double kg_lds[];
    const double* kg = A.k_grid;
    if constexpr (LDS) {
        for (int q = threadIdx.x; q < A.nk; q += 256) kg_lds[q] = A.k_grid[q];
        kg = kg_lds;
    }
    const double* part_in = A.part + (t & 1) * A.G;
    double* part_out = A.part + ((t + 1) & 1) * A.G;
    if (threadIdx.x == 0) {
        const double K = fold_partials(part_in, A.G, A.pop);
        sK = K;
        if (blockIdx.x == 0) A.K_ts[t] = K;   // :208 / :247 of the previous period
    }
    __syncthreads();
    const double K = sK;
    const int nk = A.nk, nK = A.nK;
    const int iK = seg_of_dev(A.K_grid, nK, K);
    const double K0 = A.K_grid[iK], K1 = A.K_grid[iK + 1];
    const double tK = (K - K0) / (K1 - K0);
    const int zt = A.zi[t];
    const int64_t L = (int64_t)A.G * 256;
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < A.pop; i += L) {
        const double k = A.k_pop[i];
        const int s = 2 * zt + A.eps[(int64_t)t * A.ts + i * A.is];   // :227-232
        const int ik = seg_lds(kg, nk, k);
        const double x0 = kg[ik], x1 = kg[ik + 1];
        const double tk = (k - x0) / (x1 - x0);
        const double* f = A.k_opt + ((size_t)s * nK + iK) * nk + ik;   // column (iK, s)
        const double f00 = f[0], f10 = f[1], f01 = f[nk], f11 = f[nk + 1];
        const double f0 = f00 + tk * (f10 - f00);
        const double f1 = f01 + tk * (f11 - f01);
        const double kn = f0 + tK * (f1 - f0);   // :241-245
        A.k_pop[i] = kn;                         // :246
        acc = acc + kn;
    }
    const double sb = block_fold(acc, red);
    if (threadIdx.x == 0) part_out[blockIdx.x] = sb;
}

__global__ __launch_bounds__(64) void ks_panel_final_kernel(PanelArgs A, int t) {
    if (threadIdx.x == 0) A.K_ts[t] = fold_partials(A.part + (t & 1) * A.G, A.G, A.pop);
}

int launch_ks_panel(const PanelArgs& A, hipStream_t st) {
    ks_panel_sum_kernel<<<A.G, 256, 0, st>>>(A);
    AIY_HIP(hipGetLastError());
    const bool lds = A.nk <= kPanelLdsGrid;
    const size_t sh = lds ? sizeof(double) * A.nk : 0;
    for (int t = 0; t + 1 < A.T; ++t) {
        if (lds) ks_panel_step_kernel<true><<<A.G, 256, sh, st>>>(A, t);
        else ks_panel_step_kernel<false><<<A.G, 256, 0, st>>>(A, t);
    }
    AIY_HIP(hipGetLastError());
    ks_panel_final_kernel<<<1, 64, 0, st>>>(A, A.T - 1);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}

}  // namespace aiy
