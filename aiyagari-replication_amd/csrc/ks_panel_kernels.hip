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
// period t first folds the previous launch's block partials pairwise (every block, the
// same sequence of additions, so every block holds the same K_ts(t) — no grid barrier, no
// atomics), then moves its agents and writes its own partial.  The order of the mean is fixed
// (lane-strided sums, pairwise fold per block, pairwise fold of the zero-padded block sums) and restated by
// np_oracle.ks_panel_simulate; MATLAB's own summation order is unpinned.
#include "aiy_common.hpp"
#include "ks_panel.hpp"

namespace aiy {

constexpr int kPanelLdsGrid = 8192;  // k_grid staged in LDS up to this many points

// The aggregate chain on one wave: 64 draws per round are loaded in parallel, compared with
// both thresholds (two ballots), then the wave walks the 64 steps on the masks with scalar bit
// logic — the serial part is register work, the loads are not on the dependency chain.
__global__ __launch_bounds__(64) void ks_zi_kernel(ShockArgs A) {
    const int lane = threadIdx.x;
    int z = 0;                                   // :60 zi_shock(1) = 1 (0 after :68)
    if (lane == 0) A.zi[0] = 0;
    for (int t0 = 1; t0 < A.T; t0 += 64) {       // :61-67
        const int t = t0 + lane;
        const double u = t < A.T ? A.U[t - 1] : 0.0;
        const unsigned long long g = __ballot(u > A.pgg);   // next bad if now good
        const unsigned long long b = __ballot(u > A.pbb);   // next bad if now bad
        unsigned long long zm = 0;
        const int n = min(64, A.T - t0);
        for (int q = 0; q < n; ++q) {
            z = (int)(((z ? b : g) >> q) & 1ull);
            zm |= (unsigned long long)z << q;
        }
        if (t < A.T) A.zi[t] = (int8_t)((zm >> lane) & 1ull);
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
    constexpr int UN = 32;
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

// mean of the population from the G block partials (wave 0; every lane returns it): the
// partials, zero-padded to G' = next power of two, are folded pairwise (h = G'/2 ... 1:
// s[l] + s[l+h]), then divided by the population.  Lane l holds s[l + 64m]: the folds with
// h >= 64 stay in registers, h < 64 are shuffles — one parallel load, no barrier, no serial
// chain of G dependent additions.  Split in a load and a fold phase so the loads can be in
// flight together with the block's other prefetches.
constexpr int kFoldPer = kPanelMaxBlocks / 64;   // 16 partials per lane at most
__device__ __forceinline__ void fold_load(const double* __restrict__ part, int G, double* v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int m = 0; m < kFoldPer; ++m) {
        const int i = lane + 64 * m;
        v[m] = i < G ? part[i] : 0.0;
    }
}
__device__ __forceinline__ double fold_sum(double* v, int G, int pop) {
    int Gp = 1;
    while (Gp < G) Gp <<= 1;
#pragma unroll
    for (int hm = kFoldPer / 2; hm >= 1; hm >>= 1)   // h = 64*hm
        if (64 * hm < Gp)
#pragma unroll
            for (int m = 0; m < hm; ++m) v[m] = v[m] + v[m + hm];
    double x = v[0];
#pragma unroll
    for (int h = 32; h >= 1; h >>= 1) {
        const double o = __shfl_down(x, h);
        if (h < Gp) x = x + o;
    }
    x = __shfl(x, 0);
    return x / (double)pop;
}
__device__ __forceinline__ double fold_partials(const double* __restrict__ part, int G, int pop) {
    double v[kFoldPer];
    fold_load(part, G, v);
    return fold_sum(v, G, pop);
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

// griddedInterpolant({k_grid, K_grid}, k_opt(:,:,s)) at (k, K): column (iK, s) of k_opt,
// segments ik / iK with weights tk / tK (:241-245)
__device__ __forceinline__ double move_agent(const PanelArgs& A, int iK, double tK, int s, int ik,
                                             double tk) {
    const int nk = A.nk;
    const double* f = A.k_opt + ((size_t)s * A.nK + iK) * nk + ik;
    const double f00 = f[0], f10 = f[1], f01 = f[nk], f11 = f[nk + 1];
    const double f0 = f00 + tk * (f10 - f00);
    const double f1 = f01 + tk * (f11 - f01);
    return f0 + tK * (f1 - f0);
}

// One period.  Dependent global round trips: one (the previous partials, the grids, this
// thread's first agent and its state are all loaded together before the first barrier) plus
// the k_opt gathers, which need K.
template <bool LDS>
__global__ __launch_bounds__(256) void ks_panel_step_kernel(PanelArgs A, int t) {
    __shared__ double red[256];
    __shared__ double sK;
    extern __shared__ double grid_lds[];
    const int nk = A.nk, nK = A.nK;
    const double* kg = A.k_grid;
    const double* Kg = A.K_grid;
    const int64_t L = (int64_t)A.G * 256;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    // the grids' loads and the first agent's (prefetched before the partials are folded) all in
    // flight before any LDS write: clamped, unguarded loads (a guarded load and its write in one
    // loop waited for each load in turn — two round trips before the agent's)
    double gk = 0.0, gK = 0.0;
    const bool one = LDS && nk <= 256 && nK <= 256;  // (uniform) one grid value per thread
    if (one) {
        const int q = (int)threadIdx.x;
        gk = A.k_grid[min(q, nk - 1)];
        gK = A.K_grid[min(q, nK - 1)];
    }
    const int zt = A.zi[t];
    const int8_t* __restrict__ erow = A.eps + (int64_t)t * A.ts;
    const int64_t ic = i < A.pop ? i : 0;
    const double k0 = A.k_pop[ic];
    const int e0 = erow[ic * A.is];
    const double k = i < A.pop ? k0 : 0.0;
    const int e = i < A.pop ? e0 : 0;
    if constexpr (LDS) {
        if (one) {
            const int q = (int)threadIdx.x;
            if (q < nk) grid_lds[q] = gk;
            if (q < nK) grid_lds[nk + q] = gK;
        } else {
            for (int q = threadIdx.x; q < nk; q += 256) grid_lds[q] = A.k_grid[q];
            for (int q = threadIdx.x; q < nK; q += 256) grid_lds[nk + q] = A.K_grid[q];
        }
        kg = grid_lds;
        Kg = grid_lds + nk;
    }
    double v[kFoldPer];
    if (threadIdx.x < 64) fold_load(A.part + (t & 1) * A.G, A.G, v);
    __syncthreads();           // grids staged; every prefetch has landed
    if (threadIdx.x < 64) {
        const double K = fold_sum(v, A.G, A.pop);
        if (threadIdx.x == 0) {
            sK = K;
            if (blockIdx.x == 0) A.K_ts[t] = K;   // :208 / :247 of the previous period
        }
    }
    // k-segment of the first agent does not depend on K
    int ik = seg_lds(kg, nk, k);
    double tk = (k - kg[ik]) / (kg[ik + 1] - kg[ik]);
    __syncthreads();
    const double K = sK;
    const int iK = seg_lds(Kg, nK, K);
    const double tK = (K - Kg[iK]) / (Kg[iK + 1] - Kg[iK]);
    double acc = 0.0;
    // first agent (prefetched); the lane's sum keeps agent order
    if (i < A.pop) {
        const double kn = move_agent(A, iK, tK, 2 * zt + e, ik, tk);   // :227-245
        A.k_pop[i] = kn;                                                 // :246
        acc = acc + kn;
        i += L;
    }
    // further agents (more than G*256 agents), four at a time: loads, searches and gathers
    // of the four are independent, only the lane sum is ordered
    for (; i < A.pop; i += 4 * L) {
        double kk[4], kn[4];
        int ee[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t j = i + q * L;
            kk[q] = j < A.pop ? A.k_pop[j] : kg[0];
            ee[q] = j < A.pop ? erow[j * A.is] : 0;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int jk = seg_lds(kg, nk, kk[q]);
            const double tq = (kk[q] - kg[jk]) / (kg[jk + 1] - kg[jk]);
            kn[q] = move_agent(A, iK, tK, 2 * zt + ee[q], jk, tq);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t j = i + q * L;
            if (j < A.pop) {
                A.k_pop[j] = kn[q];
                acc = acc + kn[q];
            }
        }
    }
    const double sb = block_fold(acc, red);
    if (threadIdx.x == 0) A.part[((t + 1) & 1) * A.G + blockIdx.x] = sb;
}

__global__ __launch_bounds__(64) void ks_panel_final_kernel(PanelArgs A, int t) {
    const double K = fold_partials(A.part + (t & 1) * A.G, A.G, A.pop);
    if (threadIdx.x == 0) A.K_ts[t] = K;
}

int launch_ks_panel(const PanelArgs& A, hipStream_t st) {
    ks_panel_sum_kernel<<<A.G, 256, 0, st>>>(A);
    AIY_HIP(hipGetLastError());
    const bool lds = A.nk + A.nK <= kPanelLdsGrid;
    const size_t sh = lds ? sizeof(double) * (A.nk + A.nK) : 0;
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
