// A9 — Monte-Carlo capital supply (Aiyagari_VFI.m:104-129; GE copy :174-193; the same block
// in the three other Aiyagari scripts).  The chain is serial by construction: each step needs
// the previous (z, k).  One wavefront runs it; its 64 lanes cooperate on the two searches of
// every step:
//   z_t = find(rand < cumsum(P(z_{t-1},:)), 1)      lanes m < N compare, ballot, first bit
//   k_t = interp1(a_grid, policy_k(z_t,:), k_{t-1}, 'linear', 'extrap')
//        segment = largest i with a_i <= k_{t-1} (clamped to the end segments), found by a
//        64-ary search: a window of 64 grid points per round, ballot + popcount.
// a_grid and the policy rows are staged in LDS when they fit (Na·(N+1) <= 18432 doubles),
// otherwise read through L1/L2.
// Uniform draws come from the host (MATLAB's rand stream), so the chain is reproducible.
#include "aiy_common.hpp"
#include "sim.hpp"

namespace aiy {

constexpr int kSimLdsMax = 18432;  // doubles: 147 KiB of the 160 KiB LDS

template <bool LDS>
__global__ __launch_bounds__(64) void sim_capital_kernel(SimArgs A) {
    extern __shared__ double lds[];
    const int lane = threadIdx.x;
    const int N = A.N, Na = A.Na;
    const double* a = A.a;
    const double* pol = A.pol;
    size_t zs = A.zs, as = A.as;
    if constexpr (LDS) {
        for (int k = lane; k < Na; k += 64) lds[k] = A.a[k];
        for (int q = lane; q < N * Na; q += 64) {
            int zz = q / Na, kk = q - zz * Na;
            lds[Na + q] = A.pol[(size_t)zz * A.zs + (size_t)kk * A.as];
        }
        __syncthreads();
        a = lds;
        pol = lds + Na;
        zs = Na;
        as = 1;
    }
    // cumulative transition rows, sequential sums as cumsum does
    __shared__ double cs[16 * 16];
    if (lane == 0) {
        for (int z = 0; z < N; ++z) {
            double acc = 0.0;
            for (int m = 0; m < N; ++m) {
                acc = acc + A.P[z * N + m];
                cs[z * N + m] = acc;
            }
        }
    }
    __syncthreads();
    int z = A.z1;
    double k = A.k1;
    double sum = k;
    if (lane == 0) {
        if (A.sim_k) A.sim_k[0] = k;
        if (A.sim_z) A.sim_z[0] = z;
    }
    int status = 0;
    for (int t = 1; t < A.T; ++t) {
        const double u = A.U[t - 1];
        // ---- state transition
        bool lt = lane < N && u < cs[z * N + lane];
        unsigned long long m = __ballot(lt);
        if (m == 0) {
            status = 1;  // the reference's find() would return empty and error
            break;
        }
        z = __ffsll((long long)m) - 1;
        // ---- segment of k in a_grid: largest i with a[i] <= k, clamped to [0, Na-2]
        int lo = 0, hi = Na;  // invariant: a[lo..] ... answer in [lo-1, hi-1]
        while (hi - lo > 64) {
            int step = (hi - lo + 63) / 64;
            int p = lo + lane * step;
            bool le = p < hi && a[p] <= k;
            int c = __popcll(__ballot(le));
            if (c == 0) {
                hi = lo;
                break;
            }
            lo = lo + (c - 1) * step;
            hi = min(lo + step, hi);
        }
        int cnt;
        {
            int p = lo + lane;
            bool le = p < hi && a[p] <= k;
            cnt = __popcll(__ballot(le));
        }
        int seg = lo + cnt - 1;
        seg = seg < 0 ? 0 : (seg > Na - 2 ? Na - 2 : seg);
        const double* y = pol + (size_t)z * zs;
        double x0 = a[seg], x1 = a[seg + 1];
        double y0 = y[(size_t)seg * as], y1 = y[(size_t)(seg + 1) * as];
        double tt = (k - x0) / (x1 - x0);
        k = y0 + tt * (y1 - y0);
        sum += k;
        if (lane == 0) {
            if (A.sim_k) A.sim_k[t] = k;
            if (A.sim_z) A.sim_z[t] = z;
        }
    }
    if (lane == 0) {
        A.out[0] = sum / (double)A.T;  // mean(sim_k)
        A.status[0] = status;
    }
}

int launch_sim_capital(const SimArgs& A, hipStream_t st) {
    if (A.N > 16 || A.N < 1) return fail(AIY_BAD_SHAPE, "simulation supports 1 <= N <= 16");
    if ((long long)A.Na * (A.N + 1) <= kSimLdsMax)
        sim_capital_kernel<true><<<1, 64, sizeof(double) * A.Na * (A.N + 1), st>>>(A);
    else
        sim_capital_kernel<false><<<1, 64, 0, st>>>(A);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}

}  // namespace aiy
