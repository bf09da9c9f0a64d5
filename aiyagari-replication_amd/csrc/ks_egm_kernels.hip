// A8 — Krusell-Smith EGM policy iteration (Krusell_Smith_EGM.m:129-209) on gfx950.
//
// The reference sweeps the (s_i outer, K_i inner) pairs Gauss-Seidel: k_opt(:,K_i,s_i) is
// overwritten (:199) as soon as it is computed and read by every later pair through
// k_opt(:, K''_idx, s_j) (:179).  That order is the result, so one workgroup runs the whole
// solve with k_opt resident in LDS and the pairs in sequence; inside a pair every phase is
// data-parallel over the k_size candidate k' points:
//   A  expectation (:155-189): per k' four pchip evaluations at the knot k' of the referenced
//      columns (interp1 'pchip', :179), c_next floor (:181), the expected marginal utility
//      summed s_j = 1..4 in order, c = 1/(beta*E), k_current (:188)
//   B  stable rank sort of k_current (MATLAB sort: ascending, NaN last, ties in index order,
//      :193); the valid points [k_min, k_max] are a contiguous run of the sorted order (:195)
//   C  griddedInterpolant(k_sorted, kp_sorted, 'pchip', 'nearest') at k_grid, clamped (:196-198)
// then max|k_opt - k_opt_old| (NaN ignored, :204) decides the next sweep.  All arithmetic is
// the C restatement's (oracle/aiy_oracle.c orc_ks_egm_*) operation for operation, so the
// result is bit-identical to it.
#include "aiy_common.hpp"
#include "ks_egm.hpp"
#include "pchip_dev.hpp"

namespace aiy {

constexpr int kEgmThreads = 256;

// a sorts strictly after b: ascending, NaN after every number (MATLAB sort)
__device__ __forceinline__ bool sort_gt(double a, double b) {
    return (a != a) ? (b == b) : (b == b && a > b);
}

__global__ __launch_bounds__(kEgmThreads) void ks_egm_solve_kernel(KsEgmArgs A, double* kopt_io,
                                                                   KsEgmOut* out) {
    extern __shared__ double lds[];
    const int nk = A.nk, nK = A.nK, n_all = nk * nK * 4;
    double* kg = lds;
    double* K = kg + nk;
    double* Kold = K + n_all;
    double* kc = Kold + n_all;
    double* xs = kc + nk;
    double* ys = xs + nk;
    __shared__ int s_lo, s_nv, s_flag;
    __shared__ double s_red[kEgmThreads / 64];
    const int tid = threadIdx.x;
    for (int q = tid; q < nk; q += blockDim.x) kg[q] = A.k_grid[q];
    for (int q = tid; q < n_all; q += blockDim.x) K[q] = kopt_io[q];
    __syncthreads();

    int it = 0, status = 0;
    double diff = __builtin_nan("");
    for (it = 1; it <= A.max_iter; ++it) {
        for (int q = tid; q < n_all; q += blockDim.x) Kold[q] = K[q];  // k_opt_old (:131)
        for (int s_i = 0; s_i < 4 && !status; ++s_i) {
            for (int K_i = 0; K_i < nK; ++K_i) {
                const KsEgmPair& pr = A.pairs[s_i * nK + K_i];
                if (tid == 0) {
                    s_lo = 0;
                    s_nv = 0;
                }
                // ---- A: k_current per k' (:155-189)
                for (int t = tid; t < nk; t += blockDim.x) {
                    const double kp = kg[t];
                    const int seg = seg_of_dev(kg, nk, kp);
                    double em = 0.0;
#pragma unroll
                    for (int s_j = 0; s_j < 4; ++s_j) {
                        const double* col = K + (s_j * nK + pr.kd[s_j]) * nk;
                        const double kpn = pchip_local(kg, col, nk, seg, kp);         // :179
                        const double cn = fmax((pr.Rn[s_j] * kp + pr.Wn[s_j]) - kpn, 1e-8);
                        em = em + (A.P[s_i * 4 + s_j] * pr.Rn[s_j]) / cn;          // :183
                    }
                    const double c = 1 / (A.beta * em);                             // :187
                    kc[t] = ((c + kp) - pr.We) / pr.R;                              // :188
                }
                __syncthreads();
                // ---- B: stable rank sort, valid run (:193-195)
                for (int t = tid; t < nk; t += blockDim.x) {
                    const double v = kc[t];
                    int rank = 0;
                    for (int j = 0; j < nk; ++j) {
                        const double u = kc[j];
                        rank += (sort_gt(v, u) || (j < t && !sort_gt(u, v))) ? 1 : 0;
                    }
                    xs[rank] = v;
                    ys[rank] = kg[t];
                    if (v < A.k_min) atomicAdd(&s_lo, 1);
                    if (v >= A.k_min && v <= A.k_max) atomicAdd(&s_nv, 1);
                }
                __syncthreads();
                const int lo = s_lo, nv = s_nv;
                if (nv < 2) {  // griddedInterpolant needs two sample points
                    status = 1;
                    break;
                }
                // ---- C: pchip through the valid points, 'nearest' outside, clamp (:196-199)
                const double* x = xs + lo;
                const double* y = ys + lo;
                double* dst = K + (s_i * nK + K_i) * nk;
                for (int t = tid; t < nk; t += blockDim.x) {
                    const double q = kg[t];
                    double v;
                    if (q < x[0]) v = y[0];
                    else if (q > x[nv - 1]) v = y[nv - 1];
                    else v = pchip_local(x, y, nv, seg_of_dev(x, nv, q), q);
                    v = fmin(v, A.k_max);
                    dst[t] = fmax(v, A.k_min);
                }
                __syncthreads();
            }
        }
        if (status) break;
        // max|k_opt - k_opt_old|, NaN ignored (:204)
        double m = -1.0;
        for (int q = tid; q < n_all; q += blockDim.x) {
            const double d = fabs(K[q] - Kold[q]);
            if (d == d) m = fmax(m, d);
        }
        for (int off = 32; off > 0; off >>= 1) m = fmax(m, __shfl_xor(m, off));
        if ((tid & 63) == 0) s_red[tid >> 6] = m;
        __syncthreads();
        if (tid == 0) {
            double mm = -1.0;
            for (int q = 0; q < kEgmThreads / 64; ++q) mm = fmax(mm, s_red[q]);
            const double dd = mm < 0 ? __builtin_nan("") : mm;
            s_flag = (dd < A.tol) ? 1 : 0;
            s_red[0] = dd;
        }
        __syncthreads();
        diff = s_red[0];
        const int stop = s_flag;
        __syncthreads();
        if (stop) break;
    }
    if (it > A.max_iter) it = A.max_iter;
    for (int q = tid; q < n_all; q += blockDim.x) kopt_io[q] = K[q];
    if (tid == 0) {
        out->iters = it;
        out->diff = diff;
        out->status = status;
    }
}

// F1 — the Jacobi variant (NOT the reference's result: the script is Gauss-Seidel, :199).
// Every (s_i, K_i) pair of a sweep reads the previous sweep's k_opt (`src`), so the pairs are
// independent: one workgroup per pair, all pairs of a sweep in one launch (4·K_size-way
// parallel instead of one workgroup walking them in order).  The per-pair phases A/B/C are the
// Gauss-Seidel kernel's; each workgroup also folds max|dst - src| over its column (NaN ignored)
// into the sweep's diff slots for the stop rule (:204).
__global__ __launch_bounds__(kEgmThreads) void ks_egm_jacobi_kernel(KsEgmArgs A,
                                                                    const double* __restrict__ src,
                                                                    double* __restrict__ dst,
                                                                    unsigned long long* slots,
                                                                    int* status) {
    extern __shared__ double lds[];
    const int nk = A.nk, nK = A.nK;
    double* kg = lds;
    double* kc = kg + nk;
    double* xs = kc + nk;
    double* ys = xs + nk;
    __shared__ int s_lo, s_nv;
    const int tid = threadIdx.x;
    const int pair = blockIdx.x, s_i = pair / nK;
    const KsEgmPair& pr = A.pairs[pair];
    for (int q = tid; q < nk; q += blockDim.x) kg[q] = A.k_grid[q];
    if (tid == 0) {
        s_lo = 0;
        s_nv = 0;
    }
    __syncthreads();
    for (int t = tid; t < nk; t += blockDim.x) {  // A (:155-189)
        const double kp = kg[t];
        const int seg = seg_of_dev(kg, nk, kp);
        double em = 0.0;
#pragma unroll
        for (int s_j = 0; s_j < 4; ++s_j) {
            const double* col = src + (size_t)(s_j * nK + pr.kd[s_j]) * nk;
            const double kpn = pchip_local(kg, col, nk, seg, kp);
            const double cn = fmax((pr.Rn[s_j] * kp + pr.Wn[s_j]) - kpn, 1e-8);
            em = em + (A.P[s_i * 4 + s_j] * pr.Rn[s_j]) / cn;
        }
        const double c = 1 / (A.beta * em);
        kc[t] = ((c + kp) - pr.We) / pr.R;
    }
    __syncthreads();
    for (int t = tid; t < nk; t += blockDim.x) {  // B (:193-195)
        const double v = kc[t];
        int rank = 0;
        for (int j = 0; j < nk; ++j) {
            const double u = kc[j];
            rank += (sort_gt(v, u) || (j < t && !sort_gt(u, v))) ? 1 : 0;
        }
        xs[rank] = v;
        ys[rank] = kg[t];
        if (v < A.k_min) atomicAdd(&s_lo, 1);
        if (v >= A.k_min && v <= A.k_max) atomicAdd(&s_nv, 1);
    }
    __syncthreads();
    const int lo = s_lo, nv = s_nv;
    if (nv < 2) {  // block-uniform: griddedInterpolant needs two points
        if (tid == 0) atomicOr(status, 1);
        block_max_to_slots(false, 0.0, slots);
        return;
    }
    const double* x = xs + lo;
    const double* y = ys + lo;
    const size_t base = (size_t)pair * nk;
    bool ok = false;
    double dmax = 0.0;
    for (int t = tid; t < nk; t += blockDim.x) {  // C (:196-199)
        const double q = kg[t];
        double v;
        if (q < x[0]) v = y[0];
        else if (q > x[nv - 1]) v = y[nv - 1];
        else v = pchip_local(x, y, nv, seg_of_dev(x, nv, q), q);
        v = fmin(v, A.k_max);
        v = fmax(v, A.k_min);
        dst[base + t] = v;
        const double d = fabs(v - src[base + t]);
        if (d == d) {
            dmax = ok ? fmax(dmax, d) : d;
            ok = true;
        }
    }
    block_max_to_slots(ok, dmax, slots);
}

size_t ks_egm_jacobi_lds_bytes(int nk) { return sizeof(double) * 4ull * nk; }

int launch_ks_egm_jacobi(const KsEgmArgs& A, const double* src, double* dst,
                         unsigned long long* slots, int* status, hipStream_t st) {
    ks_egm_jacobi_kernel<<<4 * A.nK, kEgmThreads, ks_egm_jacobi_lds_bytes(A.nk), st>>>(
        A, src, dst, slots, status);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}

size_t ks_egm_lds_bytes(int nk, int nK) {
    return sizeof(double) * (4ull * nk + 2ull * nk * nK * 4);
}
bool ks_egm_fits(int nk, int nK) { return ks_egm_lds_bytes(nk, nK) <= 150 * 1024; }

int launch_ks_egm_solve(const KsEgmArgs& A, double* kopt, KsEgmOut* out, hipStream_t st) {
    ks_egm_solve_kernel<<<1, kEgmThreads, ks_egm_lds_bytes(A.nk, A.nK), st>>>(A, kopt, out);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}

}  // namespace aiy
