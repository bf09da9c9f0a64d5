// A10 (new; the reference has no histogram — SURVEY §8(a) A10) — stationary distribution by
// histogram iteration:  λ'(m,k) = Σ_i P(i,m) · mass(i,k),  mass(i,k) = Σ_{j→k} λ(i,j).
//
// Scatter-free transpose-gather.  The policy maps j to a destination key k(j) (the grid index
// for a VFI policy; the bracket of a' for an off-grid EGM policy, whose mass is split between
// k and k+1 as a lottery).  Optimal policies are monotone in j (increasing differences,
// Topkis), so each key's preimage is ONE contiguous run of j.  Then:
//   heads   (per (i,j))  the first j of every run records itself in head[i][k]; a decrease of
//                        k(j) raises a flag (non-monotone policy → exact fallback kernel).
//   gather  (per (i,k))  one thread walks the run(s) ending in slot k in ascending j and
//                        accumulates — the same additions, in the same order, as the
//                        sequential scatter `mass[k(j)] += λ_j` of the C oracle, so the result
//                        is bit-identical, with no atomics and no cancellation.
//   project (per (m,k))  λ'(m,k) = Σ_i P(i,m)·mass(i,k) in i order, plus max|λ'−λ| (slots).
// Fallback (per (i,k), only when the flag is set): scan every j of the row in order.
#include "aiy_common.hpp"
#include "dist.hpp"

namespace aiy {

__global__ void dist_keys_kernel(DistArgs A) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= A.N * A.Na) return;
    const int Na = A.Na;
    int i = t / Na, j = t - i * Na;
    int key;
    if (A.lottery) {
        double x = A.kp[t];
        const double a0 = A.a[0], an = A.a[Na - 1];
        x = x < a0 ? a0 : x;
        x = x > an ? an : x;
        key = seg_of_dev(A.a, Na, x);
        A.wr[t] = (x - A.a[key]) / (A.a[key + 1] - A.a[key]);
    } else {
        key = A.idx[t];
        if (key < 0 || key >= Na) {
            atomicOr(A.flags, 2u);  // invalid index
            key = key < 0 ? 0 : Na - 1;
        }
    }
    A.key[t] = key;
    (void)i;
    (void)j;
}

__global__ void dist_heads_kernel(DistArgs A) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= A.N * A.Na) return;
    const int Na = A.Na;
    int i = t / Na, j = t - i * Na;
    int key = A.key[t];
    int prev = j > 0 ? A.key[t - 1] : -1;
    if (key != prev) {
        if (key < prev) atomicOr(A.flags, 1u);  // not monotone: a key may have several runs
        A.head[(size_t)i * Na + key] = j;
    }
}

// one thread per (i, k): accumulate the run(s) that land in slot k, ascending j
__global__ void dist_gather_kernel(DistArgs A) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= A.N * A.Na) return;
    const int Na = A.Na;
    int i = t / Na, k = t - i * Na;
    const int* __restrict__ key = A.key + (size_t)i * Na;
    const double* __restrict__ lam = A.lam + (size_t)i * Na;
    const int* __restrict__ head = A.head + (size_t)i * Na;
    double acc = 0.0;
    if (A.lottery) {
        const double* __restrict__ wr = A.wr + (size_t)i * Na;
        if (k >= 1) {
            int h = head[k - 1];
            if (h >= 0)
                for (int j = h; j < Na && key[j] == k - 1; ++j) acc = acc + lam[j] * wr[j];
        }
        int h = head[k];
        if (h >= 0)
            for (int j = h; j < Na && key[j] == k; ++j) acc = acc + lam[j] * (1 - wr[j]);
    } else {
        int h = head[k];
        if (h >= 0)
            for (int j = h; j < Na && key[j] == k; ++j) acc = acc + lam[j];
    }
    A.mass[t] = acc;
}

// exact fallback for non-monotone policies: every j of the row, in order
__global__ void dist_gather_scan_kernel(DistArgs A) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= A.N * A.Na) return;
    const int Na = A.Na;
    int i = t / Na, k = t - i * Na;
    const int* __restrict__ key = A.key + (size_t)i * Na;
    const double* __restrict__ lam = A.lam + (size_t)i * Na;
    double acc = 0.0;
    if (A.lottery) {
        const double* __restrict__ wr = A.wr + (size_t)i * Na;
        for (int j = 0; j < Na; ++j) {
            int q = key[j];
            if (q == k) acc = acc + lam[j] * (1 - wr[j]);
            else if (q + 1 == k) acc = acc + lam[j] * wr[j];
        }
    } else {
        for (int j = 0; j < Na; ++j)
            if (key[j] == k) acc = acc + lam[j];
    }
    A.mass[t] = acc;
}

__global__ void dist_project_kernel(DistArgs A) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    bool ok = false;
    double d = 0.0;
    if (t < A.N * A.Na) {
        const int N = A.N, Na = A.Na;
        int m = t / Na, k = t - m * Na;
        double acc = 0.0;
        for (int i = 0; i < N; ++i) acc = acc + A.P[i * N + m] * A.mass[(size_t)i * Na + k];
        A.out[t] = acc;
        d = fabs(acc - A.lam[t]);
        ok = (d == d);
    }
    block_max_to_slots(ok, d, A.diff);
}

// K = Σ_i Σ_j λ(i,j)·a_j: fixed-order block sums (deterministic), folded by one block
__global__ void dist_capital_kernel(const double* __restrict__ lam, const double* __restrict__ a,
                                    int N, int Na, double* __restrict__ part) {
    __shared__ double sh[256];
    double acc = 0.0;
    int n = N * Na;
    for (int t = blockIdx.x * 256 + threadIdx.x; t < n; t += gridDim.x * 256)
        acc = acc + lam[t] * a[t % Na];
    sh[threadIdx.x] = acc;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) sh[threadIdx.x] = sh[threadIdx.x] + sh[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = sh[0];
}
__global__ void fold_kernel(const double* __restrict__ part, int n, double* __restrict__ out) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        double acc = 0.0;
        for (int q = 0; q < n; ++q) acc = acc + part[q];
        out[0] = acc;
    }
}

int launch_dist_update(const DistArgs& A, bool fallback, hipStream_t st) {
    int n = A.N * A.Na;
    int g = (n + 255) / 256;
    if (!fallback) {
        AIY_HIP(hipMemsetAsync(A.head, 0xff, sizeof(int) * (size_t)n, st));
        dist_keys_kernel<<<g, 256, 0, st>>>(A);
        dist_heads_kernel<<<g, 256, 0, st>>>(A);
        dist_gather_kernel<<<g, 256, 0, st>>>(A);
    } else {
        dist_gather_scan_kernel<<<g, 256, 0, st>>>(A);
    }
    dist_project_kernel<<<g, 256, 0, st>>>(A);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}

int launch_dist_capital(const double* lam, const double* a, int N, int Na, double* part,
                        double* out, hipStream_t st) {
    constexpr int kBlocks = 256;
    dist_capital_kernel<<<kBlocks, 256, 0, st>>>(lam, a, N, Na, part);
    fold_kernel<<<1, 64, 0, st>>>(part, kBlocks, out);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}

}  // namespace aiy
