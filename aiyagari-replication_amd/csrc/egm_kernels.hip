// A4 / A5 — EGM inversion + interpolation step on gfx950.
//   A4: Aiyagari_EGM.m:75-107 (GE copy :177-211)
//   A5: Aiyagari_Endogenous_Labor_EGM.m:68-104 (GE copy :174-211)
// Arrays are [N][Na] (== MATLAB's Na x N policy_c, column j = productivity state).
//
// Kernel 1 (one thread per asset node a, all N states): u'(c_m) once per (m, a), then for
//   every j the Euler right-hand side Σ_m ((β(1+r))·P(j,m))·c_m^-σ in m order (:80-85),
//   c̃ = RHS^(-1/σ) (:88) and the endogenous grid â = ((c̃ + a) − w s_j)/(1+r) (:92) — with
//   the labour FOC l = ((w s_j) c̃^-σ / φ)^(1/θ) (:86) and â = ((c̃ + a) − (w s_j) l)/(1+r) (:87)
//   in A5.
// Kernel 2 (one thread per (j, a)): interp1(â_j, y, a_grid(a), 'linear', 'extrap') by binary
//   search on the monotone â_j (y = a_grid in A4, c̃_j in A5), the borrowing clamp, the
//   recovered policies, and max|c_next − c| ignoring NaN (:106) via atomicMax on IEEE bits.
//   It also flags a non-increasing â_j (MATLAB's interp1 would sort or error there).
// HBM-bound: 24 B per state per iteration (c in, c_next out, policy_k out), +8 B with labour.
#include "aiy_common.hpp"
#include "egm.hpp"

namespace aiy {

__device__ __forceinline__ double uprime_dev(double c, double sigma, int ns) {
    return ns > 0 ? 1.0 / aiy_ipow(c, ns) : aiy_pow(c, -sigma);  // c.^(-sigma)
}

__device__ __forceinline__ double labor_dev(double c, double ws, double sigma, int ns,
                                            double phi, double theta) {
    double x = (ws * uprime_dev(c, sigma, ns)) / phi;  // u_prime_l_inv(w s .* u_prime_c(c))
    return (1.0 / theta == 1.0) ? x : aiy_pow(x, 1.0 / theta);
}

template <int NMAX>
__global__ void egm_rhs_kernel(EgmArgs A) {
    int a_i = blockIdx.x * blockDim.x + threadIdx.x;
    if (a_i >= A.Na) return;
    const int N = A.N, Na = A.Na;
    double up[NMAX];
#pragma unroll
    for (int m = 0; m < NMAX; ++m)
        if (m < N) up[m] = uprime_dev(A.c[(size_t)m * Na + a_i], A.sigma, A.ns);
    const double coef0 = A.beta * (1 + A.r);
    const double ag = A.a[a_i];
    for (int j = 0; j < N; ++j) {
        double acc = 0.0;
#pragma unroll
        for (int m = 0; m < NMAX; ++m)
            if (m < N) acc = acc + (coef0 * A.P[j * N + m]) * up[m];
        double cn = aiy_pow(acc, -1.0 / A.sigma);  // :88
        double ws = A.w * A.s[j];
        double ah;
        if (A.labor) {
            double ls = labor_dev(cn, ws, A.sigma, A.ns, A.phi, A.theta);
            ah = ((cn + ag) - ws * ls) / (1 + A.r);
        } else {
            ah = ((cn + ag) - ws) / (1 + A.r);
        }
        A.ahat[(size_t)j * Na + a_i] = ah;
        A.cnext[(size_t)j * Na + a_i] = cn;
    }
}

__global__ void egm_interp_kernel(EgmArgs A) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    bool ok = false;
    double d = 0.0;
    if (t < A.N * A.Na) {
        const int Na = A.Na;
        int j = t / Na, a_i = t - j * Na;
        const double* __restrict__ x = A.ahat + (size_t)j * Na;
        const double* __restrict__ y = A.labor ? A.cnext + (size_t)j * Na : A.a;
        double q = A.a[a_i];
        int sgi = seg_of_dev(x, Na, q);
        double tt = (q - x[sgi]) / (x[sgi + 1] - x[sgi]);
        double g = y[sgi] + tt * (y[sgi + 1] - y[sgi]);
        if (a_i > 0 && !(x[a_i - 1] < x[a_i])) atomicOr(A.flags, 1u);
        double ws = A.w * A.s[j];
        double cn;
        if (A.labor) {
            if (q < A.amin) g = A.amin;  // :91 (a no-op for a_grid >= amin)
            cn = g;
            double l = labor_dev(g, ws, A.sigma, A.ns, A.phi, A.theta);      // :95
            double k = ((1 + A.r) * q + ws * l) - g;                           // :98
            A.pk[t] = k < 0 ? 0.0 : k;                                         // :99
            if (A.pl) A.pl[t] = l;
        } else {
            if (g < A.amin) g = A.amin;  // :98
            A.pk[t] = g;
            cn = ((1 + A.r) * q + ws) - g;  // :102
        }
        A.cout[t] = cn;
        d = fabs(cn - A.c[t]);
        ok = (d == d);
    }
    block_max_to_slots(ok, d, A.diff);
}

int launch_egm_step(const EgmArgs& A, hipStream_t st) {
    if (A.N > 16) return fail(AIY_BAD_SHAPE, "EGM kernels support N <= 16 productivity states");
    if (A.N <= 8) egm_rhs_kernel<8><<<(A.Na + 127) / 128, 128, 0, st>>>(A);
    else egm_rhs_kernel<16><<<(A.Na + 127) / 128, 128, 0, st>>>(A);
    AIY_HIP(hipGetLastError());
    int n = A.N * A.Na;
    egm_interp_kernel<<<(n + 255) / 256, 256, 0, st>>>(A);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}

}  // namespace aiy
