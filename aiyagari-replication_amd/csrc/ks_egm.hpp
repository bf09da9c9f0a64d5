// Launch interface of the Krusell-Smith EGM kernel (ks_egm_kernels.hip, A8).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace aiy {
// per (s_i, K_i) scalars of Krusell_Smith_EGM.m:139-175, computed on the host with libm in the
// script's operation order (ks_egm_host.cpp; oracle/aiy_oracle.c orc_ks_egm_pairs)
struct KsEgmPair {
    int kd[4];      // K''_idx per s_j (nearest K_grid point of the ALM forecast of K')
    double Rn[4];   // (1 + r_next) - delta
    double Wn[4];   // w_next * eps_next * l_bar
    double R;       // (1 + r) - delta
    double We;      // w * eps * l_bar
};
struct KsEgmArgs {
    int nk, nK, max_iter;
    const double* k_grid;
    const double* P;          // 4 x 4 row-major
    const KsEgmPair* pairs;   // [s_i * nK + K_i]
    double beta, k_min, k_max, tol;
};
struct KsEgmOut {
    int iters;
    int status;  // 1: an (s, K) pair had fewer than 2 valid EGM points
    double diff;
};
size_t ks_egm_lds_bytes(int nk, int nK);
bool ks_egm_fits(int nk, int nK);
int launch_ks_egm_solve(const KsEgmArgs& A, double* kopt, KsEgmOut* out, hipStream_t st);
size_t ks_egm_jacobi_lds_bytes(int nk);
int launch_ks_egm_jacobi(const KsEgmArgs& A, const double* src, double* dst,
                         unsigned long long* slots, int* status, hipStream_t st);
}  // namespace aiy
