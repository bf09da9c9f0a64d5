// Launch interface of the EGM kernels (egm_kernels.hip): A4 and A5 (labor = true).
#pragma once
#include <hip/hip_runtime.h>

#include "aiy_common.hpp"

namespace aiy {
struct EgmArgs {
    int N, Na;
    bool labor;
    int ns;  // sigma when sigma is an integer in [1, 63] (c^-sigma = 1/c^sigma), else 0
    double r, w, beta, sigma, amin, phi, theta;
    const double* c;  // policy_c [N][Na]
    const double* a;
    const double* s;
    const double* P;  // row-major N x N
    double* ahat;     // scratch [N][Na]
    double* cnext;    // scratch [N][Na]
    double* cout;     // policy_c_next
    double* pk;
    double* pl;       // A5 (nullable)
    unsigned long long* diff;  // [2]
    unsigned* flags;           // bit 0: a_hat not increasing (small-grid fused step: bit 1 of
                               // the diff slots' second word instead, see egm_fused_kernel)
    bool fused;                // Na <= 1024: one launch per step (egm_fused_kernel)
    unsigned long long* diff_clear;  // chain: the next step's slot set (kEgmSlotWords
                                     // words), zeroed by this launch's first workgroup (nullable)
    double* ahat_next;               // chain: step t+1's â and c̃ (the other scratch pair)
    double* cnext_next;
    int* seg;                        // [N][Na] interp1 segment of each query at the last step
                                     // (a verified hint for the next; -1 = none)
    long long* trace;                // (instrumentation, aiy_ws_set_timing bit 2) per-wave
                                     // phase records of the interp / chain kernels
};
constexpr int kEgmSlotWords = 2 * kDiffSlots + 2;  // {max bits, any} x kDiffSlots + flag word
constexpr int kEgmFusedMaxNa = 1024;  // egm_fused_kernel: one state per thread
int launch_egm_step(const EgmArgs& A, hipStream_t st);
// the chained solve (Na > 1,024): the Euler RHS of the first step, then one launch per step
// (interp1 of step t + the RHS of step t+1 on the same tiles)
int launch_egm_rhs(const EgmArgs& A, hipStream_t st);
int launch_egm_chain(const EgmArgs& A, hipStream_t st);
}  // namespace aiy
