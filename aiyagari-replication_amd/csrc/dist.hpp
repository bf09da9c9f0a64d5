// Launch interface of the histogram kernels (dist_kernels.hip, A10).
#pragma once
#include <hip/hip_runtime.h>

namespace aiy {
struct DistArgs {
    int N, Na;
    bool lottery;        // off-grid policy (kp) split between bracketing nodes
    const int* idx;      // on-grid policy [N][Na], 0-based
    const double* kp;    // off-grid policy [N][Na]
    const double* a;
    const double* P;     // row-major
    const double* lam;   // [N][Na]
    double* out;         // λ' [N][Na]
    int* key;            // scratch [N][Na]
    int* head;           // scratch [N][Na]
    double* wr;          // scratch [N][Na]
    double* mass;        // scratch [N][Na]
    unsigned long long* diff;  // [2*kDiffSlots]
    unsigned* flags;     // bit 0 non-monotone policy, bit 1 index out of range
};
int launch_dist_update(const DistArgs& A, bool fallback, hipStream_t st);
int launch_dist_capital(const double* lam, const double* a, int N, int Na, double* part,
                        double* out, hipStream_t st);
}  // namespace aiy
