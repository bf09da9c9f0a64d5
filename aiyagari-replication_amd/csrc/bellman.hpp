// Launch interface of the Bellman kernels (bellman_kernels.hip): A1 (Nl = 1) and A3.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace aiy {

struct BellArgs {
    int N, Na, Nl;   // Nl = 1 for A1
    bool keep_incoming;  // A3: states with no feasible choice keep v_new's incoming value
    bool labor;      // A3 semantics (cash (1+r)a + (w s) L, disutility, keep-if-infeasible)
    int np;          // sigma-1 when sigma is an integer in [2, 9]; 0 = generic sigma
    int coarse;      // init coarse stride S (0 = no coarse scan)
    int CK;          // candidates a' per work item
    int variant;     // screen kernel geometry (tuning): bit0 R=4, bit1 register cap, bit2 fp64-only screen
    double r, w, beta, sigma;
    const double* v_old;
    const double* a;
    const double* s;
    const double* P;
    const double* L;    // labour grid (A3) or nullptr
    const double* dis;  // psi*L^(1+eta)/(1+eta) per level (A3) or nullptr
    const int* hint;    // nullable: last sweep's linear index (l + Nl*k)
    // scratch
    double* EV;
    double2* T;
    float* T32;     // chunk-relative fp32 screening table (nullable: fp64 screen only)
    double* best0;
    int* idx0;
    int* kf;       // [Nl][N][Na] feasible prefix lengths #{k : a_k < coh(j, l)}
    bool kf_valid; // kf already holds the values for (r, w, a, s, L)
    int* partial;
    unsigned long long* hitcount;  // nullable
    // outputs
    double* v_new;
    int* idx;   // linear index l + Nl*k (== k for A1)
    double* pk;
    double* pl;  // A3 only (nullable)
    double* pc;
    unsigned long long* diff;  // nullable, [2]
};

int launch_bell_table(const BellArgs& A, hipStream_t st);
int launch_bell_kf(const BellArgs& A, hipStream_t st);
int launch_bell_init(const BellArgs& A, hipStream_t st);
int launch_bell_screen(const BellArgs& A, hipStream_t st);
int launch_bell_plain(const BellArgs& A, hipStream_t st);
int launch_bell_merge(const BellArgs& A, int use_partial, hipStream_t st);
size_t bell_partial_slots(const BellArgs& A);

}  // namespace aiy
