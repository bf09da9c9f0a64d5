// Launch interface of the VFI kernels (vfi_kernels.hip); used by capi.cpp.
#pragma once
#include <hip/hip_runtime.h>

namespace aiy {

struct VfiArgs {
    int N, Na;
    int np;       // sigma-1 when sigma is an integer in [2, 9]; 0 = generic sigma
    int coarse;   // coarse stride of the init scan (0 = none)
    int CK;       // candidates per work item (k-chunk)
    double r, w, beta, sigma;
    const double* v_old;
    const double* a;
    const double* s;
    const double* P;
    const int* hint;  // nullable
    // scratch
    double* EV;
    double2* T;
    double* coh;
    int* kf;
    double* best0;
    int* idx0;
    int* partial;
    unsigned long long* hitcount;  // nullable
    // outputs
    double* v_new;
    int* idx;
    double* pk;  // nullable
    double* pc;  // nullable
    unsigned long long* diff;  // nullable, [2]
};

int launch_vfi_table(const VfiArgs& A, hipStream_t st);
int launch_vfi_init(const VfiArgs& A, hipStream_t st);
int launch_vfi_screen(const VfiArgs& A, hipStream_t st);
int launch_vfi_plain(const VfiArgs& A, hipStream_t st);
int launch_vfi_merge(const VfiArgs& A, int use_partial, hipStream_t st);

}  // namespace aiy
