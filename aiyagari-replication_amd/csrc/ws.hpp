// Workspace (aiy_ws): per-shape device scratch owned by the library, reused across calls.
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

#include "../../include/aiyagari_hip.h"
#include "vfi_kernels.hpp"

struct aiy_ws {
    int64_t N = 0, Na = 0, Nl = 1;
    int dev = 0;
    // search knobs (aiy_ws_set_search)
    int coarse = 64;
    int CK = 1024;
    // VFI scratch
    double* EV = nullptr;
    double2* T = nullptr;
    double* coh = nullptr;
    double* best0 = nullptr;
    int* kf = nullptr;
    int* idx0 = nullptr;
    int* partial = nullptr;
    size_t partial_cap = 0;
    unsigned long long* diff = nullptr;      // device [2]
    unsigned long long* hitcount = nullptr;  // device [1]
    unsigned long long* hdiff = nullptr;     // pinned host [4]
    // generic scratch used by the EGM / distribution / simulation kernels
    double* g0 = nullptr;
    double* g1 = nullptr;
    double* g2 = nullptr;
    int* gi = nullptr;
    // timing of the dominant kernel
    bool timing = false, count_hits = false;
    std::vector<hipEvent_t> ev_start, ev_stop;
    int ev_used = 0;
    double tot_ms = 0;
    int64_t launches = 0;

    void free_all() {
        void* ps[] = {EV, T, coh, best0, kf, idx0, partial, diff, hitcount, g0, g1, g2, gi};
        for (void* p : ps)
            if (p) (void)hipFree(p);
        if (hdiff) (void)hipHostFree(hdiff);
        EV = nullptr; T = nullptr; coh = nullptr; best0 = nullptr; kf = nullptr;
        idx0 = nullptr; partial = nullptr; diff = nullptr; hitcount = nullptr; hdiff = nullptr;
        g0 = g1 = g2 = nullptr; gi = nullptr;
        partial_cap = 0;
    }
};

namespace aiy {
int ws_ensure_vfi(aiy_ws* ws);
int ws_timing_begin(aiy_ws* ws, hipStream_t st);
int ws_timing_end(aiy_ws* ws, hipStream_t st);
int ws_timing_drain(aiy_ws* ws);
int ws_read_diff(aiy_ws* ws, hipStream_t st, double* d);
int vfi_sweep_dev(aiy_ws* ws, const double* v_old, const double* a, const double* s,
                  const double* P, double r, double w, double beta, double sigma,
                  const int* hint, int coarse_first, int mode, double* v_new, int* idx,
                  double* pk, double* pc, double* diff_out, hipStream_t st);
int vfi_solve_dev(aiy_ws* ws, double* v_a, double* v_b, const double* a, const double* s,
                  const double* P, double r, double w, double beta, double sigma, double tol,
                  int64_t max_iter, int mode, int* idx, double* pk, double* pc,
                  const int* first_hint, int64_t* iters, int* out_new, hipStream_t st);
}  // namespace aiy
