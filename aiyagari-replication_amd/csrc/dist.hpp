// Launch interface of the histogram kernels (dist_kernels.hip, A10).
#pragma once
#include <hip/hip_runtime.h>

namespace aiy {
// Summation order of a destination's mass (the A10 definition, restated by the C oracle
// orc_dist_*): the terms landing in (i, k), in ascending source j, are summed sequentially in
// chunks of kDistChunk consecutive terms and the chunk sums are summed sequentially.  A run of
// at most kDistChunk terms is the plain sequential sum; a long run (the borrowing constraint,
// the top of the grid) has a dependent chain of ≈ L/G + G additions instead of L.
constexpr int kDistChunk = 32;
// a push wave stages its source range in LDS when it holds at most this many sources
// (8 KB per wave on the on-grid path, 16 KB with lottery weights)
constexpr int kDistStage = 1024;
// the one-launch push (a wave per productivity state) takes N <= kDistPushMaxN; larger N run
// the per-destination run gather + projection (two launches, any N)
constexpr int kDistPushMaxN = 16;

struct DistArgs {
    int N, Na;
    bool lottery;        // off-grid policy (kp) split between bracketing nodes
    const int* idx;      // on-grid policy [N][Na], 0-based
    const double* kp;    // off-grid policy [N][Na]
    const double* a;
    const double* P;     // row-major
    const double* lam;   // [N][Na]
    double* out;         // λ' [N][Na]
    int* key;            // plan [N][Na]: destination key of source j
    int* off;            // plan [N][Na+1]: off(i,k) = #{j : key(i,j) < k} (monotone keys)
    double* wr;          // plan [N][Na]: lottery weight of the upper node
    double* mass;        // scratch [N][Na] (non-monotone fallback only)
    unsigned long long* diff;  // [2*kDiffSlots]
    unsigned* flags;     // bit 0 non-monotone policy, bit 1 index out of range
    int stage;           // push: sources a wave stages in LDS (set by launch_dist_push)
    unsigned long long* diff_clear;  // push (monotone plan): the next push's slot set, zeroed
                                     // by the first workgroup (nullable)
    long long* trace;    // (instrumentation, aiy_ws_set_timing bit 2) per-wave phase records
};
// the policy's plan (keys, lottery weights, run offsets, flags) — once per policy
int launch_dist_prepare(const DistArgs& A, hipStream_t st);
// one push λ → λ' with max|λ'−λ| into A.diff (which the caller has cleared): one fused launch
// on a monotone plan with N <= kDistPushMaxN (which also zeroes A.diff_clear), the run gather +
// projection for larger N, the ordered-scan gather + projection on a non-monotone plan
int launch_dist_push(const DistArgs& A, bool fallback, hipStream_t st);
int launch_dist_capital(const double* lam, const double* a, int N, int Na, double* part,
                        double* out, hipStream_t st);
}  // namespace aiy
