// Launch interface of the Monte-Carlo capital-supply kernel (sim_kernels.hip, A9).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace aiy {
struct SimArgs {
    int N, Na, T;
    int z1;         // 0-based sim_z(1)
    double k1;      // sim_k(1)
    const double* pol;  // policy_k: element (z, k) at pol[z*zs + k*as]
    size_t zs, as;
    const double* a;
    const double* P;    // row-major N x N
    const double* U;    // T-1 uniforms
    double* out;        // [1] mean(sim_k)
    double* sim_k;      // nullable [T]
    int* sim_z;         // nullable [T], 0-based
    int* status;        // [1] 0 ok, 1 find() empty
    // batched chains (config 4): C > 1 runs C independent chains, one workgroup each; chain c
    // reads pol + c·pcs and U + c·ucs and writes out[c], status[c] (no paths)
    int C;
    size_t pcs, ucs;
    // reserve whole CUs (>= kSimExclusiveLds of LDS per chain workgroup) so no solve block
    // shares the chain's CU — opt-in (aiy_ws_set_cu_exclusive on the chain's workspace; the GE
    // driver sets it), ADVICE r5
    bool exclusive;
    // the speculative-segment chain (sim_kernels.hip): its scratch, sim_par_scratch_bytes(T, C)
    // (null: the serial kernels); par: -1 by size, 0 never, 1 whenever it applies (one
    // workgroup per chain), 2 whenever it applies (the spread four-launch variant)
    double* kscr;
    int par;
};
// the speculative chain's scratch: the k paths (T doubles per chain), the state paths (T bytes
// per chain) and per chain {Te, 16 repair flags} (ints)
inline size_t sim_par_scratch_bytes(long long T, long long C) {
    if (C < 1) C = 1;
    return (size_t)(8 * T * C) + (((size_t)(T * C) + 7) & ~(size_t)7) + (size_t)(4 * 17 * C);
}
int launch_sim_capital(const SimArgs& A, hipStream_t st);
}  // namespace aiy
