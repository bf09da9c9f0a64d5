// Launch interface of the Krusell-Smith kernels (ks_kernels.hip, A6/A7).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

#include <vector>

namespace aiy {
struct KsSlice {   // per (K_i, s_i), computed on the host with libm (Krusell_Smith_VFI.m)
    int kp_idx;    // nearest K_grid index of the ALM forecast K' (:335-343)
    double a1;     // r_val + 1 - delta at the flipped current z (:332, :353-355)
    double a2;     // w_val * (eps * l_bar)
    double b1;     // r_table + 1 - delta (correct z, :152)
    double b2;     // w_table * (eps*l_bar + (1-eps)*mu) (:153)
};
struct KsArgs {
    int nk, nK;
    int node0, n_local;  // node range handled by this launch (sharding)
    const double* k_grid;
    const double* P;     // 4 x 4 row-major
    const KsSlice* slice;  // [s][K]
    double beta, k_min, k_max, tol;
    int howard, max_vfi;
    int* seg_hint;  // nullable [node]: k-segment of clamp(k_opt), written by improve, a hint for Howard
    // several s blocks in one launch (sharded path): blockIdx.y = q handles nodes
    // node0 + q·sstride + [0, n_local); ns = 1 (sstride unused) otherwise
    int ns, sstride;
    // direct (peer-read) schedule: the value / slope column c = s'·nK + K' that a forecast reads
    // lives at colV[c] / coldV[c] (the owning shard's buffer, on this or a peer device); null:
    // the launch's own V / dV arrays
    const double* const* colV;
    const double* const* coldV;
    // staged direct schedule: the fused Howard launch runs the columns col_list[0 .. n_list)
    // (interior or boundary subset of the shard's own columns) instead of the node range
    const int* col_list;
    int n_list;
    // ... and, in the same launch, n_halo extra block rows copy halo column q from halo_src[q]
    // (a peer's buffer: system-scope loads) to halo_dst[q]
    const double* const* halo_src;
    double* const* halo_dst;
    int n_halo;
};
struct KsParams {  // the 13-double parameter block, in order
    double beta, alpha, delta, k_min, k_max, ug, ub, l_bar, mu, z1, z2, e1, e2;
};
void ks_slices(const KsParams& p, const double* B, const double* K_grid, int nK,
               std::vector<KsSlice>& out);
struct KsOut {
    int iters;
    double rel;
};
bool ks_fused_fits(int nk, int nK);
int launch_ks_fused(const KsArgs& A, double* V, double* kopt, int* nfev, KsOut* out,
                    hipStream_t st);
int launch_ks_slopes(const KsArgs& A, const double* V, double* dV, hipStream_t st);
int launch_ks_slopes_cols(const KsArgs& A, const int* cols, int ncols, const double* V,
                          double* dV, hipStream_t st);
int launch_ks_improve(const KsArgs& A, const double* V, const double* dV, double* kopt,
                      int* nfev, hipStream_t st);
int launch_ks_howard(const KsArgs& A, const double* V, const double* dV, const double* kopt,
                     double* Vn, hipStream_t st);
// Howard sweep writing the next sweep's slopes too (dV must hold the slopes of V on every
// column the launch reads; Vn and dVn are written on the launch's nodes)
int launch_ks_halo_copy(const double* const* src, double* const* dst, int ncols, int nk,
                        hipStream_t st);
int launch_ks_howard_slopes(const KsArgs& A, const double* V, const double* dV,
                            const double* kopt, double* Vn, double* dVn, hipStream_t st);
int launch_ks_hints(const KsArgs& A, const double* kopt, hipStream_t st);
int launch_ks_reldiff(const KsArgs& A, const double* V, const double* Vold,
                      unsigned long long* slots, hipStream_t st);
}  // namespace aiy
