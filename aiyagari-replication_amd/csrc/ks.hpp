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
    // nullable: the grid's slope tables (launch_ks_grid_tables: [nk] RN(1 / h_i), then [2·nk]
    // the interior weights of each node) — the tiled slopes use them, same values
    const double* kg_tab;
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
    // staged direct schedule, ONE launch per sweep (ks_dev_staged_sweep): block
    // rows [0, n_copy_rows) copy halo column q from halo_src[q] (a peer's buffer: system-scope
    // loads, after the wait below) to halo_dst[q] (n_copy_rows = n_halo; one wait-only row when
    // n_halo == 0 but wait_mask != 0); then the interior columns col_list[0 .. n_list); then the
    // boundary columns bnd_list[0 .. n_bnd), which wait in-kernel for every copy block
    const int* col_list;
    int n_list;
    const int* bnd_list;
    int n_bnd;
    const double* const* halo_src;
    double* const* halo_dst;
    int n_halo;
    int n_copy_rows;
    int copy_x;  // working copy blocks per copy row (the rest of the row returns at once)
    // copy rows wait until every slot q in wait_mask holds >= wait_v (host page, system scope;
    // timeout -> *err = 1 + q); null wait_flags: no wait
    const unsigned long long* wait_flags;
    unsigned long long wait_mask, wait_v;
    long long timeout_ticks;
    unsigned long long* err;
    // each working copy block adds 1 (agent scope, after its stores); boundary blocks start once
    // *copy_cnt >= copy_target (monotonic across launches; the host keeps the running total)
    unsigned long long* copy_cnt;
    unsigned long long copy_target;
    // block (0, 0) stores go_token (a per-handle launch sequence number, strictly increasing)
    // here once the neighbours' slots allow it; the other copy blocks poll it (one poller of the
    // host page per launch)
    unsigned long long* go;
    unsigned long long go_token;
    // the launch's first block stores pub_v into *pub_flag (system-scope release) before anything
    // else: the PREVIOUS launch on the stream (the sweep that produced version pub_v) is complete
    unsigned long long* pub_flag;
    unsigned long long pub_v;
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
int launch_ks_grid_tables(const double* kg, int nk, double* tab, hipStream_t st);
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
// the staged direct schedule's one launch per sweep (ks_staged_sweep_kernel); the working copy
// blocks per copy row (what each copy row adds to copy_cnt)
int launch_ks_staged_sweep(const KsArgs& A, const double* V, const double* dV,
                           const double* kopt, double* Vn, double* dVn, hipStream_t st);
int ks_staged_copy_blocks(int nk);
int launch_ks_hints(const KsArgs& A, const double* kopt, hipStream_t st);
int launch_ks_reldiff(const KsArgs& A, const double* V, const double* Vold,
                      unsigned long long* slots, hipStream_t st);
}  // namespace aiy
