// Launch interface of the Bellman kernels (bellman_kernels.hip): A1 (Nl = 1) and A3.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

#include "dispatch.hpp"

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
    int* mom;           // nullable [N][Na]: the argmax's shift in k over the last hinted sweep
    const int* perm;    // nullable [N·ntile]: tree dispatch order (block b → item perm[b]); see
                        // ws_tree_perm — work order only
    int perm_slots;     // entries of perm (the hybrid launch runs perm_slots / 2 workgroups)
    int tw;             // tree tile width (states per one-wave tile, R = 1); 0 = 64
                        // (tree kernel: read for an extrapolated start, rewritten; heuristic
                        // only — any start is a valid screening bar)
    // scratch
    double* EV;
    double2* T;
    float* T32;     // chunk-relative fp32 screening table (nullable: fp64 screen only)
    double* Dm;     // [N][nb] max of the screening key D over each 64-candidate block (chunked screen)
    double* Dt;     // [N][Na] the screening key D alone (tree screen)
    double* Dm8;    // [N][nb8] ... over each aligned 8-candidate block (tree screen)
    double* Dm512;  // [N][nb512] ... over each aligned 512-candidate block (tree screen)
    int nb, nb8, nb512;  // ceil(Na / 64), ceil(Na / 8), ceil(Na / 512)
    bool tree;      // tree screen (default) instead of the chunked screen + merge
    double* best0;
    int* idx0;
    int* kf;       // [Nl][N][Na] feasible prefix lengths #{k : a_k < coh(j, l)}
    bool kf_valid; // kf already holds the values for (r, w, a, s, L)
    int* partial;   // [nlb][nchunk][N][Na] chunk improvements; -1 between sweeps
    int* touched;   // [N][Na] 1 when some chunk wrote `partial` for the state this sweep
    unsigned long long* hitcount;  // nullable, [4]: exact evals, superblock, block, fine tests
    long long* trace;  // nullable: per tree work item {t0, t1, xcc, nsup, nblk, nfine, nhits, item}
    // outputs
    double* v_new;
    int* idx;   // linear index l + Nl*k (== k for A1)
    double* pk;
    double* pl;  // A3 only (nullable)
    double* pc;
    unsigned long long* diff;  // nullable, [2]
    unsigned long long* fold;  // nullable [2]: the table kernel folds the previous sweep's diff slots here
    // batched candidate rates (config 4; A1 tree screen only).  C <= 1: a single candidate.
    // C > 1: every per-state array above is C consecutive blocks of its single layout, diff is
    // [C][2][2*kDiffSlots] (parity = sweep & 1 selects the set this sweep writes).
    int C;
    bool ev_mfma;      // EV = (βP)·V by fp64 MFMA (bell_ev_mfma_kernel) before the table kernel
    const double* rv;  // [C] device: r of each candidate
    const double* wv;  // [C] device: w of each candidate
    const int* stop;   // [C] device: nonzero = stopped at that sweep (skipped from then on)
    int parity;
};

// EV by fp64 MFMA from this productivity-grid size up (the variant bits 14 / 15 force VALU /
// MFMA); below it the table kernel's sequential VALU sum, which the C oracle restates bit for
// bit.  The MFMA's accumulation order is the hardware's: parity there is to rounding (MATLAB's
// own BLAS order for beta*P*v_old is unpinned).
constexpr int kEvMfmaMinN = 32;
inline bool bell_ev_mfma(int N, int variant) {
    if (variant >= 0 && (variant & 16384)) return false;
    if (variant >= 0 && (variant & 32768)) return true;
    return N >= kEvMfmaMinN;
}
// states per tree tile (R states per lane): 64·R, or A.tw for the one-state-per-lane geometry
inline int bell_tile_width(const BellArgs& A, int R) { return (R == 1 && A.tw > 0) ? A.tw : 64 * R; }
// one-wave tiles per workgroup (variant bits 16-17: 1, 2, 4, 8), used with a dispatch
// permutation (A.perm, which then holds -1 in the last workgroup's unused slots); instantiated
// for A1 at sigma = 5 (np = 4), one state per lane, one wave per tile
inline int bell_tree_pack(const BellArgs& A) {
    if (!(A.np == 4 && !A.labor && A.tree && (A.variant & (1 | 2 | 4 | 8)) == 0)) return 1;
    return (A.variant & (1 << 26)) ? 2 : 1 << ((A.variant >> 16) & 3);
}
// variant bit 26 (with a permutation): the hybrid launch, two-wave workgroups that run either
// two one-wave tiles or one heavy tile on both waves; bits 27-29: cooperative tiles per XCD
// range, 8 << value (7: none)
inline bool bell_tree_hybrid(const BellArgs& A) {
    return (A.variant & (1 << 26)) && bell_tree_pack(A) == 2;
}
inline int bell_tree_coop_per_xcd(const BellArgs& A) {
    const int v = (A.variant >> 27) & 7;
    return v == 7 ? 0 : 8 << v;  // (7: none — the hybrid launch's own cost, for A/B)
}
// The small-grid sweep (bellman_wide_kernels.hip): ONE launch per sweep, a workgroup of NW
// waves per (64-state tile, split of the candidate range), S splits per tile.  Every workgroup
// holds its row's feasible range in LDS: (a_k, D_k) and EV_k, 24 B per candidate.
constexpr int kWideMaxSplits = 16;
constexpr size_t kWideMaxLds = 144 * 1024;  // dynamic part (the wave bests take <= 12 KiB more)
inline size_t bell_wide_lds(int Na, int S, int NW) {
    (void)S;
    (void)NW;
    return (size_t)Na * 24 + ((size_t)Na + 7) / 8 * 8;
}
// flags (results identical): kWideBatch = a block with >= 4 voted candidates evaluates all
// eight as independent chains, kWideBatch2 from 2 (the default: tools/wide_tune.py,
// profiles/r05_g47_wide_flags.txt); kWideClimb = the bar climbs from the hint's window (measured
// slower than the window alone)
constexpr int kWideBatch = 1, kWideClimb = 2, kWideBatch2 = 4;
constexpr int kWideDefaultFlags = kWideBatch2;
constexpr int kWideMaxNl = 16;  // labour levels the small-grid sweep holds in registers
// a workgroup asking for this much LDS has its CU to itself (160 KiB per CU on gfx950)
constexpr size_t kExclusiveLds = 88 * 1024;
int launch_bell_wide(const BellArgs& A, int S, int NW, int SB, unsigned long long* old_slots,
                     unsigned* cnt, unsigned long long* part, int flags, size_t min_lds,
                     hipStream_t st);
int launch_bell_ev_mfma(const BellArgs& A, hipStream_t st);
int launch_bell_table(const BellArgs& A, hipStream_t st);
int launch_bell_kf(const BellArgs& A, hipStream_t st);
int launch_kf_tile_last(const int* kf, int rows, int Na, int TW, int ntile, int* out,
                        hipStream_t st);
int launch_bell_init(const BellArgs& A, hipStream_t st);
int launch_bell_screen(const BellArgs& A, hipStream_t st);
int launch_bell_tree(const BellArgs& A, hipStream_t st);
// Timing of the dominant kernel: dispatch.hpp (events recorded by the tree launch itself).
int launch_bell_plain(const BellArgs& A, hipStream_t st);
int launch_bell_merge(const BellArgs& A, int use_partial, hipStream_t st);
int launch_bell_table_batch(const BellArgs& A, unsigned long long* slots, int sweep, double tol,
                            hipStream_t st);
size_t bell_partial_slots(const BellArgs& A);


}  // namespace aiy
