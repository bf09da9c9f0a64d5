// Workspace (aiy_ws): per-shape device scratch owned by the library, reused across calls.
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

#include "../../include/aiyagari_hip.h"
#include "bellman.hpp"

struct aiy_ws {
    int64_t N = 0, Na = 0, Nl = 1;
    int dev = 0;
    // search knobs (aiy_ws_set_search)
    int coarse = 512;
    int CK = 1024;
    int variant = -1;  // -1: by size (see bell_sweep_dev); EGM knobs: bits 18-20 (egm_knob)
    // VFI scratch
    double* EV = nullptr;
    double2* T = nullptr;
    float* T32 = nullptr;
    double* Dm = nullptr;
    double* Dm8 = nullptr;
    double* Dt = nullptr;
    double* Dm512 = nullptr;
    double* best0 = nullptr;
    int* idx0 = nullptr;
    int* mom = nullptr;  // [N][Na] last sweep's argmax shift (tree kernel start-up heuristic)
    int* touched = nullptr;
    double* dis = nullptr;
    int* kf = nullptr;
    size_t kf_cap = 0;
    // key of the cached kf table (feasible prefixes depend on r, w, a, s, L only)
    bool kf_ok = false;
    double kf_r = 0, kf_w = 0;
    const void* kf_a = nullptr;
    const void* kf_s = nullptr;
    const void* kf_L = nullptr;
    int64_t kf_Nl = 0;
    bool kf_lab = false;
    int* tree_perm = nullptr;  // tree dispatch order for the cached kf (ws_tree_perm)
    int perm_cap = 0, perm_slots = 0;
    long long perm_key = 0;
    int* kf_last = nullptr;    // [Nl][N][ntile] kf of each tile's last state (ws_tree_perm)
    int kf_last_cap = 0;
    // disutility per labour level, cached with the key below (aiy_ws_invalidate resets)
    bool dis_ok = false;
    const void* dis_L = nullptr;
    int64_t dis_Nl = 0;
    double dis_psi = 0, dis_eta = 0;
    // small-grid one-launch sweep (bellman_wide_kernels.hip; aiy_ws_set_wide): used when
    // Na <= wide_max (-1: the default bound) with `wide_S` splits of `wide_NW` waves (0: by size)
    int wide_max = -1, wide_S = 0, wide_NW = 0, wide_SB = 0;
    bool cu_exclusive = false;  // aiy_ws_set_cu_exclusive
    // A9 chains (aiy_ws_set_sim): -1 by size, 0 the serial kernels, 1 / 2 the speculative-
    // segment chain (one workgroup / spread over 16) whenever it applies; its scratch (bytes)
    int sim_par = -1;
    double* sim_kbuf = nullptr;
    size_t sim_kcap = 0;
    unsigned long long* wdiff = nullptr;  // device [2][2*kDiffSlots]: the set not current is zero
    int wcur = 0;                         // the set the last wide sweep wrote
    unsigned* wcnt = nullptr;             // device [N·ntile] per-tile arrival counters (zero)
    size_t wcnt_cap = 0;
    unsigned long long* wpart = nullptr;  // device [N·ntile][S][64][2] partial bests
    size_t wpart_cap = 0;
    bool last_wide = false;               // the last VFI sweep on this workspace was wide
    unsigned long long* vdiff = nullptr;  // the diff slots the last VFI sweep wrote
    bool perm_ok = false;
    int* partial = nullptr;
    size_t partial_cap = 0;
    unsigned long long* diff = nullptr;      // device [2*kDiffSlots] {max bits, any}
    unsigned long long* hitcount = nullptr;  // device [4 * kDiffSlots]
    long long* trace = nullptr;              // device [8 * trace_cap] (instrumentation)
    int64_t trace_cap = 0;
    bool tracing = false;
    unsigned long long* hdiff = nullptr;     // pinned host [2*kDiffSlots + 4]
    // histogram scratch (A10)
    int* d_key = nullptr;
    int* d_off = nullptr;   // [N][Na+1] run offsets of the policy (the plan)
    double* d_wr = nullptr;
    double* d_mass = nullptr;
    double* d_part = nullptr;
    // speculative histogram iteration: ring of dist_m + 1 λ buffers, per-push diff slots
    size_t dist_n = 0;
    int dist_m = 0;
    double* dist_ring = nullptr;
    unsigned long long* dist_slots = nullptr;   // device [2 dist_m + 1][2*kDiffSlots]
    unsigned long long* dist_hslots = nullptr;  // pinned host, two copies (batches in flight)
    hipEvent_t dist_ev[2] = {nullptr, nullptr};
    void free_dist_spec() {
        if (dist_ring) (void)hipFree(dist_ring);
        if (dist_slots) (void)hipFree(dist_slots);
        if (dist_hslots) (void)hipHostFree(dist_hslots);
        for (auto& e : dist_ev) {
            if (e) (void)hipEventDestroy(e);
            e = nullptr;
        }
        dist_ring = nullptr; dist_slots = nullptr; dist_hslots = nullptr;
        dist_n = 0; dist_m = 0;
    }
    // generic scratch used by the EGM / distribution / simulation kernels
    double* g0 = nullptr;
    double* g1 = nullptr;
    double* g2 = nullptr;
    int* gi = nullptr;
    // speculative solve (aiy_ws_set_speculation): ring of spec_max + 1 value buffers, spec_max
    // policy sets and one folded-diff slot per sweep of a batch
    int spec_max = 16;
    size_t spec_n = 0;  // states per buffer the rings were sized for (0 = not allocated)
    double* spec_v = nullptr;
    int* spec_idx = nullptr;
    double* spec_pol = nullptr;                 // [spec_max][3][N*Na] (k, c, l)
    int spec_m = 0;                             // spec_max the rings were sized for
    unsigned long long* spec_diff = nullptr;    // device [2 * 2*spec_max]: a pair per sweep
    unsigned long long* spec_hdiff = nullptr;   // pinned host, two copies (batches in flight)
    hipEvent_t spec_ev[2] = {nullptr, nullptr};
    // speculative EGM solve: ring of spec_max + 1 policy_c buffers, per-step diff slots + flag
    size_t egm_spec_n = 0;
    int egm_spec_m = 0;
    double* egm_ring = nullptr;
    unsigned long long* egm_slots = nullptr;    // device [2 spec_max + 1][2*kDiffSlots + 2]
    unsigned long long* egm_hslots = nullptr;   // pinned host, two copies (batches in flight)
    hipEvent_t egm_ev[2] = {nullptr, nullptr};  // end of each in-flight batch's slot copy
    // chained EGM solve (Na > 1,024): the second â / c̃ pair (step parity)
    double* egm_x2 = nullptr;
    double* egm_y2 = nullptr;
    int* egm_seg = nullptr;  // [N][Na] interp1 segments of the last step (hints), -1 = none
    void free_egm_spec() {
        if (egm_ring) (void)hipFree(egm_ring);
        if (egm_slots) (void)hipFree(egm_slots);
        if (egm_hslots) (void)hipHostFree(egm_hslots);
        for (auto& e : egm_ev) {
            if (e) (void)hipEventDestroy(e);
            e = nullptr;
        }
        egm_ring = nullptr; egm_slots = nullptr; egm_hslots = nullptr;
        egm_spec_n = 0; egm_spec_m = 0;
    }
    // batched candidate rates (config 4, aiy_vfi_solve_batch_dev): per-candidate blocks of the
    // tree-screen scratch, sized for bC candidates
    int64_t bC = 0;
    double* bEV = nullptr;
    double* bDt = nullptr;
    double* bDm8 = nullptr;
    double* bDm512 = nullptr;
    double* bbest0 = nullptr;
    int* bidx0 = nullptr;
    int* bmom = nullptr;
    int* bkf = nullptr;
    int* bstop = nullptr;                  // device [bC]
    unsigned long long* bslots = nullptr;  // device [bC][2][2*kDiffSlots]
    double* brw = nullptr;                 // device [2][bC]: r then w
    int* hstop = nullptr;                  // pinned [bC]
    unsigned long long* hslots = nullptr;  // pinned [bC][2*kDiffSlots]
    void free_batch() {
        void* ps[] = {bEV, bDt, bDm8, bDm512, bbest0, bidx0, bmom, bkf, bstop, bslots, brw};
        for (void* p : ps)
            if (p) (void)hipFree(p);
        if (hstop) (void)hipHostFree(hstop);
        if (hslots) (void)hipHostFree(hslots);
        bEV = bDt = bDm8 = bDm512 = bbest0 = brw = nullptr;
        bidx0 = bkf = bstop = bmom = nullptr;
        bslots = nullptr;
        hstop = nullptr;
        hslots = nullptr;
        bC = 0;
    }
    // timing of the dominant kernel
    bool timing = false, count_hits = false;
    std::vector<hipEvent_t> ev_start, ev_stop;
    int ev_used = 0;
    double tot_ms = 0;
    int64_t launches = 0;

    void free_spec() {
        void* ps[] = {spec_v, spec_idx, spec_pol, spec_diff};
        for (void* p : ps)
            if (p) (void)hipFree(p);
        if (spec_hdiff) (void)hipHostFree(spec_hdiff);
        for (auto& e : spec_ev) {
            if (e) (void)hipEventDestroy(e);
            e = nullptr;
        }
        spec_v = nullptr; spec_idx = nullptr; spec_pol = nullptr; spec_diff = nullptr;
        spec_hdiff = nullptr; spec_n = 0; spec_m = 0;
    }
    void free_all() {
        void* ps[] = {EV, T, T32, Dm, Dm8, Dt, Dm512, touched, best0, idx0, mom, dis, kf, partial, diff, hitcount, trace, g0, g1, g2, gi,
                      d_key, d_off, d_wr, d_mass, d_part, egm_x2, egm_y2, egm_seg, tree_perm,
                      kf_last, wdiff, wcnt, wpart, sim_kbuf};
        for (void* p : ps)
            if (p) (void)hipFree(p);
        free_spec();
        free_batch();
        free_egm_spec();
        free_dist_spec();
        if (hdiff) (void)hipHostFree(hdiff);
        EV = nullptr; T = nullptr; T32 = nullptr; Dm = nullptr; Dm8 = nullptr; Dt = nullptr; Dm512 = nullptr; touched = nullptr; best0 = nullptr; dis = nullptr; kf = nullptr; kf_cap = 0;
        kf_ok = false;
        idx0 = nullptr; mom = nullptr; partial = nullptr; diff = nullptr; hitcount = nullptr; trace = nullptr; trace_cap = 0; hdiff = nullptr;
        g0 = g1 = g2 = nullptr; gi = nullptr;
        egm_x2 = egm_y2 = nullptr;
        egm_seg = nullptr;
        tree_perm = nullptr; perm_cap = 0; perm_ok = false;
        kf_last = nullptr; kf_last_cap = 0;
        wdiff = nullptr; wcnt = nullptr; wcnt_cap = 0; wpart = nullptr; wpart_cap = 0; wcur = 0;
        sim_kbuf = nullptr; sim_kcap = 0;
        last_wide = false; vdiff = nullptr; dis_ok = false;
        d_key = d_off = nullptr; d_wr = d_mass = d_part = nullptr;
        partial_cap = 0;
    }
};

namespace aiy {
// EGM A/B knobs on the workspace's variant word, above the VFI geometry bits (0-17), so a VFI
// variant never changes the EGM path on a shared workspace
constexpr int kEgmTwoLaunch = 1 << 18;  // the two-launch step even for Na <= 1,024
constexpr int kEgmNoChain = 1 << 19;    // solve loop: two launches per step, no chaining
constexpr int kEgmNoHints = 1 << 20;    // interp1 without the previous step's segment windows
inline bool egm_knob(const aiy_ws* ws, int bit) { return ws->variant >= 0 && (ws->variant & bit); }
struct BellCall {
    bool labor = false;
    int64_t Nl = 1;
    const double* L = nullptr;
    double psi = 0, eta = 0;
    const double* v_old = nullptr;
    const double* a = nullptr;
    const double* s = nullptr;
    const double* P = nullptr;
    double r = 0, w = 0, beta = 0, sigma = 0;
    const int* hint = nullptr;
    int mode = 0;
    bool keep_incoming = true;
    double* v_new = nullptr;
    int* idx = nullptr;
    double* pk = nullptr;
    double* pl = nullptr;
    double* pc = nullptr;
    double* diff_out = nullptr;
    void* prev_diff_out = nullptr;  // [2] u64: the previous sweep's folded {max bits, any}
};
int ws_ensure_bell(aiy_ws* ws, size_t partial_slots);
int ws_timing_begin(aiy_ws* ws, hipStream_t st);
int ws_timing_end(aiy_ws* ws, hipStream_t st);
int ws_timing_drain(aiy_ws* ws);
int ws_dispatch_arm(aiy_ws* ws);
void ws_dispatch_commit(aiy_ws* ws);
int ws_read_diff(aiy_ws* ws, hipStream_t st, double* d);
int bell_sweep_dev(aiy_ws* ws, const BellCall& c, hipStream_t st);
int bell_solve_dev(aiy_ws* ws, BellCall c, double* v_a, double* v_b, double tol,
                   int64_t max_iter, int64_t* iters, int* out_new, hipStream_t st);
int bell_solve_batch_dev(aiy_ws* ws, int64_t C, const double* r, const double* w, double* v_a,
                         double* v_b, const double* a, const double* s, const double* P,
                         double beta, double sigma, double tol, int64_t max_iter, int use_hint,
                         int* idx, double* pk, double* pc, int64_t* iters, int* which,
                         hipStream_t st);
int launch_reduce_slots(const unsigned long long* slots, void* out, hipStream_t st);
double fold_slots_host(const unsigned long long* h);
int launch_disutility(const double* L, int Nl, double psi, double eta, double* dis,
                      hipStream_t st);
}  // namespace aiy
