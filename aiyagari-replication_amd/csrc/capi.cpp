// C ABI (include/aiyagari_hip.h): workspace management, the device tier (*_dev) and the
// MATLAB-layout host tier.  Host code only; kernels live in *_kernels.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "aiy_common.hpp"
#include "ws.hpp"

namespace aiy {

int wait_event(hipEvent_t ev) {
    for (int spin = 0;; ++spin) {
        const hipError_t e = hipEventQuery(ev);
        if (e == hipSuccess) return AIY_OK;
        if (e != hipErrorNotReady) {
            (void)hipGetLastError();
            return fail(AIY_HIP_ERROR, "hipEventQuery failed: %s", hipGetErrorString(e));
        }
        if (spin > 256) std::this_thread::yield();
    }
}

static thread_local std::string g_err;

void set_error(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
}

int fail(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

// ---------------------------------------------------------------------------- workspace
template <class T>
static int dalloc(T** p, size_t n) {
    if (*p) return AIY_OK;
    hipError_t e = hipMalloc((void**)p, std::max<size_t>(n, 1) * sizeof(T));
    if (e != hipSuccess)
        return fail(AIY_NO_MEMORY, "hipMalloc(%zu bytes) failed: %s", n * sizeof(T),
                    hipGetErrorString(e));
    return AIY_OK;
}
template <class T>
static void dfree(T*& p) {
    if (p) (void)hipFree((void*)p);
    p = nullptr;
}

int ws_ensure_bell(aiy_ws* ws, size_t partial_slots) {
    size_t n = (size_t)ws->N * ws->Na;
    AIY_TRY(dalloc(&ws->EV, n));
    AIY_TRY(dalloc(&ws->T, n));
    AIY_TRY(dalloc(&ws->T32, 2 * (size_t)ws->N * (ws->Na + (ws->Na & 1))));
    AIY_TRY(dalloc(&ws->Dm, (size_t)ws->N * ((ws->Na + 63) / 64)));
    AIY_TRY(dalloc(&ws->Dm8, (size_t)ws->N * ((ws->Na + 7) / 8)));
    AIY_TRY(dalloc(&ws->Dt, n));
    AIY_TRY(dalloc(&ws->Dm512, (size_t)ws->N * ((ws->Na + 511) / 512)));
    AIY_TRY(dalloc(&ws->best0, n));
    AIY_TRY(dalloc(&ws->idx0, n));
    if (!ws->mom) {
        AIY_TRY(dalloc(&ws->mom, n));
        AIY_HIP(hipMemset(ws->mom, 0, n * sizeof(int)));
    }
    if (!ws->touched) {  // the merge kernel leaves touched = 0 and partial = -1 behind
        AIY_TRY(dalloc(&ws->touched, n));
        AIY_HIP(hipMemset(ws->touched, 0, n * sizeof(int)));
    }
    if (ws->partial && ws->partial_cap < partial_slots) dfree(ws->partial);
    if (!ws->partial) {
        AIY_TRY(dalloc(&ws->partial, partial_slots));
        AIY_HIP(hipMemset(ws->partial, 0xff, partial_slots * sizeof(int)));
        ws->partial_cap = partial_slots;
    }
    AIY_TRY(dalloc(&ws->diff, 2 * kDiffSlots));
    if (!ws->hitcount) {  // zero from the start: counting may be switched on before a sweep
        AIY_TRY(dalloc(&ws->hitcount, 4 * kDiffSlots));
        AIY_HIP(hipMemset(ws->hitcount, 0, 4 * kDiffSlots * sizeof(unsigned long long)));
    }
    AIY_TRY(dalloc(&ws->dis, (size_t)std::max<int64_t>(ws->Nl, 1)));
    if (!ws->hdiff)
        AIY_HIP(hipHostMalloc((void**)&ws->hdiff, (2 * kDiffSlots + 4) * sizeof(unsigned long long)));
    return AIY_OK;
}

int ws_timing_begin(aiy_ws* ws, hipStream_t st) {
    if (!ws->timing) return AIY_OK;
    if (ws->ev_used == (int)ws->ev_start.size()) AIY_TRY(ws_timing_drain(ws));
    AIY_HIP(hipEventRecord(ws->ev_start[ws->ev_used], st));
    return AIY_OK;
}
int ws_timing_end(aiy_ws* ws, hipStream_t st) {
    if (!ws->timing) return AIY_OK;
    AIY_HIP(hipEventRecord(ws->ev_stop[ws->ev_used], st));
    ws->ev_used++;
    return AIY_OK;
}
// dispatch-recorded events (dispatch.hpp) for the next timed launch on this thread; call
// ws_dispatch_commit after the launch whatever it returned
int ws_dispatch_arm(aiy_ws* ws) {
    if (!ws->timing) return AIY_OK;
    if (ws->ev_used == (int)ws->ev_start.size()) AIY_TRY(ws_timing_drain(ws));
    g_dispatch_ev = DispatchEvents{ws->ev_start[ws->ev_used], ws->ev_stop[ws->ev_used]};
    return AIY_OK;
}
void ws_dispatch_commit(aiy_ws* ws) {
    if (!ws->timing) return;
    if (!g_dispatch_ev.start) ws->ev_used++;  // the launch consumed (recorded) them
    g_dispatch_ev = DispatchEvents{};
}
int ws_timing_drain(aiy_ws* ws) {
    for (int q = 0; q < ws->ev_used; ++q) {
        AIY_HIP(hipEventSynchronize(ws->ev_stop[q]));
        float ms = 0.f;
        AIY_HIP(hipEventElapsedTime(&ms, ws->ev_start[q], ws->ev_stop[q]));
        ws->tot_ms += ms;
        ws->launches++;
    }
    ws->ev_used = 0;
    return AIY_OK;
}

// ---------------------------------------------------------------------------- Bellman sweep
bool tree_perm_eligible(const BellArgs& A);
int ws_tree_perm(aiy_ws* ws, const BellArgs& A, hipStream_t st);
// validation, the kernel arguments of one sweep, and the cached feasible prefixes
static int bell_args(aiy_ws* ws, const BellCall& c, BellArgs& A, hipStream_t st) {
    if (!ws) return fail(AIY_BAD_ARG, "NULL workspace");
    if (!c.v_old || !c.a || !c.s || !c.P || !c.v_new || !c.idx)
        return fail(AIY_BAD_ARG, "NULL device pointer");
    if (c.labor && (!c.L || c.Nl < 1 || c.Nl > ws->Nl))
        return fail(AIY_BAD_ARG, "labour sweep needs labor_choice and 1 <= Nl <= workspace Nl");
    if (!(c.beta == c.beta) || !(c.r == c.r) || !(c.w == c.w) || !(c.sigma == c.sigma))
        return fail(AIY_NON_FINITE, "non-finite scalar argument");
    A = BellArgs{};
    A.N = (int)ws->N;
    A.Na = (int)ws->Na;
    A.Nl = c.labor ? (int)c.Nl : 1;
    A.labor = c.labor;
    A.keep_incoming = c.keep_incoming;
    A.np = is_int_ge(c.sigma, 2.0) && c.sigma <= 9.0 ? (int)c.sigma - 1 : 0;
    if (c.mode == 1 && A.np == 0)
        return fail(AIY_BAD_ARG, "screened sweep (mode 1) needs integer sigma in [2, 9]");
    A.coarse = ws->coarse;
    A.CK = ws->CK;
    // default geometry by size (measured at Na = 400: 2 cooperating waves per tile 10 % faster;
    // at Na = 20,000 one wave per tile, XCD-aware tile order: 44.3 vs 45.9 us).  Labour at
    // Na <= 4096: 4 waves per tile with the first superblock's passing 8-blocks dealt
    // round-robin (bit 12) — Na = 400 sweep 58.1 -> 41.8 us, 1,000: 61.8 -> 54.8, 2,000:
    // 81.5 -> 70.3 (profiles/r02c_s6_*); A1 is neutral to it (16.4 us either way)
    // (Na > 4096: bit 13, tiles in descending j, is faster in a solve's early sweeps — sweep 25:
    // 34.9 vs 35.8 us — and slower once the policy has settled — sweep 100: 33.6 vs 32.8 us,
    // whole solve to tol 9.37 vs 8.99 ms — so the order stays row-major, XCD-contiguous (16)).
    // Round 4, A1 at Na > 4096: bit 11 (each XCD's cheapest 2 x 128 tiles dispatched last, the
    // rest row-major) over 16 alone, three alternating runs on one box: step 39.3 -> 36.3 us,
    // solve to tol 8.74 -> 8.63 ms; heaviest-first (bit 6) 37.6 us / 8.75 ms; narrower tiles
    // (bit 13) slower, 40.6 / 39.3 us (profiles/r04_g7_order_ab.txt).  Two one-wave tiles per
    // workgroup (bits 16-17 = 1) on top: 36.5 -> 36.0 us, solve 8.68 -> 8.59 ms; four: 36.3 us,
    // eight: 47 us (profiles/r04_g9_pack_ab.txt).  Bit 21 (the start's drift extrapolated from
    // the last two shifts): A1 36.1 -> 35.6 us, labour 0.285 -> 0.276 ms; neutral at Na = 400
    // (profiles/r04_g27_*, r04_g28_*).  Bit 23 (the hint's window reduced to the hint when the
    // extrapolated window is used) on top for A1: 36.2 -> 35.75 us (profiles/r04_g33_*); bit 24
    // (no hint evaluation then at all): kernel 30.9 -> 30.6 us, step 35.7 -> 35.6 (r04_g36_*)
    const int var = ws->variant >= 0 ? ws->variant
                    : ws->Na <= 4096 ? (c.labor ? 4 | 4096 : 2)
                    : (c.labor ? 16 | 1 << 21
                               : 16 | 2048 | 1 << 16 | 1 << 21 | 1 << 23 | 1 << 24);
    A.variant = var;
    A.ev_mfma = bell_ev_mfma(A.N, ws->variant);
    // (variant bit 13) one-wave tiles of tw < 64 states, tw = ceil(N·Na / (3 waves × 1,024
    // SIMDs)): every SIMD holds three tiles instead of two or three (the 3-wave SIMDs end the
    // launch, tools/tree_trace.py); lanes tw..63 idle.  Work split only.
    A.tw = 0;
    if ((var & 8192) && !c.labor && (var & (1 | 2 | 4 | 8)) == 0) {
        const int64_t tw = (ws->N * ws->Na + 3 * 1024 - 1) / (3 * 1024);
        A.tw = (int)std::max<int64_t>(16, std::min<int64_t>(64, tw));
        if (A.tw == 64) A.tw = 0;
    }
    A.r = c.r;
    A.w = c.w;
    A.beta = c.beta;
    A.sigma = c.sigma;
    A.v_old = c.v_old;
    A.a = c.a;
    A.s = c.s;
    A.P = c.P;
    A.L = c.labor ? c.L : nullptr;
    A.hint = c.hint;
    AIY_TRY(ws_ensure_bell(ws, bell_partial_slots(A)));
    A.dis = c.labor ? ws->dis : nullptr;
    A.EV = ws->EV;
    A.T = ws->T;
    A.tree = (var & 8) == 0;
    A.T32 = (A.tree || (var & 4)) ? nullptr : ws->T32;
    A.Dm = A.tree ? nullptr : ws->Dm;
    A.Dm8 = A.tree ? ws->Dm8 : nullptr;
    A.Dt = A.tree ? ws->Dt : nullptr;
    A.Dm512 = A.tree ? ws->Dm512 : nullptr;
    A.nb = (int)((ws->Na + 63) / 64);
    A.nb8 = (int)((ws->Na + 7) / 8);
    A.nb512 = (int)((ws->Na + 511) / 512);
    A.best0 = ws->best0;
    A.idx0 = ws->idx0;
    A.mom = ws->mom;
    A.partial = ws->partial;
    A.touched = ws->touched;
    A.hitcount = ws->count_hits ? ws->hitcount : nullptr;
    A.trace = nullptr;
    if (ws->tracing) {
        const int64_t cap = (int64_t)ws->N * ((ws->Na + 15) / 16);  // quad tiles: 16 states
        if (ws->trace_cap < cap) {
            dfree(ws->trace);
            AIY_TRY(dalloc(&ws->trace, 16 * (size_t)cap));
            AIY_HIP(hipMemset(ws->trace, 0, 16 * (size_t)cap * sizeof(long long)));
            ws->trace_cap = cap;
        }
        A.trace = ws->trace;
    }
    A.v_new = c.v_new;
    A.idx = c.idx;
    A.pk = c.pk;
    A.pl = c.pl;
    A.pc = c.pc;
    A.diff = ws->diff;
    A.fold = (unsigned long long*)c.prev_diff_out;
    // disutility per level: cached while (L, Nl, psi, eta) are unchanged (a launch per sweep
    // otherwise — a dependent launch in the small-grid sweep's one-launch chain)
    if (c.labor && !(ws->dis_ok && ws->dis_L == c.L && ws->dis_Nl == c.Nl &&
                     ws->dis_psi == c.psi && ws->dis_eta == c.eta)) {
        AIY_TRY(launch_disutility(c.L, (int)c.Nl, c.psi, c.eta, ws->dis, st));
        ws->dis_ok = true;
        ws->dis_L = c.L; ws->dis_Nl = c.Nl; ws->dis_psi = c.psi; ws->dis_eta = c.eta;
    }
    // feasible prefixes: cached while (r, w, a, s, L) are unchanged (aiy_ws_invalidate resets)
    size_t kf_need = (size_t)A.Nl * A.N * A.Na;
    if (ws->kf && ws->kf_cap < kf_need) {
        (void)hipFree(ws->kf);
        ws->kf = nullptr;
        ws->kf_ok = false;
    }
    if (!ws->kf) {
        AIY_HIP(hipMalloc((void**)&ws->kf, kf_need * sizeof(int)));
        ws->kf_cap = kf_need;
    }
    A.kf = ws->kf;
    bool fresh = ws->kf_ok && ws->kf_r == c.r && ws->kf_w == c.w && ws->kf_a == c.a &&
                 ws->kf_s == c.s && ws->kf_L == A.L && ws->kf_Nl == A.Nl && ws->kf_lab == A.labor;
    if (!fresh) {
        AIY_TRY(launch_bell_kf(A, st));
        ws->kf_ok = true;
        ws->kf_r = c.r; ws->kf_w = c.w; ws->kf_a = c.a; ws->kf_s = c.s; ws->kf_L = A.L;
        ws->kf_Nl = A.Nl; ws->kf_lab = A.labor;
        ws->perm_ok = false;
    }
    A.perm = nullptr;
    A.perm_slots = 0;
    if (tree_perm_eligible(A)) {
        const long long key = (long long)A.tw * (1ll << 31) +
                              (A.variant & (64 | 2048 | (3 << 16) | (15 << 26)));
        if (!ws->perm_ok || ws->perm_key != key) {
            AIY_TRY(ws_tree_perm(ws, A, st));
            ws->perm_key = key;
        }
        A.perm = ws->tree_perm;
        A.perm_slots = ws->perm_slots;
    }
    return AIY_OK;
}

// Dispatch order of the one-wave-per-tile A1 tree launch (variant bit 6).  A launch of N·ntile
// one-wave items on 1,024 SIMDs puts three waves on some SIMDs — the last-dispatched items of
// each XCD — and those items end the launch (tools/tree_trace.py: every last-to-finish item sits
// on a 3-wave SIMD).  The order keeps each XCD's item range (xcd_remap: the same L2 sets) and
// deals it heaviest first, by the feasible prefix of the tile's last state (the bound tree's
// superblock count), so the third waves are the cheapest tiles.  Work order only.
bool tree_perm_eligible(const BellArgs& A) {
    return (A.variant & (64 | 2048)) && A.tree && A.C <= 1 && A.np >= 1 && A.np <= 8 &&
           (A.variant & (1 | 2 | 4 | 8)) == 0;
}
constexpr int kSimdsPerXcd = 128;  // MI355X: 32 CUs x 4 SIMDs per XCD
static int ws_tree_perm_hybrid(aiy_ws* ws, const BellArgs& A, const std::vector<int>& kl,
                               int ntile, hipStream_t st);
int ws_tree_perm(aiy_ws* ws, const BellArgs& A, hipStream_t st) {
    const int N = A.N, Na = A.Na, TW = bell_tile_width(A, 1), ntile = (Na + TW - 1) / TW;
    const int G = N * ntile;
    // PK one-wave tiles per workgroup (bell_tree_pack); workgroup b runs on XCD b mod 8, its
    // waves take slots b·PK .. b·PK + PK - 1; the last workgroup's unused slots hold -1
    const int PK = bell_tree_pack(A), nwg = (G + PK - 1) / PK, slots = nwg * PK;
    // only each tile's last state's prefixes cross to the host (not all of kf)
    const int rows = A.Nl * N;
    if (ws->kf_last_cap < rows * ntile) {
        if (ws->kf_last) (void)hipFree(ws->kf_last);
        ws->kf_last = nullptr;
        ws->kf_last_cap = 0;
        AIY_HIP(hipMalloc((void**)&ws->kf_last, (size_t)rows * ntile * sizeof(int)));
        ws->kf_last_cap = rows * ntile;
    }
    std::vector<int> kl((size_t)rows * ntile);  // [labour level][row][tile]
    AIY_TRY(launch_kf_tile_last(A.kf, rows, Na, TW, ntile, ws->kf_last, st));
    AIY_HIP(hipMemcpyAsync(kl.data(), ws->kf_last, kl.size() * sizeof(int),
                           hipMemcpyDeviceToHost, st));
    AIY_HIP(hipStreamSynchronize(st));
    if (bell_tree_hybrid(A)) return ws_tree_perm_hybrid(ws, A, kl, ntile, st);
    std::vector<int> perm(slots, -1);
    int start = 0;
    for (int x = 0; x < 8; ++x) {
        int size = (nwg / 8 + (x < nwg % 8 ? 1 : 0)) * PK;
        if (x == (nwg - 1) % 8) size -= slots - G;
        std::vector<int> items(size);
        for (int u = 0; u < size; ++u) items[u] = start + u;
        auto cost = [&](int it) {  // the feasible prefixes of the tile's last state
            const int i = it / ntile, t = it % ntile;
            long long c = 0;
            for (int l = 0; l < A.Nl; ++l) c += kl[((size_t)l * N + i) * ntile + t];
            return c;
        };
        if (A.variant & 64) {  // the whole range heaviest first
            std::stable_sort(items.begin(), items.end(),
                             [&](int a, int b) { return cost(a) > cost(b); });
        } else {  // (bit 11) row-major, but the range's cheapest tiles dispatched last
            const int tail = std::max(0, std::min(size, size - 2 * kSimdsPerXcd));
            std::vector<int> by(items);
            std::stable_sort(by.begin(), by.end(), [&](int a, int b) { return cost(a) < cost(b); });
            std::vector<char> last(G, 0);
            for (int u = 0; u < tail; ++u) last[by[u]] = 1;
            std::vector<int> out;
            for (int it : items)
                if (!last[it]) out.push_back(it);
            for (int u = tail - 1; u >= 0; --u) out.push_back(by[u]);
            items.swap(out);
        }
        for (int u = 0; u < size; ++u)  // the XCD's (u / PK)-th workgroup b = 8(u / PK) + x
            perm[(size_t)(8 * (u / PK) + x) * PK + u % PK] = items[u];
        start += size;
    }
    if (!ws->tree_perm || ws->perm_cap < slots) {
        if (ws->tree_perm) (void)hipFree(ws->tree_perm);
        ws->tree_perm = nullptr;
        AIY_HIP(hipMalloc((void**)&ws->tree_perm, (size_t)slots * sizeof(int)));
        ws->perm_cap = slots;
    }
    AIY_HIP(hipMemcpyAsync(ws->tree_perm, perm.data(), (size_t)slots * sizeof(int),
                           hipMemcpyHostToDevice, st));
    AIY_HIP(hipStreamSynchronize(st));
    ws->perm_ok = true;
    ws->perm_slots = slots;
    return AIY_OK;
}

// The hybrid launch's order (variant bit 26): each XCD keeps its contiguous row-major range as
// above; its H heaviest tiles (bits 27-29) become cooperative workgroups (slots {item, -2}),
// dealt first, heaviest first; the rest are packed two per workgroup in row-major order with
// the range's cheapest tiles last (the third waves on a SIMD).  Workgroup b runs on XCD b mod 8.
static int ws_tree_perm_hybrid(aiy_ws* ws, const BellArgs& A, const std::vector<int>& kl,
                               int ntile, hipStream_t st) {
    const int N = A.N, G = N * ntile;
    auto cost = [&](int it) {
        const int i = it / ntile, t = it % ntile;
        long long c = 0;
        for (int l = 0; l < A.Nl; ++l) c += kl[((size_t)l * N + i) * ntile + t];
        return c;
    };
    // split the items into 8 contiguous ranges, then each range into workgroups
    std::vector<std::vector<int>> wg[8];  // per XCD: its workgroups' slot pairs, in order
    int start = 0;
    for (int x = 0; x < 8; ++x) {
        const int size = G / 8 + (x < G % 8 ? 1 : 0);
        std::vector<int> items(size);
        for (int u = 0; u < size; ++u) items[u] = start + u;
        start += size;
        std::vector<int> by(items);
        std::stable_sort(by.begin(), by.end(), [&](int a, int b) { return cost(a) > cost(b); });
        const int H = std::min(size, bell_tree_coop_per_xcd(A));
        std::vector<char> coop(G, 0);
        for (int u = 0; u < H; ++u) {
            coop[by[u]] = 1;
            wg[x].push_back({by[u], -2});
        }
        std::vector<int> rest;
        for (int it : items)
            if (!coop[it]) rest.push_back(it);
        // the cheapest (size - H) - 2·128 one-wave tiles last, cheapest at the very end
        const int R = (int)rest.size();
        const int tail = std::max(0, R - 2 * kSimdsPerXcd);
        std::vector<int> rb(rest);
        std::stable_sort(rb.begin(), rb.end(), [&](int a, int b) { return cost(a) < cost(b); });
        std::vector<char> last(G, 0);
        for (int u = 0; u < tail; ++u) last[rb[u]] = 1;
        std::vector<int> out;
        for (int it : rest)
            if (!last[it]) out.push_back(it);
        for (int u = tail - 1; u >= 0; --u) out.push_back(rb[u]);
        for (size_t u = 0; u < out.size(); u += 2)
            wg[x].push_back({out[u], u + 1 < out.size() ? out[u + 1] : -1});
    }
    // interleave: workgroup b = 8q + x is XCD x's q-th; XCDs with fewer workgroups get empty
    // ({-1, -1}) ones so that b mod 8 still names the XCD
    size_t nq = 0;
    for (int x = 0; x < 8; ++x) nq = std::max(nq, wg[x].size());
    const int slots = (int)(8 * nq * 2);
    std::vector<int> perm(slots, -1);
    for (size_t q = 0; q < nq; ++q)
        for (int x = 0; x < 8; ++x)
            if (q < wg[x].size()) {
                perm[(8 * q + x) * 2] = wg[x][q][0];
                perm[(8 * q + x) * 2 + 1] = wg[x][q][1];
            }
    if (!ws->tree_perm || ws->perm_cap < slots) {
        if (ws->tree_perm) (void)hipFree(ws->tree_perm);
        ws->tree_perm = nullptr;
        AIY_HIP(hipMalloc((void**)&ws->tree_perm, (size_t)slots * sizeof(int)));
        ws->perm_cap = slots;
    }
    AIY_HIP(hipMemcpyAsync(ws->tree_perm, perm.data(), (size_t)slots * sizeof(int),
                           hipMemcpyHostToDevice, st));
    AIY_HIP(hipStreamSynchronize(st));
    ws->perm_ok = true;
    ws->perm_slots = slots;
    return AIY_OK;
}

// The small-grid one-launch sweep (bellman_wide_kernels.hip) and its geometry.  Default: every
// screened sweep at Na <= 1,536 (A1) / 2,048 (labour) unless a tree geometry was asked for
// (variant >= 0 without bit 25); aiy_ws_set_wide overrides the bound and the geometry.
// Measured (tools/wide_tune.py, profiles/r05_wide_tune.jsonl; sweeps 11-60 from v = 0, per
// sweep, tree = table + tree launch): A1 Na = 400 7.7 vs 13.8 us, 1,000 10.2 vs 16.4, 2,048
// 16.7 vs 16.5 (a tie: the tree from there); labour Na = 400 17 vs 32 us, 1,000 25 vs 52, 2,000
// 56 vs 60.  One workgroup per tile (splits = 1): the cross-workgroup hand-off (sc1 partials,
// an arrival counter) costs more than the extra workgroups save at every size measured.
static bool wide_pick(const aiy_ws* ws, const BellArgs& A, int* S, int* NW, int* SB) {
    if (A.np < 1 || A.np > 8 || A.C > 1 || A.ev_mfma || A.Nl > kWideMaxNl) return false;
    const int vmax = ws->wide_max >= 0 ? ws->wide_max : (A.labor ? 2048 : 1536);
    if (A.Na > vmax) return false;
    if (ws->variant >= 0 && !(ws->variant & (1 << 25))) return false;
    // states per wave: labour 16 up to Na = 512, then 32 (profiles/r05_wide_ab.txt, r05_g52:
    // Na = 1,000 30.8 -> 21.8 us, 2,000 69.9 -> 56.4); A1 32 up to 1,024, then 64
    const int sb = ws->wide_SB > 0 ? ws->wide_SB
                                   : (A.labor ? (A.Na <= 512 ? 16 : 32) : (A.Na <= 1024 ? 32 : 64));
    const int nw = ws->wide_NW > 0 ? ws->wide_NW : 8;
    const int s = ws->wide_S > 0 ? ws->wide_S : 1;
    if (bell_wide_lds(A.Na, s, nw) > kWideMaxLds) return false;
    *S = s;
    *NW = nw;
    *SB = sb;
    return true;
}

static int bell_sweep_wide(aiy_ws* ws, BellArgs& A, int S, int NW, int SB, hipStream_t st) {
    const int ntile = (int)((ws->Na + SB - 1) / SB);
    const size_t items = (size_t)ws->N * ntile;
    if (!ws->wdiff) {
        AIY_TRY(dalloc(&ws->wdiff, 4 * (size_t)kDiffSlots));
        AIY_HIP(hipMemsetAsync(ws->wdiff, 0, 4 * kDiffSlots * sizeof(unsigned long long), st));
        ws->wcur = 0;
    }
    if (ws->wcnt_cap < items) {
        dfree(ws->wcnt);
        AIY_TRY(dalloc(&ws->wcnt, items));
        AIY_HIP(hipMemsetAsync(ws->wcnt, 0, items * sizeof(unsigned), st));
        ws->wcnt_cap = items;
    }
    const size_t pneed = items * (size_t)S * 64 * 2;
    if (S > 1 && ws->wpart_cap < pneed) {
        dfree(ws->wpart);
        AIY_TRY(dalloc(&ws->wpart, pneed));
        ws->wpart_cap = pneed;
    }
    unsigned long long* cur = ws->wdiff + (size_t)ws->wcur * 2 * kDiffSlots;
    unsigned long long* nxt = ws->wdiff + (size_t)(ws->wcur ^ 1) * 2 * kDiffSlots;
    if (A.fold && !ws->last_wide) {  // the previous sweep's slots are the table path's
        AIY_TRY(launch_reduce_slots(ws->diff, A.fold, st));
        A.fold = nullptr;
    }
    A.diff = nxt;  // zero (the set not current); block 0 folds and clears `cur`
    A.trace = nullptr;
    if (ws->tracing) {  // one 64-word record per block (instrumentation)
        const int64_t blocks = ((int64_t)items + 7) / 8 * 8 * S * 4;  // (in 16-word units)
        if (ws->trace_cap < blocks) {
            dfree(ws->trace);
            AIY_TRY(dalloc(&ws->trace, 16 * (size_t)blocks));
            ws->trace_cap = blocks;
        }
        AIY_HIP(hipMemsetAsync(ws->trace, 0, 16 * (size_t)ws->trace_cap * sizeof(long long), st));
        A.trace = ws->trace;
    }
    const char* fl = getenv("AIY_WIDE_FLAGS");  // (A/B tooling: tools/wide_tune.py)
    AIY_TRY(ws_dispatch_arm(ws));
    const int rc = launch_bell_wide(A, S, NW, SB, cur, ws->wcnt, ws->wpart, fl ? atoi(fl) : kWideDefaultFlags,
                                    ws->cu_exclusive ? kExclusiveLds : 0, st);
    ws_dispatch_commit(ws);
    AIY_TRY(rc);
    ws->wcur ^= 1;
    ws->vdiff = nxt;
    ws->last_wide = true;
    return AIY_OK;
}

int bell_sweep_dev(aiy_ws* ws, const BellCall& c, hipStream_t st) {
    BellArgs A;
    AIY_TRY(bell_args(ws, c, A, st));
    // mode 2 / variant bit 10: the exhaustive scan (one launch after the table, outputs written
    // by the scan itself); otherwise the bound tree (or the chunked screen, variant bit 3)
    const bool exhaustive = c.mode == 2 || A.np == 0 || (A.variant & 1024);
    const bool screened = !exhaustive;
    int wS = 0, wNW = 0, wSB = 0;
    if (screened && wide_pick(ws, A, &wS, &wNW, &wSB)) {  // small grids: one launch per sweep
        AIY_TRY(bell_sweep_wide(ws, A, wS, wNW, wSB, st));
        if (c.diff_out) AIY_TRY(launch_reduce_slots(ws->vdiff, c.diff_out, st));
        return AIY_OK;
    }
    if (ws->last_wide && A.fold) {  // the previous sweep's slots are the wide path's
        AIY_TRY(launch_reduce_slots(ws->vdiff, A.fold, st));
        A.fold = nullptr;
    }
    ws->last_wide = false;
    ws->vdiff = ws->diff;
    AIY_TRY(launch_bell_table(A, st));  // also clears the diff slots
    if (!screened) A.coarse = 0, A.hint = nullptr;
    if (screened && A.tree) {
        // tree screen: the hint (or, cold, the init kernel's candidate) sets the first bar;
        // the tree kernel writes the outputs itself
        if (!A.hint) AIY_TRY(launch_bell_init(A, st));
        AIY_TRY(ws_dispatch_arm(ws));  // events recorded by the dispatch itself
        const int rc = launch_bell_tree(A, st);
        ws_dispatch_commit(ws);
        AIY_TRY(rc);
    } else if (screened) {
        AIY_TRY(launch_bell_init(A, st));
        AIY_TRY(ws_timing_begin(ws, st));
        AIY_TRY(launch_bell_screen(A, st));
        AIY_TRY(ws_timing_end(ws, st));
        AIY_TRY(launch_bell_merge(A, 1, st));
    } else {
        AIY_TRY(ws_timing_begin(ws, st));
        AIY_TRY(launch_bell_plain(A, st));
        AIY_TRY(ws_timing_end(ws, st));
    }
    if (c.diff_out) AIY_TRY(launch_reduce_slots(ws->diff, c.diff_out, st));
    return AIY_OK;
}

// read {max|Δ| bits, any} from the workspace diff word (synchronises the stream)
int ws_read_diff(aiy_ws* ws, hipStream_t st, double* d) {
    const unsigned long long* sl = ws->vdiff ? ws->vdiff : ws->diff;  // the last sweep's slots
    AIY_HIP(hipMemcpyAsync(ws->hdiff, sl, 2 * kDiffSlots * sizeof(unsigned long long),
                           hipMemcpyDeviceToHost, st));
    AIY_HIP(hipStreamSynchronize(st));
    *d = fold_slots_host(ws->hdiff);
    return AIY_OK;
}

// A2 with speculative batches.  The one-sweep-at-a-time loop pays a stream synchronisation per
// sweep to read max|Δv| (at the script's Na = 400 that round trip costs more than the sweep).
// Here sweeps are enqueued m at a time: sweep g reads ring slot (g−1) mod R and writes slot
// g mod R (R = 2·spec_max + 1 value buffers), its policies go to set g mod 2·spec_max, its folded
// diff to its own slot, and one D2H read per batch finds the first sweep below tol.  Sweeps
// are deterministic and each depends only on its predecessor, so sweeps 1..g* are exactly the
// ones the plain loop runs; later sweeps of the batch are discarded and the ring still holds
// v_new(g*), v_old = v(g*−1) and the policies of g*.  m follows the observed geometric decay
// of the diff (sweeps still needed to reach tol), capped at spec_max.
static int bell_solve_spec(aiy_ws* ws, BellCall c, double* v_a, double* v_b, double tol,
                           int64_t max_iter, int64_t* iters, int* out_new, hipStream_t st) {
    // rings sized for two batches in flight: v 2M + 1 (the stopping sweep's v_new and v_old
    // survive the next batch), idx / policies 2M, diff pairs 2M (indexed by sweep)
    const int M = ws->spec_max, R = 2 * M + 1, Rp = 2 * M, D = 2 * M;
    const size_t n = (size_t)ws->N * ws->Na;
    if (ws->spec_n != n || ws->spec_m != M) {
        ws->free_spec();
        AIY_TRY(dalloc(&ws->spec_v, (size_t)R * n));
        AIY_TRY(dalloc(&ws->spec_idx, (size_t)Rp * n));
        AIY_TRY(dalloc(&ws->spec_pol, (size_t)Rp * 3 * n));
        AIY_TRY(dalloc(&ws->spec_diff, 2 * (size_t)D));
        AIY_HIP(hipHostMalloc((void**)&ws->spec_hdiff, 2 * 2 * (size_t)D * sizeof(unsigned long long)));
        for (int b = 0; b < 2; ++b)
            AIY_HIP(hipEventCreateWithFlags(&ws->spec_ev[b], hipEventDisableTiming));
        ws->spec_n = n;
        ws->spec_m = M;
    }
    auto vslot = [&](int64_t g) { return ws->spec_v + (size_t)(g % R) * n; };
    auto islot = [&](int64_t g) { return ws->spec_idx + (size_t)(g % Rp) * n; };
    auto pslot = [&](int64_t g, int q) { return ws->spec_pol + ((size_t)(g % Rp) * 3 + q) * n; };
    auto dslot = [&](int64_t g) { return ws->spec_diff + 2 * (size_t)(g % D); };
    const size_t vb = n * sizeof(double);
    // slot 0 = v_old of sweep 1; slot 1 = the incoming v_new buffer (the labour sweep's
    // keep-incoming rule reads it on sweep 1)
    AIY_HIP(hipMemcpyAsync(vslot(0), v_a, vb, hipMemcpyDeviceToDevice, st));
    AIY_HIP(hipMemcpyAsync(vslot(1), v_b, vb, hipMemcpyDeviceToDevice, st));
    const int* first_hint = c.hint;
    double* const upk = c.pk;
    double* const upc = c.pc;
    double* const upl = c.pl;
    int* const uidx = c.idx;
    if (c.labor) {
        // Labor_VFI.m:85: a state with no feasible choice keeps its incoming policies (the
        // kernels do not write them).  The plain loop reuses the caller's buffers, so those
        // entries stay the caller's; every ring slot starts as a copy of them to match
        // (feasibility depends on (r, w, grids) only, so it is fixed within a solve).
        for (int q = 0; q < Rp; ++q) {
            AIY_HIP(hipMemcpyAsync(ws->spec_idx + (size_t)q * n, uidx, n * sizeof(int),
                                   hipMemcpyDeviceToDevice, st));
            double* const src[3] = {upk, upc, upl};
            for (int p = 0; p < 3; ++p)
                if (src[p])
                    AIY_HIP(hipMemcpyAsync(ws->spec_pol + ((size_t)q * 3 + p) * n, src[p], vb,
                                           hipMemcpyDeviceToDevice, st));
        }
    }
    // Batches of m sweeps, each ending with a D2H copy of the diff pairs and an event; two in
    // flight: the host reads batch k while batch k+1 runs, so the device never waits for a read
    struct Batch {
        int64_t s0, m;  // sweeps s0 + 1 .. s0 + m
        int hb;         // host half holding its diff pairs
    };
    Batch q[2];
    int nq = 0, hb_next = 0;
    int64_t enq = 0, stop = 0;
    double d_prev = NAN, d_last = NAN;
    auto enqueue = [&]() -> int {
        int64_t m = M;
        if (d_last == d_last && d_prev == d_prev && d_last < d_prev && d_last > 0) {
            const double need = std::ceil(std::log(tol / d_last) / std::log(d_last / d_prev));
            int64_t ahead = 0;  // sweeps in flight, not yet read
            for (int b = 0; b < nq; ++b) ahead += q[b].m;
            if (need >= 1 && need - (double)ahead < (double)m)
                m = (int64_t)std::max(1.0, need - (double)ahead);
        }
        m = std::min<int64_t>(std::max<int64_t>(m, 1), max_iter - enq);
        for (int64_t t = 0; t < m; ++t) {
            const int64_t g = enq + 1 + t;
            c.hint = (g == 1) ? first_hint : islot(g - 1);
            c.keep_incoming = (g == 1);
            c.v_old = vslot(g - 1);
            c.v_new = vslot(g);
            c.idx = islot(g);
            c.pk = upk ? pslot(g, 0) : nullptr;
            c.pc = upc ? pslot(g, 1) : nullptr;
            c.pl = upl ? pslot(g, 2) : nullptr;
            // sweep g's {max bits, any} lands in pair g: folded by sweep g+1's table kernel,
            // or by a reduce launch after the batch's last sweep
            c.prev_diff_out = t ? dslot(g - 1) : nullptr;
            c.diff_out = (t == m - 1) ? reinterpret_cast<double*>(dslot(g)) : nullptr;
            AIY_TRY(bell_sweep_dev(ws, c, st));
        }
        unsigned long long* h = ws->spec_hdiff + (size_t)hb_next * 2 * D;
        AIY_HIP(hipMemcpyAsync(h, ws->spec_diff, 2 * (size_t)D * sizeof(unsigned long long),
                               hipMemcpyDeviceToHost, st));
        AIY_HIP(hipEventRecord(ws->spec_ev[hb_next], st));
        q[nq++] = Batch{enq, m, hb_next};
        hb_next ^= 1;
        enq += m;
        return AIY_OK;
    };
    if (max_iter > 0) AIY_TRY(enqueue());
    while (nq > 0) {
        if (nq < 2 && enq < max_iter) AIY_TRY(enqueue());
        const Batch b = q[0];
        AIY_TRY(wait_event(ws->spec_ev[b.hb]));
        const unsigned long long* hs = ws->spec_hdiff + (size_t)b.hb * 2 * D;
        for (int64_t t = 0; t < b.m; ++t) {
            const unsigned long long* h = hs + 2 * ((b.s0 + 1 + t) % D);
            double d = NAN;  // {max|Δ| bits, any non-NaN} (reduce_slots_kernel)
            if (h[1]) std::memcpy(&d, &h[0], sizeof d);
            d_prev = d_last;
            d_last = d;
            if (d < tol) {  // Aiyagari_VFI.m:85-86
                stop = b.s0 + 1 + t;
                break;
            }
        }
        q[0] = q[1];
        --nq;
        if (stop) break;
    }
    const int64_t g = stop ? stop : enq;
    // the plain loop leaves v_new in v_b after odd sweep counts (ping-pong from v_a)
    const int nw = (g & 1) ? 1 : 0;
    double* vnew = nw ? v_b : v_a;
    double* vold = nw ? v_a : v_b;
    AIY_HIP(hipMemcpyAsync(vnew, vslot(g), vb, hipMemcpyDeviceToDevice, st));
    // exhausted: v_old = v_new after the last sweep (:88); else the previous iterate
    AIY_HIP(hipMemcpyAsync(vold, stop ? vslot(g - 1) : vslot(g), vb, hipMemcpyDeviceToDevice, st));
    AIY_HIP(hipMemcpyAsync(uidx, islot(g), n * sizeof(int), hipMemcpyDeviceToDevice, st));
    if (upk) AIY_HIP(hipMemcpyAsync(upk, pslot(g, 0), vb, hipMemcpyDeviceToDevice, st));
    if (upc) AIY_HIP(hipMemcpyAsync(upc, pslot(g, 1), vb, hipMemcpyDeviceToDevice, st));
    if (upl) AIY_HIP(hipMemcpyAsync(upl, pslot(g, 2), vb, hipMemcpyDeviceToDevice, st));
    *iters = g;
    *out_new = nw;
    return AIY_OK;
}

int bell_solve_dev(aiy_ws* ws, BellCall c, double* v_a, double* v_b, double tol,
                   int64_t max_iter, int64_t* iters, int* out_new, hipStream_t st) {
    if (max_iter < 1) return fail(AIY_BAD_ARG, "max_iter must be >= 1");
    if (!c.idx) return fail(AIY_BAD_ARG, "NULL device pointer");
    if (ws && ws->spec_max > 1 && !c.diff_out) {
        // rings (two batches in flight, bell_solve_spec): 2M + 1 value buffers, 2M idx slots
        // and 2M x 3 policy slots, M = spec_max
        const size_t n = (size_t)ws->N * ws->Na, M2 = 2 * (size_t)ws->spec_max;
        const size_t bytes = ((M2 + 1) + 3 * M2) * n * sizeof(double) + M2 * n * sizeof(int);
        if (bytes <= ((size_t)8 << 30)) {
            int rc = bell_solve_spec(ws, c, v_a, v_b, tol, max_iter, iters, out_new, st);
            if (rc != AIY_NO_MEMORY) return rc;
            ws->free_spec();  // no room for the rings: one synchronisation per sweep instead
        }
    }
    double* cur = v_a;
    double* nxt = v_b;
    const int* first_hint = c.hint;
    int64_t it;
    for (it = 1; it <= max_iter; ++it) {
        c.hint = (it == 1) ? first_hint : c.idx;
        c.keep_incoming = (it == 1);
        c.v_old = cur;
        c.v_new = nxt;
        AIY_TRY(bell_sweep_dev(ws, c, st));
        double d;
        AIY_TRY(ws_read_diff(ws, st, &d));
        if (d < tol) break;  // Aiyagari_VFI.m:85-86 (v_old keeps the previous iterate)
        std::swap(cur, nxt); // :88
    }
    if (it > max_iter) {  // loop exhausted: v_old = v_new after the last sweep
        it = max_iter;
        AIY_HIP(hipMemcpyAsync(nxt, cur, sizeof(double) * ws->N * ws->Na,
                               hipMemcpyDeviceToDevice, st));
        std::swap(cur, nxt);
    }
    *iters = it;
    *out_new = (nxt == v_a) ? 0 : 1;
    return AIY_OK;
}

// Config 4 (BASELINE configs[3]): C candidate interest rates, each the A2 loop of
// Aiyagari_VFI.m:147-171 from its own v_old, solved together: every sweep is ONE table launch
// and ONE tree launch over all candidates still running (C·N·Na states), so the GPU sees C
// times the parallelism of one solve.  Each candidate stops at its own first sweep below tol
// (the table kernel applies :85 per candidate on the device and freezes it), so iteration
// counts, v_new, v_old and policies are exactly those of C separate solves.  The host reads the
// stop flags once per `spec_max` sweeps.  Buffers: sweep g reads buf[(g-1) & 1] and writes
// buf[g & 1] with buf[0] = v_a, so a candidate that stopped at g* holds v_new in buf[g* & 1].
int bell_solve_batch_dev(aiy_ws* ws, int64_t C, const double* r, const double* w, double* v_a,
                         double* v_b, const double* a, const double* s, const double* P,
                         double beta, double sigma, double tol, int64_t max_iter, int use_hint,
                         int* idx, double* pk, double* pc, int64_t* iters, int* which,
                         hipStream_t st) {
    if (!ws) return fail(AIY_BAD_ARG, "NULL workspace");
    if (C < 1 || C > (1 << 20)) return fail(AIY_BAD_SHAPE, "need 1 <= C <= 2^20 candidates");
    if (!r || !w || !v_a || !v_b || !a || !s || !P || !idx || !iters || !which)
        return fail(AIY_BAD_ARG, "NULL argument");
    if (max_iter < 1) return fail(AIY_BAD_ARG, "max_iter must be >= 1");
    for (int64_t c = 0; c < C; ++c)
        if (!(r[c] == r[c]) || !(w[c] == w[c])) return fail(AIY_NON_FINITE, "non-finite r or w");
    const size_t n = (size_t)ws->N * ws->Na;
    const int np = is_int_ge(sigma, 2.0) && sigma <= 9.0 ? (int)sigma - 1 : 0;
    if (np == 0 || C == 1) {
        // generic sigma (plain sweeps) or a single rate: one solve after another, same results
        for (int64_t c = 0; c < C; ++c) {
            BellCall bc{};
            bc.a = a; bc.s = s; bc.P = P; bc.r = r[c]; bc.w = w[c]; bc.beta = beta;
            bc.sigma = sigma; bc.idx = idx + c * n; bc.pk = pk ? pk + c * n : nullptr;
            bc.pc = pc ? pc + c * n : nullptr;
            bc.hint = use_hint ? idx + c * n : nullptr;
            AIY_TRY(bell_solve_dev(ws, bc, v_a + c * n, v_b + c * n, tol, max_iter, &iters[c],
                                   &which[c], st));
        }
        return AIY_OK;
    }
    if ((size_t)C * n > (size_t)INT32_MAX) return fail(AIY_BAD_SHAPE, "C*N*Na must fit int32");
    const int nb8 = (int)((ws->Na + 7) / 8), nb512 = (int)((ws->Na + 511) / 512);
    if (ws->bC != C) {
        ws->free_batch();
        AIY_TRY(dalloc(&ws->bEV, C * n));
        AIY_TRY(dalloc(&ws->bDt, C * n));
        AIY_TRY(dalloc(&ws->bDm8, (size_t)C * ws->N * nb8));
        AIY_TRY(dalloc(&ws->bDm512, (size_t)C * ws->N * nb512));
        AIY_TRY(dalloc(&ws->bbest0, C * n));
        AIY_TRY(dalloc(&ws->bidx0, C * n));
        AIY_TRY(dalloc(&ws->bmom, C * n));
        AIY_HIP(hipMemset(ws->bmom, 0, C * n * sizeof(int)));
        AIY_TRY(dalloc(&ws->bkf, C * n));
        AIY_TRY(dalloc(&ws->bstop, (size_t)C));
        AIY_TRY(dalloc(&ws->bslots, (size_t)C * 2 * 2 * kDiffSlots));
        AIY_TRY(dalloc(&ws->brw, 2 * (size_t)C));
        AIY_HIP(hipHostMalloc((void**)&ws->hstop, C * sizeof(int)));
        AIY_HIP(hipHostMalloc((void**)&ws->hslots, (size_t)C * 2 * kDiffSlots * sizeof(unsigned long long)));
        ws->bC = C;
    }
    AIY_TRY(ws_ensure_bell(ws, 1));  // diff/hitcount scratch and events (single-rate buffers)
    AIY_HIP(hipMemcpyAsync(ws->brw, r, C * sizeof(double), hipMemcpyHostToDevice, st));
    AIY_HIP(hipMemcpyAsync(ws->brw + C, w, C * sizeof(double), hipMemcpyHostToDevice, st));
    AIY_HIP(hipMemsetAsync(ws->bstop, 0, C * sizeof(int), st));
    BellArgs A{};
    A.N = (int)ws->N; A.Na = (int)ws->Na; A.Nl = 1; A.labor = false; A.np = np;
    A.coarse = ws->coarse; A.CK = ws->CK;
    A.variant = ws->variant >= 0 ? ws->variant : (ws->Na <= 4096 ? 0 : 16 | 1 << 21);
    A.variant &= ~(1 | 2 | 4 | 8);  // one state per lane, one wave per tile, tree screen
    A.ev_mfma = bell_ev_mfma(A.N, ws->variant);
    A.beta = beta; A.sigma = sigma; A.a = a; A.s = s; A.P = P;
    A.EV = ws->bEV; A.Dt = ws->bDt; A.Dm8 = ws->bDm8; A.Dm512 = ws->bDm512;
    A.nb = (int)((ws->Na + 63) / 64); A.nb8 = nb8; A.nb512 = nb512;
    A.tree = true; A.best0 = ws->bbest0; A.idx0 = ws->bidx0; A.kf = ws->bkf; A.mom = ws->bmom;
    A.hitcount = ws->count_hits ? ws->hitcount : nullptr;
    A.idx = idx; A.pk = pk; A.pc = pc; A.diff = ws->bslots;
    A.C = (int)C; A.rv = ws->brw; A.wv = ws->brw + C; A.stop = ws->bstop;
    AIY_TRY(launch_bell_kf(A, st));  // per-candidate feasible prefixes, once per solve
    ws->kf_ok = false;               // (the single-rate kf cache is not this table)
    double* buf[2] = {v_a, v_b};
    int64_t g = 0;
    bool all_stopped = false;
    const int64_t m = std::max(ws->spec_max, 1);
    while (!all_stopped && g < max_iter) {
        const int64_t gend = std::min(max_iter, g + m);
        for (++g; g <= gend; ++g) {
            A.v_old = buf[(g - 1) & 1];
            A.v_new = buf[g & 1];
            A.parity = (int)(g & 1);
            A.hint = (g == 1 && !use_hint) ? nullptr : idx;
            if (A.ev_mfma) AIY_TRY(launch_bell_ev_mfma(A, st));
            AIY_TRY(launch_bell_table_batch(A, ws->bslots, (int)g, tol, st));
            if (!A.hint) AIY_TRY(launch_bell_init(A, st));
            AIY_TRY(ws_timing_begin(ws, st));
            AIY_TRY(launch_bell_tree(A, st));
            AIY_TRY(ws_timing_end(ws, st));
        }
        --g;  // sweeps launched so far
        AIY_HIP(hipMemcpyAsync(ws->hstop, ws->bstop, C * sizeof(int), hipMemcpyDeviceToHost, st));
        AIY_HIP(hipStreamSynchronize(st));
        all_stopped = true;
        for (int64_t c = 0; c < C; ++c) all_stopped = all_stopped && ws->hstop[c] != 0;
    }
    // candidates still running after the last sweep G = max_iter: fold their sweep-G slots
    // (its :85 test), else the loop was exhausted and v_old = v_new (:88)
    const int64_t G = g;
    bool any_running = false;
    for (int64_t c = 0; c < C; ++c) any_running = any_running || ws->hstop[c] == 0;
    if (any_running) {
        for (int64_t c = 0; c < C; ++c)
            if (ws->hstop[c] == 0)
                AIY_HIP(hipMemcpyAsync(ws->hslots + c * 2 * kDiffSlots,
                                       ws->bslots + ((size_t)c * 2 + (G & 1)) * 2 * kDiffSlots,
                                       2 * kDiffSlots * sizeof(unsigned long long),
                                       hipMemcpyDeviceToHost, st));
        AIY_HIP(hipStreamSynchronize(st));
    }
    for (int64_t c = 0; c < C; ++c) {
        int64_t it = ws->hstop[c];
        if (it == 0) {
            const double d = fold_slots_host(ws->hslots + c * 2 * kDiffSlots);
            it = G;
            if (!(d < tol))  // exhausted: v_old = v_new after the last sweep
                AIY_HIP(hipMemcpyAsync(buf[(G - 1) & 1] + c * n, buf[G & 1] + c * n,
                                       n * sizeof(double), hipMemcpyDeviceToDevice, st));
        }
        iters[c] = it;
        which[c] = (int)(it & 1);
    }
    AIY_HIP(hipStreamSynchronize(st));
    return AIY_OK;
}

}  // namespace aiy

using namespace aiy;

// ============================================================================ C ABI
extern "C" {

const char* aiy_last_error(void) { return g_err.c_str(); }
int aiy_version(void) { return 100; }
int aiy_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int aiy_ws_create(int64_t N, int64_t Na, int64_t Nl, aiy_ws** out) {
    if (!out) return fail(AIY_BAD_ARG, "NULL out pointer");
    if (N < 1 || Na < 2 || N > (1 << 16) || Na > (1 << 28) || N * Na > (1ll << 31) - 1)
        return fail(AIY_BAD_SHAPE, "unsupported shape N=%lld Na=%lld", (long long)N,
                    (long long)Na);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1)
        return fail(AIY_NO_DEVICE, "no HIP device visible");
    aiy_ws* ws = new aiy_ws();
    ws->N = N;
    ws->Na = Na;
    ws->Nl = Nl < 1 ? 1 : Nl;
    (void)hipGetDevice(&ws->dev);
    ws->ev_start.resize(64);
    ws->ev_stop.resize(64);
    for (int q = 0; q < 64; ++q) {
        if (hipEventCreate(&ws->ev_start[q]) != hipSuccess ||
            hipEventCreate(&ws->ev_stop[q]) != hipSuccess) {
            aiy_ws_destroy(ws);
            return fail(AIY_HIP_ERROR, "hipEventCreate failed");
        }
    }
    *out = ws;
    return AIY_OK;
}

int aiy_ws_destroy(aiy_ws* ws) {
    if (!ws) return AIY_OK;
    ws->free_all();
    for (auto& e : ws->ev_start)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : ws->ev_stop)
        if (e) (void)hipEventDestroy(e);
    delete ws;
    return AIY_OK;
}

int aiy_ws_set_timing(aiy_ws* ws, int enable) {
    if (!ws) return fail(AIY_BAD_ARG, "NULL workspace");
    AIY_TRY(ws_timing_drain(ws));
    ws->timing = (enable & 1) != 0;
    ws->count_hits = (enable & 2) != 0;
    ws->tracing = (enable & 4) != 0;
    ws->tot_ms = 0;
    ws->launches = 0;
    if (ws->hitcount) AIY_HIP(hipMemset(ws->hitcount, 0, 4 * kDiffSlots * sizeof(unsigned long long)));
    if (ws->tracing && ws->trace)  // records of an earlier geometry must not linger
        AIY_HIP(hipMemset(ws->trace, 0, 16 * (size_t)ws->trace_cap * sizeof(long long)));
    return AIY_OK;
}

int aiy_ws_timing(aiy_ws* ws, double* total_ms, int64_t* launches, int64_t* hits) {
    if (!ws) return fail(AIY_BAD_ARG, "NULL workspace");
    AIY_TRY(ws_timing_drain(ws));
    if (total_ms) *total_ms = ws->tot_ms;
    if (launches) *launches = ws->launches;
    if (hits) {
        int64_t c[4];
        AIY_TRY(aiy_ws_counters(ws, c));
        *hits = c[0];
    }
    return AIY_OK;
}

int aiy_ws_counters(aiy_ws* ws, int64_t out[4]) {
    if (!ws || !out) return fail(AIY_BAD_ARG, "NULL workspace/out");
    std::vector<unsigned long long> h(4 * kDiffSlots, 0ull);
    if (ws->hitcount)
        AIY_HIP(hipMemcpy(h.data(), ws->hitcount, h.size() * sizeof(unsigned long long),
                          hipMemcpyDeviceToHost));
    for (int q = 0; q < 4; ++q) {
        unsigned long long t = 0;
        for (int sl = 0; sl < kDiffSlots; ++sl) t += h[4 * sl + q];
        out[q] = (int64_t)t;
    }
    return AIY_OK;
}

int aiy_ws_trace(aiy_ws* ws, int64_t* out, int64_t cap, int64_t* n) {
    if (!ws || !out || !n) return fail(AIY_BAD_ARG, "NULL argument");
    *n = 0;
    if (!ws->trace) return AIY_OK;
    int64_t m = std::min(cap, ws->trace_cap);
    AIY_HIP(hipMemcpy(out, ws->trace, 16 * (size_t)m * sizeof(int64_t), hipMemcpyDeviceToHost));
    *n = m;
    return AIY_OK;
}

int aiy_ws_invalidate(aiy_ws* ws) {
    if (!ws) return fail(AIY_BAD_ARG, "NULL workspace");
    ws->kf_ok = false;
    ws->dis_ok = false;
    return AIY_OK;
}

int aiy_ws_set_variant(aiy_ws* ws, int variant) {
    if (!ws) return fail(AIY_BAD_ARG, "NULL workspace");
    if (variant < -1 || variant >= (1 << 30)) return fail(AIY_BAD_ARG, "variant in [-1, 2^30)");
    ws->variant = variant;
    return AIY_OK;
}

int aiy_ws_set_wide(aiy_ws* ws, int max_na, int splits, int waves, int states) {
    if (!ws) return fail(AIY_BAD_ARG, "NULL workspace");
    if (max_na < -1 || splits < 0 || splits > kWideMaxSplits ||
        (waves != 0 && waves != 4 && waves != 8 && waves != 16) ||
        (states != 0 && states != 8 && states != 16 && states != 32 && states != 64))
        return fail(AIY_BAD_ARG, "max_na >= -1, splits in [0, %d], waves in {0, 4, 8, 16}, "
                    "states in {0, 8, 16, 32, 64}", kWideMaxSplits);
    ws->wide_max = max_na;
    ws->wide_S = splits;
    ws->wide_NW = waves;
    ws->wide_SB = states;
    return AIY_OK;
}

int aiy_ws_set_cu_exclusive(aiy_ws* ws, int on) {
    if (!ws) return fail(AIY_BAD_ARG, "NULL workspace");
    ws->cu_exclusive = on != 0;
    return AIY_OK;
}

int aiy_ws_set_speculation(aiy_ws* ws, int max_batch) {
    if (!ws) return fail(AIY_BAD_ARG, "NULL workspace");
    if (max_batch < 0 || max_batch > 256) return fail(AIY_BAD_ARG, "max_batch in [0, 256]");
    if (max_batch != ws->spec_max) ws->free_spec();
    ws->spec_max = max_batch;
    return AIY_OK;
}

int aiy_ws_set_search(aiy_ws* ws, int coarse_stride, int k_chunk) {
    if (!ws) return fail(AIY_BAD_ARG, "NULL workspace");
    if (coarse_stride < 0 || k_chunk < 64 || k_chunk % 64)
        return fail(AIY_BAD_ARG, "coarse_stride >= 0, k_chunk >= 64 and a multiple of 64");
    if (coarse_stride) ws->coarse = coarse_stride;
    if (k_chunk != ws->CK) {
        ws->CK = k_chunk;
        if (ws->partial) {
            (void)hipFree(ws->partial);
            ws->partial = nullptr;
            ws->partial_cap = 0;
        }
    }
    return AIY_OK;
}

int aiy_vfi_sweep_dev(aiy_ws* ws, const double* v_old, const double* a_grid, const double* s,
                      const double* P, double r, double w, double beta, double sigma,
                      const int32_t* hint, int mode, double* v_new, int32_t* idx,
                      double* policy_k, double* policy_c, double* diff, void* stream) {
    BellCall c{};
    c.v_old = v_old; c.a = a_grid; c.s = s; c.P = P; c.r = r; c.w = w; c.beta = beta;
    c.sigma = sigma; c.hint = hint; c.mode = mode; c.v_new = v_new; c.idx = idx;
    c.pk = policy_k; c.pc = policy_c; c.diff_out = diff;
    return bell_sweep_dev(ws, c, (hipStream_t)stream);
}

int aiy_vfi_sweeps_dev(aiy_ws* ws, double* v_a, double* v_b, const double* a_grid,
                       const double* s, const double* P, double r, double w, double beta,
                       double sigma, const int32_t* hint, int64_t nsweeps, int mode, int32_t* idx,
                       double* policy_k, double* policy_c, double* diff, void* stream) {
    if (!ws) return fail(AIY_BAD_ARG, "NULL workspace");
    if (nsweeps < 1) return fail(AIY_BAD_ARG, "nsweeps >= 1");
    if (!v_a || !v_b || v_a == v_b) return fail(AIY_BAD_ARG, "two distinct value buffers");
    if (!idx) return fail(AIY_BAD_ARG, "NULL idx (the next sweep's hint)");
    BellCall c{};
    c.a = a_grid; c.s = s; c.P = P; c.r = r; c.w = w; c.beta = beta; c.sigma = sigma;
    c.mode = mode; c.idx = idx; c.pk = policy_k; c.pc = policy_c;
    for (int64_t g = 0; g < nsweeps; ++g) {  // sweep g + 1 of the plain loop: ping-pong v_a / v_b
        c.v_old = (g & 1) ? v_b : v_a;
        c.v_new = (g & 1) ? v_a : v_b;
        c.hint = g ? idx : hint;
        c.diff_out = (g == nsweeps - 1) ? diff : nullptr;
        AIY_TRY(bell_sweep_dev(ws, c, (hipStream_t)stream));
    }
    return AIY_OK;
}

int aiy_vfi_solve_dev(aiy_ws* ws, double* v_a, double* v_b, const double* a_grid,
                      const double* s, const double* P, double r, double w, double beta,
                      double sigma, double tol, int64_t max_iter, int mode, int32_t* idx,
                      double* policy_k, double* policy_c, int64_t* iters, int* out_new,
                      void* stream) {
    if (!iters || !out_new) return fail(AIY_BAD_ARG, "NULL iters/out_new");
    BellCall c{};
    c.a = a_grid; c.s = s; c.P = P; c.r = r; c.w = w; c.beta = beta; c.sigma = sigma;
    c.mode = mode; c.idx = idx; c.pk = policy_k; c.pc = policy_c;
    return bell_solve_dev(ws, c, v_a, v_b, tol, max_iter, iters, out_new, (hipStream_t)stream);
}

int aiy_vfi_solve_batch_dev(aiy_ws* ws, int64_t C, const double* r, const double* w,
                            double* v_a, double* v_b, const double* a_grid, const double* s,
                            const double* P, double beta, double sigma, double tol,
                            int64_t max_iter, int use_hint, int32_t* idx, double* policy_k,
                            double* policy_c, int64_t* iters, int32_t* which, void* stream) {
    return bell_solve_batch_dev(ws, C, r, w, v_a, v_b, a_grid, s, P, beta, sigma, tol, max_iter,
                                use_hint, idx, policy_k, policy_c, iters, which,
                                (hipStream_t)stream);
}

int aiy_labor_vfi_sweep_dev(aiy_ws* ws, const double* v_old, const double* a_grid,
                            const double* s, const double* P, const double* labor_choice,
                            double r, double w, double beta, double sigma, double psi,
                            double eta, const int32_t* hint, double* v_new, int32_t* lin,
                            double* policy_k, double* policy_l, double* policy_c, double* diff,
                            void* stream) {
    BellCall c{};
    c.labor = true; c.Nl = ws ? ws->Nl : 0; c.L = labor_choice; c.psi = psi; c.eta = eta;
    c.v_old = v_old; c.a = a_grid; c.s = s; c.P = P; c.r = r; c.w = w; c.beta = beta;
    c.sigma = sigma; c.hint = hint; c.v_new = v_new; c.idx = lin; c.pk = policy_k;
    c.pl = policy_l; c.pc = policy_c; c.diff_out = diff;
    return bell_sweep_dev(ws, c, (hipStream_t)stream);
}

int aiy_labor_vfi_sweeps_dev(aiy_ws* ws, double* v_a, double* v_b, const double* a_grid,
                             const double* s, const double* P, const double* labor_choice,
                             double r, double w, double beta, double sigma, double psi,
                             double eta, const int32_t* hint, int64_t nsweeps, int32_t* lin,
                             double* policy_k, double* policy_l, double* policy_c, double* diff,
                             void* stream) {
    if (!ws) return fail(AIY_BAD_ARG, "NULL workspace");
    if (nsweeps < 1) return fail(AIY_BAD_ARG, "nsweeps >= 1");
    if (!v_a || !v_b || v_a == v_b) return fail(AIY_BAD_ARG, "two distinct value buffers");
    if (!lin) return fail(AIY_BAD_ARG, "NULL lin (the next sweep's hint)");
    BellCall c{};
    c.labor = true; c.Nl = ws->Nl; c.L = labor_choice; c.psi = psi; c.eta = eta;
    c.a = a_grid; c.s = s; c.P = P; c.r = r; c.w = w; c.beta = beta; c.sigma = sigma;
    c.idx = lin; c.pk = policy_k; c.pl = policy_l; c.pc = policy_c;
    for (int64_t g = 0; g < nsweeps; ++g) {  // sweep g + 1 of the loop: ping-pong v_a / v_b
        c.v_old = (g & 1) ? v_b : v_a;
        c.v_new = (g & 1) ? v_a : v_b;
        c.hint = g ? lin : hint;
        c.keep_incoming = (g == 0);
        c.diff_out = (g == nsweeps - 1) ? diff : nullptr;
        AIY_TRY(bell_sweep_dev(ws, c, (hipStream_t)stream));
    }
    return AIY_OK;
}

}  // extern "C"
