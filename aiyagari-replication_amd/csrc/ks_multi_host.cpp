// The MATLAB-facing multi-device Krusell-Smith VFI (ks_vfi_solve(n_devices > 1) /
// ks_vfi_solve_sharded; SURVEY §8(b) B5: one process, the gateway's thread drives every device;
// §8(e) E3).  Krusell_Smith_VFI.m:141-204 for one ALM coefficient B.
//
// Shards are the (K, Z) slices of ks_dist.shard_slices: up to nK shards split the K range (all
// four s); up to 2·nK split each K range again by aggregate state (s ∈ {0,1} vs {2,3}), so the
// reference grid (K = 4) runs on 8 devices.  Shard d lives on device d % visible and owns one
// ks_dev handle per ghost rectangle R_0 (its slice) .. R_{m−1} (ks_dist.ghost_rects: R_j is the
// smallest K range × all-s rectangle holding R_{j−1} and every column its nodes forecast into).
//
// Communication-avoiding Howard schedule (depth m): before a block of L ≤ m sweeps a shard
// receives every foreign column of R_L from its owner (peer copies over xGMI; a column is
// contiguous, so a run of columns is one copy), builds the slopes of what R_{L−1} reads, then
// sweep i of the block runs on R_{L−i} with the fused Howard+slopes kernel (one launch per
// sweep).  Other shards' columns are swept redundantly by the same kernels on the same
// inputs, so every value is the single-device solve's bit for bit.  After a policy
// improvement a shard receives k_opt on R_{m−1} and rebuilds the segment hints there.
// Synchronisation is by events on the streams, never the host, except for the one read of
// the stop criterion per VFI iteration: a reader's copies wait for the owner's `done`; an
// owner's next write into the buffer that was read waits for its readers' `copied`.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <vector>

#include "aiy_common.hpp"
#include "host_ctx.hpp"
#include "ks.hpp"
#include "ws.hpp"

namespace aiy {

namespace {

struct Rect {
    int K0, K1, s0, s1;
};

// ks_dist.shard_slices
Rect shard_slice(int nK, int rank, int world) {
    auto range = [](int n, int r, int w) { return std::make_pair(n * r / w, n * (r + 1) / w); };
    if (world <= nK) {
        auto k = range(nK, rank, world);
        return {k.first, k.second, 0, 4};
    }
    const int h = (world + 1) / 2;
    if (rank < h) {
        auto k = range(nK, rank, h);
        return {k.first, k.second, 0, 2};
    }
    auto k = range(nK, rank - h, world - h);
    return {k.first, k.second, 2, 4};
}

// ks_dist.ghost_rects
std::vector<Rect> ghost_rects(const std::vector<KsSlice>& sl, int nK, Rect r0, int depth) {
    std::vector<Rect> out{r0};
    for (int j = 0; j < depth; ++j) {
        const Rect r = out.back();
        int lo = r.K0, hi = r.K1;
        for (int s = r.s0; s < r.s1; ++s)
            for (int K = r.K0; K < r.K1; ++K) {
                const int t = sl[s * nK + K].kp_idx;
                lo = std::min(lo, t);
                hi = std::max(hi, t + 1);
            }
        out.push_back({lo, hi, 0, 4});
    }
    return out;
}

struct Run {
    int owner, c0, c1;  // flat columns [c0, c1) (c = s·nK + K) held by shard `owner`
};

struct Shard {
    int dev = 0;
    hipStream_t st = nullptr;
    hipEvent_t done = nullptr, copied = nullptr;
    Rect own{};
    std::vector<Rect> rects;             // R_0 .. R_m
    std::vector<ks_dev*> h;              // handles of R_0 .. R_{m−1} (ghosts share R_0's hints)
    std::vector<std::vector<Run>> recv;  // recv[L]: foreign columns of R_L, L = 1..m
    double *V[2] = {nullptr, nullptr}, *dV[2] = {nullptr, nullptr};
    double *kopt = nullptr, *Vold = nullptr;
    unsigned long long* red = nullptr;   // device [2]: ks_dev_reldiff's folded slots
    std::vector<int> guardV[2], guardK;  // shards whose `copied` must precede our next write
};

// foreign columns of rect r for shard q, as runs of consecutive columns with one owner
std::vector<Run> foreign_runs(const Rect& r, int nK, const std::vector<int>& owner, int q) {
    std::vector<Run> out;
    for (int s = r.s0; s < r.s1; ++s)
        for (int K = r.K0; K < r.K1; ++K) {
            const int c = s * nK + K, o = owner[c];
            if (o == q) continue;
            if (!out.empty() && out.back().owner == o && out.back().c1 == c) out.back().c1 = c + 1;
            else out.push_back({o, c, c + 1});
        }
    return out;
}

}  // namespace

// The direct (peer-read) schedule, depth = 0.  Every shard keeps only its OWN columns of value
// and slopes current, in its own double-buffered arrays; the fused Howard+slopes sweep and the
// improvement read each forecast column (Krusell_Smith_VFI.m:343-349) where its owner keeps it,
// through a per-shard table of column pointers into the owners' buffers (peer pointers over
// xGMI, peer access enabled) — no column is copied and no ghost column is swept.  Sweep t reads
// parity cur and writes cur ^ 1; before it a shard waits (stream waits on events, never the
// host) for the sweep t − 1 of every neighbour — the owners of what it reads (their values are
// complete) and the shards that read its columns (they are done with the buffer it is about to
// overwrite).  Same kernels on the same values: bit for bit the single-device solve.
int ks_vfi_solve_direct_impl(double* value, double* k_opt, const double* k_grid,
                             const double* K_grid, const double* B, const double* P,
                             const double* params, int64_t nk, int64_t nK, int64_t howard_steps,
                             double tol, int64_t max_vfi, int n_shards, int64_t* iters,
                             double* rel_diff) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1)
        return fail(AIY_NO_DEVICE, "no HIP device visible");
    AIY_TRY(check_grid(k_grid, nk));
    const int W = (int)std::max<int64_t>(1, std::min<int64_t>(n_shards, 2 * nK));
    KsParams p;
    memcpy(&p, params, sizeof p);
    std::vector<KsSlice> sl;
    ks_slices(p, B, K_grid, (int)nK, sl);
    const int C = (int)(4 * nK);
    const size_t n = (size_t)nk * C, nb = n * sizeof(double), colb = nk * sizeof(double);
    std::vector<int> owner(C, -1);
    struct DShard {
        int dev = 0;
        hipStream_t st = nullptr;
        hipEvent_t done[2] = {nullptr, nullptr};  // sweep writing parity b complete
        Rect own{};
        ks_dev* h = nullptr;
        double *V[2] = {nullptr, nullptr}, *dV[2] = {nullptr, nullptr};
        double *kopt = nullptr, *Vold = nullptr;
        const double** tab[2] = {nullptr, nullptr};  // device: column pointers per parity
        unsigned long long* red = nullptr;
        std::vector<int> nbr;  // shards this one waits for before each sweep
    };
    std::vector<DShard> S(W);
    for (int q = 0; q < W; ++q) {
        S[q].own = shard_slice((int)nK, q, W);
        for (int s = S[q].own.s0; s < S[q].own.s1; ++s)
            for (int K = S[q].own.K0; K < S[q].own.K1; ++K) owner[s * nK + K] = q;
    }
    // neighbours: owners of the forecast columns a shard reads, and the shards reading its own
    std::vector<std::vector<char>> nb_m(W, std::vector<char>(W, 0));
    for (int q = 0; q < W; ++q) {
        const Rect& r = S[q].own;
        for (int s = r.s0; s < r.s1; ++s)
            for (int K = r.K0; K < r.K1; ++K)
                for (int sn = 0; sn < 4; ++sn) {
                    const int o = owner[sn * nK + sl[s * nK + K].kp_idx];
                    if (o != q) nb_m[q][o] = nb_m[o][q] = 1;
                }
    }
    for (int q = 0; q < W; ++q)
        for (int o = 0; o < W; ++o)
            if (nb_m[q][o]) S[q].nbr.push_back(o);
    int rc = AIY_OK;
    auto cleanup = [&]() {
        for (auto& sh : S) {
            (void)hipSetDevice(sh.dev);
            if (sh.st) (void)hipStreamSynchronize(sh.st);
        }
        for (auto& sh : S) {
            (void)hipSetDevice(sh.dev);
            if (sh.h) ks_dev_destroy(sh.h);
            void* ps[] = {sh.V[0], sh.V[1], sh.dV[0], sh.dV[1], sh.kopt, sh.Vold, sh.red,
                          (void*)sh.tab[0], (void*)sh.tab[1]};
            for (void* q : ps)
                if (q) (void)hipFree(q);
            for (auto& e : sh.done)
                if (e) (void)hipEventDestroy(e);
            if (sh.st) (void)hipStreamDestroy(sh.st);
        }
    };
#define KD_CHECK(call)                                                                   \
    do {                                                                                 \
        hipError_t e_ = (call);                                                          \
        if (e_ != hipSuccess) {                                                          \
            rc = fail(AIY_HIP_ERROR, "%s: %s", #call, hipGetErrorString(e_));            \
            cleanup();                                                                   \
            return rc;                                                                   \
        }                                                                                \
    } while (0)
#define KD_TRY(expr)          \
    do {                      \
        rc = (expr);          \
        if (rc != AIY_OK) {   \
            cleanup();        \
            return rc;        \
        }                     \
    } while (0)
    const int nd = std::min(ndev, W);
    for (int a = 0; a < nd; ++a)
        for (int b = 0; b < nd; ++b) {
            if (a == b) continue;
            int can = 0;
            KD_CHECK(hipDeviceCanAccessPeer(&can, a, b));
            if (!can) {
                rc = fail(AIY_HIP_ERROR, "device %d cannot access device %d: the direct schedule "
                          "reads peer memory (use depth >= 1)", a, b);
                cleanup();
                return rc;
            }
            KD_CHECK(hipSetDevice(a));
            const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) KD_CHECK(e);
            (void)hipGetLastError();
        }
    for (int q = 0; q < W; ++q) {
        DShard& sh = S[q];
        sh.dev = q % ndev;
        KD_CHECK(hipSetDevice(sh.dev));
        KD_CHECK(hipStreamCreateWithFlags(&sh.st, hipStreamNonBlocking));
        for (auto& e : sh.done) KD_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        for (int b = 0; b < 2; ++b) {
            KD_CHECK(hipMalloc((void**)&sh.V[b], nb));
            KD_CHECK(hipMalloc((void**)&sh.dV[b], nb));
            KD_CHECK(hipMalloc((void**)&sh.tab[b], 2 * (size_t)C * sizeof(double*)));
        }
        KD_CHECK(hipMalloc((void**)&sh.kopt, nb));
        KD_CHECK(hipMalloc((void**)&sh.Vold, nb));
        KD_CHECK(hipMalloc((void**)&sh.red, 2 * sizeof(unsigned long long)));
        KD_TRY(ks_dev_create_slice(k_grid, K_grid, B, P, params, nk, nK, sh.own.K0, sh.own.K1,
                                   sh.own.s0, sh.own.s1, &sh.h));
        KD_CHECK(hipMemcpyAsync(sh.V[0], value, nb, hipMemcpyHostToDevice, sh.st));
        KD_CHECK(hipMemcpyAsync(sh.kopt, k_opt, nb, hipMemcpyHostToDevice, sh.st));
    }
    for (int q = 0; q < W; ++q) {  // column tables: column c of parity b lives at its owner
        DShard& sh = S[q];
        KD_CHECK(hipSetDevice(sh.dev));
        for (int b = 0; b < 2; ++b) {
            std::vector<const double*> t(2 * (size_t)C);
            for (int c = 0; c < C; ++c) {
                const DShard& o = S[owner[c]];
                t[c] = o.V[b] + (size_t)c * nk;
                t[C + c] = o.dV[b] + (size_t)c * nk;
            }
            KD_CHECK(hipMemcpy(sh.tab[b], t.data(), t.size() * sizeof(double*), hipMemcpyHostToDevice));
        }
        // the slopes of the own columns of the incoming value (what sweep 1 and the first
        // improvement read), then "sweep 0 writing parity 0" is done
        KD_TRY(ks_dev_slopes_own(sh.h, sh.V[0], sh.dV[0], sh.st));
        KD_CHECK(hipEventRecord(sh.done[0], sh.st));
    }
    int cur = 0;
    auto wait_nbrs = [&](DShard& sh) -> int {  // the neighbours' sweep that wrote parity cur
        for (int o : sh.nbr) AIY_HIP(hipStreamWaitEvent(sh.st, S[o].done[cur], 0));
        return AIY_OK;
    };
    double rel = NAN;
    int64_t it;
    std::vector<unsigned long long> hred(2 * W);
    for (it = 1; it <= max_vfi; ++it) {
        for (auto& sh : S) {  // value_old = value (:145), own columns
            KD_CHECK(hipSetDevice(sh.dev));
            for (int s = sh.own.s0; s < sh.own.s1; ++s) {
                const size_t off = (size_t)(s * nK + sh.own.K0) * nk;
                KD_CHECK(hipMemcpyAsync(sh.Vold + off, sh.V[cur] + off,
                                        (size_t)(sh.own.K1 - sh.own.K0) * colb,
                                        hipMemcpyDeviceToDevice, sh.st));
            }
        }
        if ((it - 1) % 5 == 0) {  // policy improvement (:148-168), forecast columns in place
            for (auto& sh : S) {
                KD_CHECK(hipSetDevice(sh.dev));
                KD_TRY(wait_nbrs(sh));
                KD_TRY(ks_dev_set_columns(sh.h, (const void* const*)sh.tab[cur]));
                KD_TRY(ks_dev_improve_direct(sh.h, sh.kopt, sh.st));
            }
        }
        for (int64_t hs = 0; hs < howard_steps; ++hs) {  // Jacobi Howard sweeps (:172-192)
            for (auto& sh : S) {
                KD_CHECK(hipSetDevice(sh.dev));
                KD_TRY(wait_nbrs(sh));
                KD_TRY(ks_dev_set_columns(sh.h, (const void* const*)sh.tab[cur]));
                KD_TRY(ks_dev_howard_fused(sh.h, sh.V[cur], sh.dV[cur], sh.kopt, sh.V[cur ^ 1],
                                           sh.dV[cur ^ 1], sh.st));
                KD_CHECK(hipEventRecord(sh.done[cur ^ 1], sh.st));
            }
            cur ^= 1;
        }
        for (int q = 0; q < W; ++q) {  // :195, NaN ignored, max over shards
            DShard& sh = S[q];
            KD_CHECK(hipSetDevice(sh.dev));
            KD_TRY(ks_dev_reldiff(sh.h, sh.V[cur], sh.Vold, sh.red, sh.st));
            KD_CHECK(hipMemcpyAsync(&hred[2 * q], sh.red, 2 * sizeof(unsigned long long),
                                    hipMemcpyDeviceToHost, sh.st));
        }
        double mx = NAN;
        for (int q = 0; q < W; ++q) {
            KD_CHECK(hipSetDevice(S[q].dev));
            KD_CHECK(hipStreamSynchronize(S[q].st));
            if (hred[2 * q + 1]) {
                const double d = aiy_bitsd(hred[2 * q]);
                if (d == d && !(mx >= d)) mx = d;
            }
        }
        rel = mx;
        if (rel < tol) break;
    }
    if (it > max_vfi) it = max_vfi;
    for (auto& sh : S) {  // every shard's own columns of value and k_opt
        KD_CHECK(hipSetDevice(sh.dev));
        for (int s = sh.own.s0; s < sh.own.s1; ++s) {
            const size_t off = (size_t)(s * nK + sh.own.K0) * nk;
            const size_t bytes = (size_t)(sh.own.K1 - sh.own.K0) * colb;
            KD_CHECK(hipMemcpyAsync(value + off, sh.V[cur] + off, bytes, hipMemcpyDeviceToHost, sh.st));
            KD_CHECK(hipMemcpyAsync(k_opt + off, sh.kopt + off, bytes, hipMemcpyDeviceToHost, sh.st));
        }
        KD_CHECK(hipStreamSynchronize(sh.st));
    }
    cleanup();
    *iters = it;
    *rel_diff = rel;
    return AIY_OK;
#undef KD_CHECK
#undef KD_TRY
}

int ks_vfi_solve_sharded_impl(double* value, double* k_opt, const double* k_grid,
                              const double* K_grid, const double* B, const double* P,
                              const double* params, int64_t nk, int64_t nK,
                              int64_t howard_steps, double tol, int64_t max_vfi, int n_shards,
                              int depth, int64_t* iters, double* rel_diff) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1)
        return fail(AIY_NO_DEVICE, "no HIP device visible");
    AIY_TRY(check_grid(k_grid, nk));
    const int W = (int)std::max<int64_t>(1, std::min<int64_t>(n_shards, 2 * nK));
    const int m = std::max(1, depth);
    KsParams p;
    memcpy(&p, params, sizeof p);
    std::vector<KsSlice> sl;
    ks_slices(p, B, K_grid, (int)nK, sl);
    const size_t n = (size_t)nk * nK * 4, nb = n * sizeof(double), colb = nk * sizeof(double);
    std::vector<int> owner(4 * nK, -1);
    std::vector<Shard> S(W);
    for (int q = 0; q < W; ++q) {
        S[q].own = shard_slice((int)nK, q, W);
        for (int s = S[q].own.s0; s < S[q].own.s1; ++s)
            for (int K = S[q].own.K0; K < S[q].own.K1; ++K) owner[s * nK + K] = q;
    }
    int rc = AIY_OK;
    auto cleanup = [&]() {
        for (auto& sh : S) {
            (void)hipSetDevice(sh.dev);
            if (sh.st) (void)hipStreamSynchronize(sh.st);
            for (size_t j = sh.h.size(); j-- > 0;) ks_dev_destroy(sh.h[j]);  // ghosts first
            void* ps[] = {sh.V[0], sh.V[1], sh.dV[0], sh.dV[1], sh.kopt, sh.Vold, sh.red};
            for (void* q : ps)
                if (q) (void)hipFree(q);
            if (sh.done) (void)hipEventDestroy(sh.done);
            if (sh.copied) (void)hipEventDestroy(sh.copied);
            if (sh.st) (void)hipStreamDestroy(sh.st);
        }
    };
#define KS_CHECK(call)                                                                   \
    do {                                                                                 \
        hipError_t e_ = (call);                                                          \
        if (e_ != hipSuccess) {                                                          \
            rc = fail(AIY_HIP_ERROR, "%s: %s", #call, hipGetErrorString(e_));            \
            cleanup();                                                                   \
            return rc;                                                                   \
        }                                                                                \
    } while (0)
#define KS_TRY(expr)          \
    do {                      \
        rc = (expr);          \
        if (rc != AIY_OK) {   \
            cleanup();        \
            return rc;        \
        }                     \
    } while (0)
    // peer access between every pair of devices in use (once; already-enabled is fine)
    const int nd = std::min(ndev, W);
    for (int a = 0; a < nd; ++a)
        for (int b = 0; b < nd; ++b) {
            if (a == b) continue;
            int can = 0;
            KS_CHECK(hipDeviceCanAccessPeer(&can, a, b));
            if (!can) continue;
            KS_CHECK(hipSetDevice(a));
            const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) KS_CHECK(e);
            (void)hipGetLastError();  // clear a sticky "already enabled"
        }
    for (int q = 0; q < W; ++q) {
        Shard& sh = S[q];
        sh.dev = q % ndev;
        sh.rects = ghost_rects(sl, (int)nK, sh.own, m);
        sh.recv.resize(m + 1);
        for (int L = 1; L <= m; ++L) sh.recv[L] = foreign_runs(sh.rects[L], (int)nK, owner, q);
        KS_CHECK(hipSetDevice(sh.dev));
        KS_CHECK(hipStreamCreateWithFlags(&sh.st, hipStreamNonBlocking));
        KS_CHECK(hipEventCreateWithFlags(&sh.done, hipEventDisableTiming));
        KS_CHECK(hipEventCreateWithFlags(&sh.copied, hipEventDisableTiming));
        for (int b = 0; b < 2; ++b) {
            KS_CHECK(hipMalloc((void**)&sh.V[b], nb));
            KS_CHECK(hipMalloc((void**)&sh.dV[b], nb));
        }
        KS_CHECK(hipMalloc((void**)&sh.kopt, nb));
        KS_CHECK(hipMalloc((void**)&sh.Vold, nb));
        KS_CHECK(hipMalloc((void**)&sh.red, 2 * sizeof(unsigned long long)));
        for (int j = 0; j < m; ++j) {
            const Rect& r = sh.rects[j];
            ks_dev* hd = nullptr;
            KS_TRY(ks_dev_create_slice(k_grid, K_grid, B, P, params, nk, nK, r.K0, r.K1, r.s0,
                                       r.s1, &hd));
            sh.h.push_back(hd);
            if (j) KS_TRY(ks_dev_share_hints(hd, sh.h[0]));
        }
        KS_CHECK(hipMemcpyAsync(sh.V[0], value, nb, hipMemcpyHostToDevice, sh.st));
        KS_CHECK(hipMemcpyAsync(sh.kopt, k_opt, nb, hipMemcpyHostToDevice, sh.st));
        KS_CHECK(hipStreamSynchronize(sh.st));
    }
    // hints of the ghost rectangles from the incoming k_opt (improve writes R_0's; the first
    // iteration improves before any sweep, but a hint is only a hint: this keeps them sane)
    int cur = 0;
    auto wait_guard = [&](Shard& sh, std::vector<int>& g) -> int {
        for (int r : g) AIY_HIP(hipStreamWaitEvent(sh.st, S[r].copied, 0));
        g.clear();
        return AIY_OK;
    };
    // every shard receives plan[L] of buffer `buf` (V[cur] or kopt) from the owners
    auto exchange = [&](int L, bool kbuf) -> int {
        for (auto& sh : S) {
            AIY_HIP(hipSetDevice(sh.dev));
            AIY_HIP(hipEventRecord(sh.done, sh.st));
        }
        for (int q = 0; q < W; ++q) {
            Shard& sh = S[q];
            if (sh.recv[L].empty()) continue;
            AIY_HIP(hipSetDevice(sh.dev));
            std::vector<char> waited(W, 0);
            for (const Run& r : sh.recv[L]) {
                Shard& o = S[r.owner];
                if (!waited[r.owner]) {
                    AIY_HIP(hipStreamWaitEvent(sh.st, o.done, 0));
                    waited[r.owner] = 1;
                    (kbuf ? o.guardK : o.guardV[cur]).push_back(q);
                }
                const size_t off = (size_t)r.c0 * nk, bytes = (size_t)(r.c1 - r.c0) * colb;
                double* dst = (kbuf ? sh.kopt : sh.V[cur]) + off;
                const double* src = (kbuf ? o.kopt : o.V[cur]) + off;
                if (o.dev == sh.dev)
                    AIY_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, sh.st));
                else
                    AIY_HIP(hipMemcpyPeerAsync(dst, sh.dev, src, o.dev, bytes, sh.st));
            }
            AIY_HIP(hipEventRecord(sh.copied, sh.st));
        }
        return AIY_OK;
    };
    double rel = NAN;
    int64_t it;
    std::vector<unsigned long long> hred(2 * W);
    for (it = 1; it <= max_vfi; ++it) {
        for (auto& sh : S) {  // value_old = value (:145), the shard's own columns
            KS_CHECK(hipSetDevice(sh.dev));
            for (int s = sh.own.s0; s < sh.own.s1; ++s) {
                const size_t off = (size_t)(s * nK + sh.own.K0) * nk;
                KS_CHECK(hipMemcpyAsync(sh.Vold + off, sh.V[cur] + off,
                                        (size_t)(sh.own.K1 - sh.own.K0) * colb,
                                        hipMemcpyDeviceToDevice, sh.st));
            }
        }
        if ((it - 1) % 5 == 0) {  // policy improvement (:148-168): reads the halo of R_0
            KS_TRY(exchange(1, false));
            for (auto& sh : S) {
                KS_CHECK(hipSetDevice(sh.dev));
                KS_TRY(wait_guard(sh, sh.guardK));
                KS_TRY(ks_dev_improve(sh.h[0], sh.V[cur], sh.kopt, sh.st));
            }
            if (m > 1) {  // the ghost sweeps read k_opt on R_{m−1}
                KS_TRY(exchange(m - 1, true));
                for (auto& sh : S) {
                    KS_CHECK(hipSetDevice(sh.dev));
                    KS_TRY(ks_dev_hints(sh.h[m - 1], sh.kopt, sh.st));
                }
            }
        }
        for (int64_t done = 0; done < howard_steps;) {  // Jacobi Howard sweeps (:172-192)
            const int L = (int)std::min<int64_t>(m, howard_steps - done);
            KS_TRY(exchange(L, false));
            for (auto& sh : S) {
                KS_CHECK(hipSetDevice(sh.dev));
                KS_TRY(ks_dev_slopes(sh.h[L - 1], sh.V[cur], sh.dV[cur], sh.st));
            }
            for (int i = 1; i <= L; ++i) {
                for (auto& sh : S) {
                    KS_CHECK(hipSetDevice(sh.dev));
                    KS_TRY(wait_guard(sh, sh.guardV[cur ^ 1]));  // about to write V[cur ^ 1]
                    KS_TRY(ks_dev_howard_fused(sh.h[L - i], sh.V[cur], sh.dV[cur], sh.kopt,
                                               sh.V[cur ^ 1], sh.dV[cur ^ 1], sh.st));
                }
                cur ^= 1;
            }
            done += L;
        }
        for (int q = 0; q < W; ++q) {  // :195, NaN ignored, max over shards
            Shard& sh = S[q];
            KS_CHECK(hipSetDevice(sh.dev));
            KS_TRY(ks_dev_reldiff(sh.h[0], sh.V[cur], sh.Vold, sh.red, sh.st));
            KS_CHECK(hipMemcpyAsync(&hred[2 * q], sh.red, 2 * sizeof(unsigned long long),
                                    hipMemcpyDeviceToHost, sh.st));
        }
        double mx = NAN;
        for (int q = 0; q < W; ++q) {
            KS_CHECK(hipSetDevice(S[q].dev));
            KS_CHECK(hipStreamSynchronize(S[q].st));
            if (hred[2 * q + 1]) {
                const double d = aiy_bitsd(hred[2 * q]);
                if (d == d && !(mx >= d)) mx = d;
            }
        }
        rel = mx;
        if (rel < tol) break;
    }
    if (it > max_vfi) it = max_vfi;
    for (auto& sh : S) {  // every shard's own columns of value and k_opt
        KS_CHECK(hipSetDevice(sh.dev));
        for (int s = sh.own.s0; s < sh.own.s1; ++s) {
            const size_t off = (size_t)(s * nK + sh.own.K0) * nk;
            const size_t bytes = (size_t)(sh.own.K1 - sh.own.K0) * colb;
            KS_CHECK(hipMemcpyAsync(value + off, sh.V[cur] + off, bytes, hipMemcpyDeviceToHost, sh.st));
            KS_CHECK(hipMemcpyAsync(k_opt + off, sh.kopt + off, bytes, hipMemcpyDeviceToHost, sh.st));
        }
        KS_CHECK(hipStreamSynchronize(sh.st));
    }
    cleanup();
    *iters = it;
    *rel_diff = rel;
    return AIY_OK;
#undef KS_CHECK
#undef KS_TRY
}

}  // namespace aiy

using namespace aiy;

extern "C" int ks_vfi_solve_sharded(double* value, double* k_opt, const double* k_grid,
                                    const double* K_grid, const double* B, const double* P,
                                    const double* params, int64_t nk, int64_t nK,
                                    int64_t howard_steps, double tol, int64_t max_vfi,
                                    int n_shards, int depth, int64_t* iters, double* rel_diff) {
    if (!value || !k_opt || !k_grid || !K_grid || !B || !P || !params || !iters || !rel_diff)
        return fail(AIY_BAD_ARG, "NULL argument");
    if (max_vfi < 1 || howard_steps < 0) return fail(AIY_BAD_ARG, "max_vfi >= 1, howard_steps >= 0");
    if (nk < 3 || nK < 1) return fail(AIY_BAD_SHAPE, "need k_size >= 3 and K_size >= 1");
    if (n_shards < 1 || depth < 0) return fail(AIY_BAD_ARG, "n_shards >= 1 and depth >= 0");
    std::lock_guard<std::mutex> lk(host_mutex());
    int cur = 0;
    (void)hipGetDevice(&cur);
    const int rc =
        depth == 0 ? ks_vfi_solve_direct_impl(value, k_opt, k_grid, K_grid, B, P, params, nk, nK,
                                              howard_steps, tol, max_vfi, n_shards, iters,
                                              rel_diff)
                   : ks_vfi_solve_sharded_impl(value, k_opt, k_grid, K_grid, B, P, params, nk,
                                               nK, howard_steps, tol, max_vfi, n_shards, depth,
                                               iters, rel_diff);
    (void)hipSetDevice(cur);
    return rc;
}
