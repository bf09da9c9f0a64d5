// A6/A7 entry points (Krusell_Smith_VFI.m:143-204).  value / k_opt are k x K x S
// column-major, exactly as in the script; P is MATLAB's 4 x 4; params = 13 doubles
// {beta, alpha, delta, k_min, k_max, ug, ub, l_bar, mu, z_grid(1:2), eps_grid(1:2)}.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <mutex>
#include <vector>

#include "aiy_common.hpp"
#include "host_ctx.hpp"
#include "ks.hpp"
#include "ws.hpp"

namespace aiy {

// per-slice constants, in the script's own operation order (libm pow/exp/log on the host)
void ks_slices(const KsParams& p, const double* B, const double* K_grid, int nK,
                      std::vector<KsSlice>& out) {
    out.resize(4 * nK);
    const double zg[2] = {p.z1, p.z2}, eg[2] = {p.e1, p.e2};
    for (int si = 0; si < 4; ++si)
        for (int Ki = 0; Ki < nK; ++Ki) {
            KsSlice sl{};
            double K = K_grid[Ki];
            // bellman_value: current_z = z_grid((s_i <= 2) + 1)  (flipped, :332)
            double z = zg[(si + 1 <= 2) ? 1 : 0];
            double Kp;
            if (z == zg[0]) Kp = exp(B[0] + B[1] * log(fmax(K, 1e-8)));
            else Kp = exp(B[2] + B[3] * log(fmax(K, 1e-8)));
            Kp = fmax(fmin(Kp, K_grid[nK - 1]), K_grid[0]);
            int idx = 0;
            double bd = fabs(K_grid[0] - Kp);
            for (int q = 1; q < nK; ++q) {
                double dd = fabs(K_grid[q] - Kp);
                if (dd < bd) { bd = dd; idx = q; }
            }
            sl.kp_idx = idx;
            double L = p.l_bar * (1 - p.ug * (double)(z == zg[0]) - p.ub * (double)(z == zg[1]));
            double r_val = p.alpha * z * pow(K, p.alpha - 1) * pow(L, 1 - p.alpha);
            double w_val = (1 - p.alpha) * z * pow(K, p.alpha) * pow(L, -p.alpha);
            double eps = (si % 2 == 0) ? eg[0] : eg[1];  // s_grid(s_i, 2), :19-20
            sl.a1 = r_val + 1 - p.delta;
            sl.a2 = w_val * (eps * p.l_bar);
            // resources for fminbnd's upper bound use the table z (:107-115, :149-155)
            double zt = (si < 2) ? zg[0] : zg[1];
            double Lt = p.l_bar * (1 - p.ug * (double)(zt == zg[0]) - p.ub * (double)(zt == zg[1]));
            double wt = (1 - p.alpha) * zt * pow(K, p.alpha) * pow(Lt, -p.alpha);
            double rt = p.alpha * zt * pow(K, p.alpha - 1) * pow(Lt, 1 - p.alpha);
            sl.b1 = rt + 1 - p.delta;
            sl.b2 = wt * (eps * p.l_bar + (1 - eps) * p.mu);
            out[si * nK + Ki] = sl;
        }
}

struct KsDev {
    double *kg, *P, *V, *V2, *dV, *Vold, *kopt;
    int* nfev;
    int* seg;  // Howard segment hints (verified before use, so never initialised)
    KsSlice* sl;
    KsOut* out;
    unsigned long long* slots;
};

static int ks_stage(HostCtx* c, const double* value, const double* k_opt, const double* k_grid,
                    const double* K_grid, const double* B, const double* P, const double* params,
                    int64_t nk, int64_t nK, KsArgs& A, KsDev& D) {
    if (!value || !k_grid || !K_grid || !B || !P || !params)
        return fail(AIY_BAD_ARG, "NULL argument");
    if (nk < 3 || nK < 1) return fail(AIY_BAD_SHAPE, "need k_size >= 3 and K_size >= 1");
    AIY_TRY(check_grid(k_grid, nk));
    KsParams p;
    memcpy(&p, params, sizeof p);
    std::vector<KsSlice> sl;
    ks_slices(p, B, K_grid, (int)nK, sl);
    size_t n = (size_t)nk * nK * 4, nb = n * sizeof(double);
    AIY_TRY(c->buf("ks_kg", nk * sizeof(double), (void**)&D.kg));
    AIY_TRY(c->buf("ks_P", 16 * sizeof(double), (void**)&D.P));
    AIY_TRY(c->buf("ks_V", nb, (void**)&D.V));
    AIY_TRY(c->buf("ks_V2", nb, (void**)&D.V2));
    AIY_TRY(c->buf("ks_dV", nb, (void**)&D.dV));
    AIY_TRY(c->buf("ks_Vold", nb, (void**)&D.Vold));
    AIY_TRY(c->buf("ks_kopt", nb, (void**)&D.kopt));
    AIY_TRY(c->buf("ks_nfev", n * sizeof(int), (void**)&D.nfev));
    AIY_TRY(c->buf("ks_seg", n * sizeof(int), (void**)&D.seg));
    AIY_TRY(c->buf("ks_sl", sl.size() * sizeof(KsSlice), (void**)&D.sl));
    AIY_TRY(c->buf("ks_out", sizeof(KsOut), (void**)&D.out));
    AIY_TRY(c->buf("ks_slots", 2 * kDiffSlots * sizeof(unsigned long long), (void**)&D.slots));
    double Pr[16];
    for (int i = 0; i < 4; ++i)
        for (int m = 0; m < 4; ++m) Pr[i * 4 + m] = P[i + m * 4];
    AIY_HIP(hipMemcpyAsync(D.kg, k_grid, nk * sizeof(double), hipMemcpyHostToDevice, c->st));
    AIY_HIP(hipMemcpyAsync(D.P, Pr, sizeof Pr, hipMemcpyHostToDevice, c->st));
    AIY_HIP(hipMemcpyAsync(D.V, value, nb, hipMemcpyHostToDevice, c->st));
    if (k_opt) AIY_HIP(hipMemcpyAsync(D.kopt, k_opt, nb, hipMemcpyHostToDevice, c->st));
    AIY_HIP(hipMemcpyAsync(D.sl, sl.data(), sl.size() * sizeof(KsSlice), hipMemcpyHostToDevice, c->st));
    AIY_HIP(hipStreamSynchronize(c->st));
    A = KsArgs{};
    A.nk = (int)nk; A.nK = (int)nK; A.node0 = 0; A.n_local = (int)n;
    A.k_grid = D.kg; A.P = D.P; A.slice = D.sl;
    A.beta = p.beta; A.k_min = p.k_min; A.k_max = p.k_max;
    A.seg_hint = D.seg;
    return AIY_OK;
}

int ks_vfi_solve_multi(double* value, double* k_opt, const double* k_grid, const double* K_grid,
                       const double* B, const double* P, const double* params, int64_t nk,
                       int64_t nK, int64_t howard_steps, double tol, int64_t max_vfi,
                       int n_devices, int64_t* iters, double* rel_diff);

static int ks_read_slots(HostCtx* c, const unsigned long long* slots, double* d) {
    std::vector<unsigned long long> h(2 * kDiffSlots);
    AIY_HIP(hipMemcpyAsync(h.data(), slots, h.size() * sizeof(unsigned long long),
                           hipMemcpyDeviceToHost, c->st));
    AIY_HIP(hipStreamSynchronize(c->st));
    *d = fold_slots_host(h.data());
    return AIY_OK;
}

// ---------------------------------------------------------------------------- multi-device
// Shards own contiguous K ranges for all four s (columns (s, K) with K in range); shard d
// runs on device d % visible.  A Howard sweep reads, for each owned slice, the columns
// (K'_idx, s') — with the identity-like ALM mostly its own; the remote ones are refreshed by
// peer copies (xGMI) after every sweep.  Results equal the single-device solve bit for bit.
struct KsShard {
    int dev;
    hipStream_t st = nullptr;
    hipEvent_t done = nullptr;
    int K0, K1;                      // owned K range
    std::vector<int> cols;           // columns to keep fresh (own ∪ needed), sn*nK + K
    std::vector<std::pair<int, int>> remote;  // (column, owner shard)
    double *kg = nullptr, *P = nullptr, *V = nullptr, *V2 = nullptr, *dV = nullptr,
           *Vold = nullptr, *kopt = nullptr;
    int* seg = nullptr;              // Howard segment hints (verified before use)
    int* dcols = nullptr;
    KsSlice* sl = nullptr;
    unsigned long long* slots = nullptr;
};

static int ks_vfi_solve_multi_impl(double* value, double* k_opt, const double* k_grid,
                                   const double* K_grid, const double* B, const double* P,
                                   const double* params, int64_t nk, int64_t nK,
                                   int64_t howard_steps, double tol, int64_t max_vfi,
                                   int n_shards, int64_t* iters, double* rel_diff) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1)
        return fail(AIY_NO_DEVICE, "no HIP device visible");
    if (n_shards > nK) n_shards = (int)nK;
    AIY_TRY(check_grid(k_grid, nk));
    KsParams p;
    memcpy(&p, params, sizeof p);
    std::vector<KsSlice> sl;
    ks_slices(p, B, K_grid, (int)nK, sl);
    double Pr[16];
    for (int i = 0; i < 4; ++i)
        for (int m = 0; m < 4; ++m) Pr[i * 4 + m] = P[i + m * 4];
    const size_t n = (size_t)nk * nK * 4, nb = n * sizeof(double), colb = nk * sizeof(double);
    std::vector<KsShard> S(n_shards);
    std::vector<int> owner(nK);
    for (int d = 0; d < n_shards; ++d) {
        S[d].K0 = (int)(nK * d / n_shards);
        S[d].K1 = (int)(nK * (d + 1) / n_shards);
        for (int K = S[d].K0; K < S[d].K1; ++K) owner[K] = d;
    }
    int rc = AIY_OK;
    auto cleanup = [&]() {
        for (auto& sh : S) {
            (void)hipSetDevice(sh.dev);
            void* ps[] = {sh.kg, sh.P, sh.V, sh.V2, sh.dV, sh.Vold, sh.kopt, sh.dcols, sh.sl, sh.slots, sh.seg};
            for (void* q : ps)
                if (q) (void)hipFree(q);
            if (sh.done) (void)hipEventDestroy(sh.done);
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
    for (int d = 0; d < n_shards; ++d) {
        KsShard& sh = S[d];
        sh.dev = d % ndev;
        std::vector<char> need(4 * nK, 0);
        for (int si = 0; si < 4; ++si)
            for (int K = sh.K0; K < sh.K1; ++K) {
                need[si * nK + K] = 1;  // own columns
                int kp = sl[si * nK + K].kp_idx;
                for (int sn = 0; sn < 4; ++sn) need[sn * nK + kp] = 1;
            }
        for (int c = 0; c < 4 * nK; ++c)
            if (need[c]) {
                sh.cols.push_back(c);
                int o = owner[c % nK];
                if (o != d) sh.remote.push_back({c, o});
            }
        KS_CHECK(hipSetDevice(sh.dev));
        KS_CHECK(hipStreamCreateWithFlags(&sh.st, hipStreamNonBlocking));
        KS_CHECK(hipEventCreateWithFlags(&sh.done, hipEventDisableTiming));
        KS_CHECK(hipMalloc((void**)&sh.kg, colb));
        KS_CHECK(hipMalloc((void**)&sh.P, sizeof Pr));
        KS_CHECK(hipMalloc((void**)&sh.V, nb));
        KS_CHECK(hipMalloc((void**)&sh.V2, nb));
        KS_CHECK(hipMalloc((void**)&sh.dV, nb));
        KS_CHECK(hipMalloc((void**)&sh.Vold, nb));
        KS_CHECK(hipMalloc((void**)&sh.kopt, nb));
        KS_CHECK(hipMalloc((void**)&sh.seg, n * sizeof(int)));
        KS_CHECK(hipMalloc((void**)&sh.dcols, sh.cols.size() * sizeof(int) + 4));
        KS_CHECK(hipMalloc((void**)&sh.sl, sl.size() * sizeof(KsSlice)));
        KS_CHECK(hipMalloc((void**)&sh.slots, 2 * kDiffSlots * sizeof(unsigned long long)));
        KS_CHECK(hipMemcpyAsync(sh.kg, k_grid, colb, hipMemcpyHostToDevice, sh.st));
        KS_CHECK(hipMemcpyAsync(sh.P, Pr, sizeof Pr, hipMemcpyHostToDevice, sh.st));
        KS_CHECK(hipMemcpyAsync(sh.V, value, nb, hipMemcpyHostToDevice, sh.st));
        KS_CHECK(hipMemcpyAsync(sh.V2, value, nb, hipMemcpyHostToDevice, sh.st));
        KS_CHECK(hipMemcpyAsync(sh.kopt, k_opt, nb, hipMemcpyHostToDevice, sh.st));
        KS_CHECK(hipMemcpyAsync(sh.dcols, sh.cols.data(), sh.cols.size() * sizeof(int),
                                hipMemcpyHostToDevice, sh.st));
        KS_CHECK(hipMemcpyAsync(sh.sl, sl.data(), sl.size() * sizeof(KsSlice), hipMemcpyHostToDevice, sh.st));
        KS_CHECK(hipStreamSynchronize(sh.st));
    }
    auto args = [&](KsShard& sh, int si) {
        KsArgs A{};
        A.nk = (int)nk; A.nK = (int)nK;
        A.node0 = (int)((si * nK + sh.K0) * nk);
        A.n_local = (int)((sh.K1 - sh.K0) * nk);
        A.k_grid = sh.kg; A.P = sh.P; A.slice = sh.sl;
        A.beta = p.beta; A.k_min = p.k_min; A.k_max = p.k_max;
        A.seg_hint = sh.seg;
        return A;
    };
    // the four s blocks of a shard in one launch each (blockIdx.y = s)
    auto args4 = [&](KsShard& sh) {
        KsArgs A = args(sh, 0);
        A.ns = 4;
        A.sstride = (int)(nK * nk);
        return A;
    };
    // peer copies of the columns each shard reads from others (after all shards finished)
    auto exchange = [&]() -> int {
        for (auto& sh : S) {
            KS_CHECK(hipSetDevice(sh.dev));
            KS_CHECK(hipEventRecord(sh.done, sh.st));
        }
        for (auto& sh : S) {
            KS_CHECK(hipSetDevice(sh.dev));
            for (auto& o : S)
                if (&o != &sh) KS_CHECK(hipStreamWaitEvent(sh.st, o.done, 0));
            for (auto& rc2 : sh.remote) {
                KsShard& o = S[rc2.second];
                size_t off = (size_t)rc2.first * nk;
                if (o.dev == sh.dev)
                    KS_CHECK(hipMemcpyAsync(sh.V + off, o.V + off, colb, hipMemcpyDeviceToDevice, sh.st));
                else
                    KS_CHECK(hipMemcpyPeerAsync(sh.V + off, sh.dev, o.V + off, o.dev, colb, sh.st));
            }
        }
        // nobody may overwrite its V (next sweep) before every reader has copied from it
        for (auto& sh : S) {
            KS_CHECK(hipSetDevice(sh.dev));
            KS_CHECK(hipEventRecord(sh.done, sh.st));
        }
        for (auto& sh : S) {
            KS_CHECK(hipSetDevice(sh.dev));
            for (auto& o : S)
                if (&o != &sh) KS_CHECK(hipStreamWaitEvent(sh.st, o.done, 0));
        }
        return AIY_OK;
    };
    double rel = NAN;
    int64_t it;
    for (it = 1; it <= max_vfi; ++it) {
        for (auto& sh : S) {
            KS_CHECK(hipSetDevice(sh.dev));
            KS_CHECK(hipMemcpyAsync(sh.Vold, sh.V, nb, hipMemcpyDeviceToDevice, sh.st));
            if ((it - 1) % 5 == 0) {
                KsArgs A0 = args(sh, 0);
                KS_TRY(launch_ks_slopes_cols(A0, sh.dcols, (int)sh.cols.size(), sh.V, sh.dV, sh.st));
                KS_TRY(launch_ks_improve(args4(sh), sh.V, sh.dV, sh.kopt, nullptr, sh.st));
            }
        }
        for (int64_t h = 0; h < howard_steps; ++h) {
            for (auto& sh : S) {
                KS_CHECK(hipSetDevice(sh.dev));
                KsArgs A0 = args(sh, 0);
                KS_TRY(launch_ks_slopes_cols(A0, sh.dcols, (int)sh.cols.size(), sh.V, sh.dV, sh.st));
                KS_TRY(launch_ks_howard(args4(sh), sh.V, sh.dV, sh.kopt, sh.V2, sh.st));
                std::swap(sh.V, sh.V2);
            }
            KS_TRY(exchange());
        }
        double m = NAN;
        for (auto& sh : S) {
            KS_CHECK(hipSetDevice(sh.dev));
            KS_CHECK(hipMemsetAsync(sh.slots, 0, 2 * kDiffSlots * sizeof(unsigned long long), sh.st));
            KS_TRY(launch_ks_reldiff(args4(sh), sh.V, sh.Vold, sh.slots, sh.st));
        }
        for (auto& sh : S) {
            KS_CHECK(hipSetDevice(sh.dev));
            std::vector<unsigned long long> h(2 * kDiffSlots);
            KS_CHECK(hipMemcpyAsync(h.data(), sh.slots, h.size() * 8, hipMemcpyDeviceToHost, sh.st));
            KS_CHECK(hipStreamSynchronize(sh.st));
            double d = fold_slots_host(h.data());
            if (d == d && !(m >= d)) m = d;
        }
        rel = m;
        if (rel < tol) break;
    }
    if (it > max_vfi) it = max_vfi;
    for (auto& sh : S) {
        KS_CHECK(hipSetDevice(sh.dev));
        for (int si = 0; si < 4; ++si) {
            size_t off = (size_t)(si * nK + sh.K0) * nk, cnt = (size_t)(sh.K1 - sh.K0) * nk;
            KS_CHECK(hipMemcpyAsync(value + off, sh.V + off, cnt * 8, hipMemcpyDeviceToHost, sh.st));
            KS_CHECK(hipMemcpyAsync(k_opt + off, sh.kopt + off, cnt * 8, hipMemcpyDeviceToHost, sh.st));
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

int ks_vfi_solve_multi(double* value, double* k_opt, const double* k_grid, const double* K_grid,
                       const double* B, const double* P, const double* params, int64_t nk,
                       int64_t nK, int64_t howard_steps, double tol, int64_t max_vfi,
                       int n_devices, int64_t* iters, double* rel_diff) {
    std::lock_guard<std::mutex> lk(host_mutex());
    int cur = 0;
    (void)hipGetDevice(&cur);
    int rc = ks_vfi_solve_multi_impl(value, k_opt, k_grid, K_grid, B, P, params, nk, nK,
                                     howard_steps, tol, max_vfi, n_devices, iters, rel_diff);
    (void)hipSetDevice(cur);
    return rc;
}

}  // namespace aiy

using namespace aiy;

extern "C" {

int ks_policy_improve(const double* value, const double* k_grid, const double* K_grid,
                      const double* B, const double* P, const double* params, int64_t nk,
                      int64_t nK, double* k_opt, int32_t* nfev) {
    if (!k_opt) return fail(AIY_BAD_ARG, "NULL k_opt");
    std::lock_guard<std::mutex> lk(host_mutex());
    HostCtx* c;
    AIY_TRY(get_ctx(4 * nK, nk, 1, &c));
    KsArgs A;
    KsDev D;
    AIY_TRY(ks_stage(c, value, nullptr, k_grid, K_grid, B, P, params, nk, nK, A, D));
    AIY_TRY(launch_ks_slopes(A, D.V, D.dV, c->st));
    AIY_TRY(launch_ks_improve(A, D.V, D.dV, D.kopt, D.nfev, c->st));
    size_t n = (size_t)nk * nK * 4;
    AIY_HIP(hipMemcpyAsync(k_opt, D.kopt, n * sizeof(double), hipMemcpyDeviceToHost, c->st));
    if (nfev) AIY_HIP(hipMemcpyAsync(nfev, D.nfev, n * sizeof(int), hipMemcpyDeviceToHost, c->st));
    AIY_HIP(hipStreamSynchronize(c->st));
    return AIY_OK;
}

int ks_howard(double* value, const double* k_opt, const double* k_grid, const double* K_grid,
              const double* B, const double* P, const double* params, int64_t nk, int64_t nK,
              int64_t steps) {
    if (!k_opt) return fail(AIY_BAD_ARG, "NULL k_opt");
    std::lock_guard<std::mutex> lk(host_mutex());
    HostCtx* c;
    AIY_TRY(get_ctx(4 * nK, nk, 1, &c));
    KsArgs A;
    KsDev D;
    AIY_TRY(ks_stage(c, value, k_opt, k_grid, K_grid, B, P, params, nk, nK, A, D));
    double* cur = D.V;
    double* nxt = D.V2;
    for (int64_t h = 0; h < steps; ++h) {
        AIY_TRY(launch_ks_slopes(A, cur, D.dV, c->st));
        AIY_TRY(launch_ks_howard(A, cur, D.dV, D.kopt, nxt, c->st));
        std::swap(cur, nxt);
    }
    size_t n = (size_t)nk * nK * 4;
    AIY_HIP(hipMemcpyAsync(value, cur, n * sizeof(double), hipMemcpyDeviceToHost, c->st));
    AIY_HIP(hipStreamSynchronize(c->st));
    return AIY_OK;
}

int ks_vfi_solve(double* value, double* k_opt, const double* k_grid, const double* K_grid,
                 const double* B, const double* P, const double* params, int64_t nk,
                 int64_t nK, int64_t howard_steps, double tol, int64_t max_vfi, int n_devices,
                 int64_t* iters, double* rel_diff) {
    if (!k_opt || !iters || !rel_diff) return fail(AIY_BAD_ARG, "NULL argument");
    if (max_vfi < 1 || howard_steps < 0) return fail(AIY_BAD_ARG, "max_vfi >= 1, howard_steps >= 0");
    // the checks ks_stage makes, before the multi-device branch (which does not stage)
    if (!value || !k_grid || !K_grid || !B || !P || !params) return fail(AIY_BAD_ARG, "NULL argument");
    if (nk < 3 || nK < 1) return fail(AIY_BAD_SHAPE, "need k_size >= 3 and K_size >= 1");
    if (n_devices > 1) return ks_vfi_solve_multi(value, k_opt, k_grid, K_grid, B, P, params, nk,
                                                 nK, howard_steps, tol, max_vfi, n_devices,
                                                 iters, rel_diff);
    std::lock_guard<std::mutex> lk(host_mutex());
    HostCtx* c;
    AIY_TRY(get_ctx(4 * nK, nk, 1, &c));
    KsArgs A;
    KsDev D;
    AIY_TRY(ks_stage(c, value, k_opt, k_grid, K_grid, B, P, params, nk, nK, A, D));
    A.howard = (int)howard_steps;
    A.max_vfi = (int)max_vfi;
    A.tol = tol;
    size_t n = (size_t)nk * nK * 4;
    if (ks_fused_fits((int)nk, (int)nK)) {
        AIY_TRY(launch_ks_fused(A, D.V, D.kopt, nullptr, D.out, c->st));
        KsOut o;
        AIY_HIP(hipMemcpyAsync(&o, D.out, sizeof o, hipMemcpyDeviceToHost, c->st));
        AIY_HIP(hipMemcpyAsync(value, D.V, n * sizeof(double), hipMemcpyDeviceToHost, c->st));
        AIY_HIP(hipMemcpyAsync(k_opt, D.kopt, n * sizeof(double), hipMemcpyDeviceToHost, c->st));
        AIY_HIP(hipStreamSynchronize(c->st));
        *iters = o.iters;
        *rel_diff = o.rel;
        return AIY_OK;
    }
    double* cur = D.V;
    double* nxt = D.V2;
    double rel = NAN;
    int64_t it;
    for (it = 1; it <= max_vfi; ++it) {
        AIY_HIP(hipMemcpyAsync(D.Vold, cur, n * sizeof(double), hipMemcpyDeviceToDevice, c->st));
        if ((it - 1) % 5 == 0) {
            AIY_TRY(launch_ks_slopes(A, cur, D.dV, c->st));
            AIY_TRY(launch_ks_improve(A, cur, D.dV, D.kopt, nullptr, c->st));
        }
        for (int64_t h = 0; h < howard_steps; ++h) {
            AIY_TRY(launch_ks_slopes(A, cur, D.dV, c->st));
            AIY_TRY(launch_ks_howard(A, cur, D.dV, D.kopt, nxt, c->st));
            std::swap(cur, nxt);
        }
        AIY_HIP(hipMemsetAsync(D.slots, 0, 2 * kDiffSlots * sizeof(unsigned long long), c->st));
        AIY_TRY(launch_ks_reldiff(A, cur, D.Vold, D.slots, c->st));
        AIY_TRY(ks_read_slots(c, D.slots, &rel));
        if (rel < tol) break;
    }
    if (it > max_vfi) it = max_vfi;
    AIY_HIP(hipMemcpyAsync(value, cur, n * sizeof(double), hipMemcpyDeviceToHost, c->st));
    AIY_HIP(hipMemcpyAsync(k_opt, D.kopt, n * sizeof(double), hipMemcpyDeviceToHost, c->st));
    AIY_HIP(hipStreamSynchronize(c->st));
    *iters = it;
    *rel_diff = rel;
    return AIY_OK;
}

}  // extern "C"
