// Device tier of the Krusell-Smith VFI (A6/A7) for one process per GPU: a handle owns one
// shard — the K range [K0, K1) of all four s, or of one z's two s ((K, Z) slices, so the
// reference's K = 4 grid spreads over 8 ranks) — and runs the improvement, Howard and
// relative-difference kernels on it, reading full k x K x S arrays already in HBM — or, on
// the direct schedule, the forecast columns through a table of pointers into the owners'
// buffers (ks_dev_set_columns).  The caller (aiyagari-replication_amd/ks_dist.py, or
// ks_multi_host.cpp for one process) moves halos / ghost blocks between shards or, on the
// direct schedule, only orders the sweeps.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "aiy_common.hpp"
#include "host_ctx.hpp"
#include "ks.hpp"
#include "ws.hpp"

struct ks_dev {
    int dev = 0;
    int nk = 0, nK = 0, K0 = 0, K1 = 0;
    int s0 = 0, s1 = 4;  // owned s blocks [s0, s1): all four, or one z's pair ((K, Z) slices)
    double beta = 0, k_min = 0, k_max = 0;
    double* kg = nullptr;
    double* kgt = nullptr;  // the grid's slope tables (launch_ks_grid_tables), 3·nk doubles
    double* P = nullptr;
    aiy::KsSlice* sl = nullptr;
    double* dV = nullptr;
    int* cols = nullptr;   // value columns (s*nK + K) this shard reads: own and K'_idx targets
    int ncols = 0;
    unsigned long long* slots = nullptr;
    int* seg = nullptr;    // [node] segment hints: improve writes them, Howard checks and uses them
    ks_dev* seg_owner = nullptr;  // set: seg is that handle's array (ks_dev_share_hints)
    int sharers = 0;              // handles using this handle's seg array
    int* own_cols = nullptr;      // the shard's own columns (direct schedule: its slopes)
    int n_own = 0;
    // direct schedule (ks_dev_set_columns): device table of 4·nK value then 4·nK slope column
    // pointers into the owners' buffers; null = the caller's full arrays
    const double* const* colV = nullptr;
    // staged direct schedule (ks_dev_set_split): own columns whose four forecast columns are all
    // owned (interior) and the rest (boundary), device lists
    int* cols_int = nullptr;
    int* cols_bnd = nullptr;
    int n_int = 0, n_bnd = 0;
    // staged sweeps: the copy blocks' arrival counter (device; [1]: the launch's go word) and
    // its running total (host)
    unsigned long long* copy_cnt = nullptr;
    unsigned long long copy_total = 0;
    unsigned long long launches = 0;  // staged launches so far (the go word's tokens)
};

namespace aiy {
// the shard's nodes: K in [K0, K1) of every owned s, the s blocks as blockIdx.y of one launch
static KsArgs shard_args(const ks_dev* h) {
    KsArgs A{};
    A.nk = h->nk;
    A.nK = h->nK;
    A.node0 = (h->s0 * h->nK + h->K0) * h->nk;
    A.n_local = (h->K1 - h->K0) * h->nk;
    A.ns = h->s1 - h->s0;
    A.sstride = h->nK * h->nk;
    A.k_grid = h->kg;
    A.kg_tab = h->kgt;
    A.P = h->P;
    A.slice = h->sl;
    A.beta = h->beta;
    A.k_min = h->k_min;
    A.k_max = h->k_max;
    A.seg_hint = h->seg;
    A.colV = h->colV;
    A.coldV = h->colV ? h->colV + 4 * h->nK : nullptr;
    return A;
}
}  // namespace aiy

using namespace aiy;

extern "C" {

int ks_dev_destroy(ks_dev* h) {
    if (!h) return AIY_OK;
    if (h->sharers > 0)
        return fail(AIY_BAD_ARG, "ks_dev_destroy: %d handle(s) still share this handle's hints; "
                    "destroy them first", h->sharers);
    if (h->seg_owner) h->seg_owner->sharers--;
    void* ps[] = {h->kg, h->kgt, h->P, h->sl, h->dV, h->cols, h->own_cols, h->slots,
                  h->seg_owner ? nullptr : h->seg, h->cols_int, h->cols_bnd, h->copy_cnt};
    for (void* q : ps)
        if (q) (void)hipFree(q);
    delete h;
    return AIY_OK;
}

int ks_dev_create(const double* k_grid, const double* K_grid, const double* B, const double* P,
                  const double* params, int64_t nk, int64_t nK, int64_t K0, int64_t K1,
                  ks_dev** out) {
    return ks_dev_create_slice(k_grid, K_grid, B, P, params, nk, nK, K0, K1, 0, 4, out);
}

int ks_dev_create_slice(const double* k_grid, const double* K_grid, const double* B,
                        const double* P, const double* params, int64_t nk, int64_t nK,
                        int64_t K0, int64_t K1, int64_t s0, int64_t s1, ks_dev** out) {
    if (!out || !k_grid || !K_grid || !B || !P || !params) return fail(AIY_BAD_ARG, "NULL argument");
    if (nk < 3 || nK < 1 || nk * nK * 4 > (1ll << 30))
        return fail(AIY_BAD_SHAPE, "need k_size >= 3, K_size >= 1");
    if (K0 < 0 || K1 > nK || K0 >= K1) return fail(AIY_BAD_ARG, "shard [K0, K1) must be inside [0, K_size)");
    if (s0 < 0 || s1 > 4 || s0 >= s1) return fail(AIY_BAD_ARG, "shard [s0, s1) must be inside [0, 4)");
    AIY_TRY(check_grid(k_grid, nk));
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return fail(AIY_NO_DEVICE, "no HIP device visible");
    KsParams p;
    memcpy(&p, params, sizeof p);
    std::vector<KsSlice> sl;
    ks_slices(p, B, K_grid, (int)nK, sl);
    std::vector<char> need(4 * nK, 0);
    for (int64_t s = s0; s < s1; ++s)
        for (int64_t K = K0; K < K1; ++K) {
            need[s * nK + K] = 1;
            const int kp = sl[s * nK + K].kp_idx;
            for (int sn = 0; sn < 4; ++sn) need[sn * nK + kp] = 1;
        }
    std::vector<int> cols, own;
    for (int c = 0; c < 4 * nK; ++c)
        if (need[c]) cols.push_back(c);
    for (int64_t s = s0; s < s1; ++s)
        for (int64_t K = K0; K < K1; ++K) own.push_back((int)(s * nK + K));
    double Pr[16];
    for (int i = 0; i < 4; ++i)
        for (int m = 0; m < 4; ++m) Pr[i * 4 + m] = P[i + m * 4];
    ks_dev* h = new ks_dev();
    (void)hipGetDevice(&h->dev);
    h->nk = (int)nk; h->nK = (int)nK; h->K0 = (int)K0; h->K1 = (int)K1;
    h->s0 = (int)s0; h->s1 = (int)s1;
    h->beta = p.beta; h->k_min = p.k_min; h->k_max = p.k_max;
    h->ncols = (int)cols.size();
    h->n_own = (int)own.size();
    const size_t n = (size_t)nk * nK * 4;
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = hipMalloc((void**)&h->kg, nk * sizeof(double));
    if (e == hipSuccess) e = hipMalloc((void**)&h->kgt, 3 * nk * sizeof(double));
    if (e == hipSuccess) e = hipMalloc((void**)&h->P, sizeof Pr);
    if (e == hipSuccess) e = hipMalloc((void**)&h->sl, sl.size() * sizeof(KsSlice));
    if (e == hipSuccess) e = hipMalloc((void**)&h->dV, n * sizeof(double));
    if (e == hipSuccess) e = hipMalloc((void**)&h->cols, cols.size() * sizeof(int));
    if (e == hipSuccess) e = hipMalloc((void**)&h->own_cols, own.size() * sizeof(int));
    if (e == hipSuccess) e = hipMalloc((void**)&h->slots, 2 * kDiffSlots * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMalloc((void**)&h->seg, n * sizeof(int));
    if (e == hipSuccess) e = hipMemset(h->seg, 0, n * sizeof(int));
    if (e == hipSuccess) e = hipMalloc((void**)&h->copy_cnt, 2 * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemset(h->copy_cnt, 0, 2 * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemcpy(h->kg, k_grid, nk * sizeof(double), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = launch_ks_grid_tables(h->kg, (int)nk, h->kgt, nullptr) == AIY_OK
                                 ? hipStreamSynchronize(nullptr) : hipErrorLaunchFailure;
    if (e == hipSuccess) e = hipMemcpy(h->P, Pr, sizeof Pr, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(h->sl, sl.data(), sl.size() * sizeof(KsSlice), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(h->cols, cols.data(), cols.size() * sizeof(int), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(h->own_cols, own.data(), own.size() * sizeof(int), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        ks_dev_destroy(h);
        return fail(AIY_HIP_ERROR, "ks_dev_create: %s", hipGetErrorString(e));
    }
    *out = h;
    return AIY_OK;
}

// Krusell_Smith_VFI.m:148-168 on the shard's nodes: slopes of the columns it reads, then
// fminbnd per node.  V: full k x K x S (device); kopt: full array, owned nodes written.
int ks_dev_improve(ks_dev* h, const double* V, double* kopt, void* stream) {
    if (!h || !V || !kopt) return fail(AIY_BAD_ARG, "NULL argument");
    hipStream_t st = (hipStream_t)stream;
    AIY_TRY(launch_ks_slopes_cols(shard_args(h), h->cols, h->ncols, V, h->dV, st));
    AIY_TRY(launch_ks_improve(shard_args(h), V, h->dV, kopt, nullptr, st));
    return AIY_OK;
}

// one Jacobi Howard sweep (:173-191) on the shard's nodes: slopes from V, owned nodes of Vout
int ks_dev_howard(ks_dev* h, const double* V, const double* kopt, double* Vout, void* stream) {
    if (!h || !V || !kopt || !Vout) return fail(AIY_BAD_ARG, "NULL argument");
    if (V == Vout) return fail(AIY_BAD_ARG, "Howard sweeps are Jacobi: V and Vout must differ");
    hipStream_t st = (hipStream_t)stream;
    AIY_TRY(launch_ks_slopes_cols(shard_args(h), h->cols, h->ncols, V, h->dV, st));
    AIY_TRY(launch_ks_howard(shard_args(h), V, h->dV, kopt, Vout, st));
    return AIY_OK;
}

// the pchip slopes of every column h's sweep reads (own columns and forecast targets) into
// the caller's dV (full k x K x S); what a fused sweep needs before its first launch
int ks_dev_slopes(ks_dev* h, const double* V, double* dV, void* stream) {
    if (!h || !V || !dV) return fail(AIY_BAD_ARG, "NULL argument");
    return launch_ks_slopes_cols(shard_args(h), h->cols, h->ncols, V, dV, (hipStream_t)stream);
}

// one Jacobi Howard sweep on h's nodes that also writes the next sweep's slopes: reads V and
// dV (slopes of V on every column h reads), writes Vout and dVout on h's nodes
int ks_dev_howard_fused(ks_dev* h, const double* V, const double* dV, const double* kopt,
                        double* Vout, double* dVout, void* stream) {
    if (!h || !V || !dV || !kopt || !Vout || !dVout) return fail(AIY_BAD_ARG, "NULL argument");
    if (V == Vout || dV == dVout)
        return fail(AIY_BAD_ARG, "Howard sweeps are Jacobi: V/Vout and dV/dVout must differ");
    return launch_ks_howard_slopes(shard_args(h), V, dV, kopt, Vout, dVout, (hipStream_t)stream);
}

// Direct (peer-read) schedule: every shard keeps the value and slopes of its OWN columns current
// in its own buffers; a sweep or improvement reads a forecast column wherever its owner keeps
// it (table: 4·nK value column pointers, then 4·nK slope column pointers, on this device or a
// peer's), so no column is ever copied.  table = NULL returns to the caller's full arrays.
int ks_dev_set_columns(ks_dev* h, const void* const* table) {
    if (!h) return fail(AIY_BAD_ARG, "NULL handle");
    h->colV = reinterpret_cast<const double* const*>(table);
    return AIY_OK;
}

// The staged direct schedule's split of the shard's own columns (c = s·nK + K): `interior`
// columns read only owned forecast columns, `boundary` columns read at least one a peer owns
// (through the local halo copy).  Every own column must be in exactly one list.
int ks_dev_set_split(ks_dev* h, const int32_t* interior, int32_t n_int, const int32_t* boundary,
                     int32_t n_bnd) {
    if (!h || n_int < 0 || n_bnd < 0 || (n_int && !interior) || (n_bnd && !boundary))
        return fail(AIY_BAD_ARG, "bad argument");
    if (n_int + n_bnd != h->n_own)
        return fail(AIY_BAD_ARG, "ks_dev_set_split: %d + %d columns, the shard owns %d", n_int,
                    n_bnd, h->n_own);
    std::vector<char> seen(4 * h->nK, 0);
    for (int i = 0; i < n_int + n_bnd; ++i) {
        const int c = i < n_int ? interior[i] : boundary[i - n_int];
        const int s = c / h->nK, K = c % h->nK;
        if (c < 0 || c >= 4 * h->nK || s < h->s0 || s >= h->s1 || K < h->K0 || K >= h->K1 || seen[c])
            return fail(AIY_BAD_ARG, "ks_dev_set_split: column %d is not an own column (or repeats)", c);
        seen[c] = 1;
    }
    for (int** q : {&h->cols_int, &h->cols_bnd})
        if (*q) {
            AIY_HIP(hipFree(*q));
            *q = nullptr;
        }
    if (n_int) {
        AIY_HIP(hipMalloc((void**)&h->cols_int, n_int * sizeof(int)));
        AIY_HIP(hipMemcpy(h->cols_int, interior, n_int * sizeof(int), hipMemcpyHostToDevice));
    }
    if (n_bnd) {
        AIY_HIP(hipMalloc((void**)&h->cols_bnd, n_bnd * sizeof(int)));
        AIY_HIP(hipMemcpy(h->cols_bnd, boundary, n_bnd * sizeof(int), hipMemcpyHostToDevice));
    }
    h->n_int = n_int;
    h->n_bnd = n_bnd;
    return AIY_OK;
}

// the fused Howard sweep over one subset of the own columns (0 = interior, 1 = boundary)
int ks_dev_howard_fused_part(ks_dev* h, int part, const double* V, const double* dV,
                             const double* kopt, double* Vout, double* dVout, void* stream) {
    if (!h || !V || !dV || !kopt || !Vout || !dVout || (part & ~1))
        return fail(AIY_BAD_ARG, "bad argument");
    if (V == Vout || dV == dVout)
        return fail(AIY_BAD_ARG, "Howard sweeps are Jacobi: V/Vout and dV/dVout must differ");
    if (h->n_int + h->n_bnd == 0)  // no split set: part 0 is the whole shard, part 1 nothing
        return part ? AIY_OK : ks_dev_howard_fused(h, V, dV, kopt, Vout, dVout, stream);
    KsArgs A = shard_args(h);
    A.col_list = part ? h->cols_bnd : h->cols_int;
    A.n_list = part ? h->n_bnd : h->n_int;
    return launch_ks_staged_sweep(A, V, dV, kopt, Vout, dVout, (hipStream_t)stream);
}

// The staged direct schedule's whole sweep in ONE launch (ks_staged_sweep_kernel): publish
// pub_v in slot `slot` of `flags` first (the previous launch on the stream produced it), copy
// the n_halo peer columns src[q] -> dst[q] (device pointer arrays) once the slots in `mask` hold
// >= wait_v, sweep the interior columns meanwhile and the boundary columns after the copies.
// flags = NULL: no publish and no wait (one process; the tests' single-launch checks).
int ks_dev_staged_sweep(ks_dev* h, const double* V, const double* dV, const double* kopt,
                        double* Vout, double* dVout, const void* const* src, void* const* dst,
                        int32_t n_halo, void* flags, uint64_t mask, uint64_t wait_v, int32_t slot,
                        uint64_t pub_v, double timeout_s, void* err, void* stream) {
    if (!h || !V || !dV || !kopt || !Vout || !dVout || n_halo < 0 || (n_halo && (!src || !dst)) ||
        (flags && (!err || !(timeout_s > 0) || slot < 0 || slot >= 64)))
        return fail(AIY_BAD_ARG, "bad argument");
    if (V == Vout || dV == dVout)
        return fail(AIY_BAD_ARG, "Howard sweeps are Jacobi: V/Vout and dV/dVout must differ");
    if (h->n_int + h->n_bnd == 0) return fail(AIY_BAD_ARG, "staged sweeps need ks_dev_set_split");
    if (n_halo && !h->n_bnd)
        return fail(AIY_BAD_ARG, "halo columns without boundary columns (ks_dev_set_split)");
    KsArgs A = shard_args(h);
    // empty lists are fine here (the rows are counted, not inferred from a null pointer): a
    // shard with no interior column is all copy and boundary rows (the r05 g37 case)
    A.col_list = h->cols_int;
    A.n_list = h->n_int;
    A.bnd_list = h->cols_bnd;
    A.n_bnd = h->n_bnd;
    A.halo_src = reinterpret_cast<const double* const*>(src);
    A.halo_dst = reinterpret_cast<double* const*>(dst);
    A.n_halo = n_halo;
    const bool waits = flags && mask;
    A.n_copy_rows = n_halo ? n_halo : (waits ? 1 : 0);
    A.copy_x = n_halo ? ks_staged_copy_blocks(h->nk) : 1;
    if (waits) {
        A.wait_flags = (const unsigned long long*)flags;
        A.wait_mask = mask;
        A.wait_v = wait_v;
        A.timeout_ticks = (long long)(timeout_s * 1e8);
        A.err = (unsigned long long*)err;
    }
    if (flags) {
        A.pub_flag = (unsigned long long*)flags + (size_t)slot * 16;
        A.pub_v = pub_v;
    }
    A.copy_cnt = h->copy_cnt;
    A.go = h->copy_cnt + 1;
    A.go_token = h->launches + 1;
    const unsigned long long add = (unsigned long long)n_halo * (unsigned long long)A.copy_x;
    A.copy_target = h->copy_total + add;
    AIY_TRY(launch_ks_staged_sweep(A, V, dV, kopt, Vout, dVout, (hipStream_t)stream));
    h->copy_total += add;
    h->launches += 1;
    return AIY_OK;
}

// the slopes of the shard's own columns of V into dV (the start of a direct schedule)
int ks_dev_slopes_own(ks_dev* h, const double* V, double* dV, void* stream) {
    if (!h || !V || !dV) return fail(AIY_BAD_ARG, "NULL argument");
    return launch_ks_slopes_cols(shard_args(h), h->own_cols, h->n_own, V, dV,
                                 (hipStream_t)stream);
}

// the improvement of the direct schedule: fminbnd on the shard's nodes, every forecast column
// (value and slopes) read through the table — the owners' slopes are current, so no slope launch
int ks_dev_improve_direct(ks_dev* h, double* kopt, void* stream) {
    if (!h || !kopt) return fail(AIY_BAD_ARG, "NULL argument");
    if (!h->colV) return fail(AIY_BAD_ARG, "ks_dev_improve_direct: no column table (ks_dev_set_columns)");
    const KsArgs A = shard_args(h);
    return launch_ks_improve(A, nullptr, nullptr, kopt, nullptr, (hipStream_t)stream);
}

// max over the shard's nodes of |V - Vold| / (|Vold| + 1e-10), NaN ignored (:195).
// out (device, 2 x uint64): {IEEE bits of the max, nonzero if any node was not NaN}
int ks_dev_reldiff(ks_dev* h, const double* V, const double* Vold, void* out, void* stream) {
    if (!h || !V || !Vold || !out) return fail(AIY_BAD_ARG, "NULL argument");
    hipStream_t st = (hipStream_t)stream;
    AIY_HIP(hipMemsetAsync(h->slots, 0, 2 * kDiffSlots * sizeof(unsigned long long), st));
    AIY_TRY(launch_ks_reldiff(shard_args(h), V, Vold, h->slots, st));
    AIY_TRY(launch_reduce_slots(h->slots, out, st));
    return AIY_OK;
}

// Ghost shards (ks_dist.py, exchanges every m Howard sweeps): h reads and writes the segment
// hints of `owner` (same grid), so the hints improve stores for the owner's nodes serve h's
// sweeps over those nodes too.  owner must outlive h.
int ks_dev_share_hints(ks_dev* h, ks_dev* owner) {
    if (!h || !owner) return fail(AIY_BAD_ARG, "NULL argument");
    if (h == owner) return AIY_OK;
    if (owner->seg_owner) return fail(AIY_BAD_ARG, "owner shares another handle's hints");
    if (h->nk != owner->nk || h->nK != owner->nK || h->dev != owner->dev)
        return fail(AIY_BAD_SHAPE, "ks_dev_share_hints: handles of different grids or devices");
    if (h->sharers > 0) return fail(AIY_BAD_ARG, "other handles share h's hints");
    if (h->seg_owner == owner) return AIY_OK;
    if (h->seg_owner) h->seg_owner->sharers--;
    else AIY_HIP(hipFree(h->seg));
    h->seg = owner->seg;
    h->seg_owner = owner;
    owner->sharers++;
    return AIY_OK;
}

// the segment hints of h's nodes from kopt (nodes whose k_opt another rank computed); a
// hint only short-cuts Howard's search, so results never depend on it
int ks_dev_hints(ks_dev* h, const double* kopt, void* stream) {
    if (!h || !kopt) return fail(AIY_BAD_ARG, "NULL argument");
    AIY_TRY(launch_ks_hints(shard_args(h), kopt, (hipStream_t)stream));
    return AIY_OK;
}

int ks_forecast_index(const double* K_grid, const double* B, const double* params, int64_t nK,
                      int32_t* out) {
    if (!K_grid || !B || !params || !out) return fail(AIY_BAD_ARG, "NULL argument");
    if (nK < 1 || nK > (1 << 24)) return fail(AIY_BAD_SHAPE, "need 1 <= K_size");
    KsParams p;
    memcpy(&p, params, sizeof p);
    std::vector<KsSlice> sl;
    ks_slices(p, B, K_grid, (int)nK, sl);
    for (size_t c = 0; c < sl.size(); ++c) out[c] = sl[c].kp_idx;
    return AIY_OK;
}

}  // extern "C"
