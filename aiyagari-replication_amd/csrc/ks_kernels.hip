// A6/A7 — Krusell-Smith VFI on gfx950 (Krusell_Smith_VFI.m:143-204; bellman_value :329-364).
//
// Node = (k_i, K_i, s_i); value/k_opt are k x K x S column-major (node n = (s*K + Ki)*nk + ki).
// Everything that depends only on the slice (K_i, s_i) — the ALM forecast K' and its nearest
// grid index, the prices r, w at the (flipped, :332) current z, the budget coefficients — is
// computed on the host (libm) once per B and passed as a KsSlice table.  Per node:
//   bellman(kp) = log(max((a1·k + a2) − kp, 1e-10)) + β Σ_s' P(s,s')·pchip_{K',s'}(clamp(kp))
// with pchip slopes (Fritsch–Butland, MATLAB end rules) rebuilt from the current value after
// every Howard sweep (the .Values refresh at :186-191) and evaluated in MATLAB's pwch/ppval form.
//   improve  fminbnd(−bellman, k_min, min(res, k_max)) per node — MATLAB's Brent/FMM with
//            seps = sqrt(eps), TolX = 1e-4, MaxFunEvals = MaxIter = 500 (:157-167)
//   howard   Jacobi: value_new(n) = bellman_n(k_opt(n)) from the previous sweep's value
// log is aiy_log (fdlibm, identical on host and device), so fminbnd's value-dependent branches
// take the same path as in the C oracle: k_opt and value are bit-exact.
//
// Two execution shapes:
//   fused    one workgroup holds the whole problem in LDS (reference size: 1,600 nodes) and runs
//            the complete VFI loop — improvement every 5th iteration, H Howard sweeps, the
//            relative-difference stop (:195-203) — in ONE launch (barriers between phases).
//   tiled    slopes / improve / howard / reldiff as separate grid-wide kernels (any size).
#include <algorithm>

#include "aiy_common.hpp"
#include "ks.hpp"
#include "ipc_dev.hpp"
#include "pchip_dev.hpp"

namespace aiy {


struct KsView {  // where the value/slope columns and the grid live (LDS or global)
    const double* kg;
    const double* V;
    const double* dV;
};

// seg_of_dev(x, n, q) given a guess g: the guess is accepted only where it is provably the
// search's answer (largest j <= n-2 with x[j] <= q, else 0; x non-decreasing), so a stale or
// garbage hint costs a search, never a different result.
__device__ __forceinline__ int seg_hinted_dev(const double* __restrict__ x, int n, double q,
                                              int g) {
    g = g < 0 ? 0 : (g > n - 2 ? n - 2 : g);
    const bool lo_ok = g == 0 || x[g] <= q;
    const bool hi_ok = g == n - 2 || q < x[g + 1];
    if (lo_ok && hi_ok && q == q) return g;
    return seg_of_dev(x, n, q);
}

// hint: a guess of the segment (verified); [slo, shi]: segments the answer provably lies in
// when the checks of seg_range_dev pass (fminbnd's bracket); seg_out: the segment used
template <bool SC1 = false>
__device__ __forceinline__ double ks_bellman_dev(const KsArgs& A, const KsView& W,
                                                 const KsSlice& sl, int si, double k, double kp,
                                                 int hint = -1, int slo = -1, int shi = -1,
                                                 int* seg_out = nullptr) {
    const int nk = A.nk;
    double kq = fmax(fmin(kp, W.kg[nk - 1]), W.kg[0]);
    int seg = hint >= 0 ? seg_hinted_dev(W.kg, nk, kq, hint)
                        : (slo >= 0 ? seg_range_dev(W.kg, nk, kq, slo, shi) : seg_of_dev(W.kg, nk, kq));
    if (seg_out) *seg_out = seg;
    double expec = 0;
    const double h = W.kg[seg + 1] - W.kg[seg], rh = 1.0 / h;  // the four queries' segment
#pragma unroll
    for (int sn = 0; sn < 4; ++sn) {
        const int c = sn * A.nK + sl.kp_idx;  // (slice-uniform: scalar loads of the table)
        const size_t col = (size_t)c * nk;
        const double* Vc = A.colV ? A.colV[c] : W.V + col;
        const double* dVc = A.colV ? A.coldV[c] : W.dV + col;
        expec = expec + A.P[si * 4 + sn] * pchip_at<SC1>(W.kg, Vc, dVc, seg, kq, h, rh);
    }
    double c = (sl.a1 * k + sl.a2) - kp;
    c = fmax(c, 1e-10);
    return aiy_log(c) + A.beta * expec;
}

// MATLAB fminbnd on −bellman over [ax, bx]
// Every evaluation after the first lies in the bracket [a, b] whose ends are evaluated points
// (or the interval's ends), so its segment is searched between theirs (sa, sb) — verified by
// seg_range_dev, so the segments, hence the values, are the full search's.
__device__ double ks_fminbnd_dev(const KsArgs& A, const KsView& W, const KsSlice& sl, int si,
                                 double k, double ax, double bx, int* nfev) {
    int sa = 0, sb = A.nk - 2, su = 0;
#define F(X) (-ks_bellman_dev(A, W, sl, si, k, (X), -1, sa, sb, &su))
    const double seps = 1.4901161193847656e-08;  // sqrt(eps)
    const double tolx = 1e-4;
    const double cg = 0.5 * (3.0 - 2.23606797749978969641);  // 0.5*(3 - sqrt(5))
    double a = ax, b = bx, v = a + cg * (b - a), w = v, xf = v, d = 0, e = 0, x = xf;
    double fx = F(x);
    int sxf = su;
    int num = 1, it = 0;
    double fv = fx, fw = fx, xm = 0.5 * (a + b);
    double tol1 = seps * fabs(xf) + tolx / 3.0, tol2 = 2.0 * tol1;
    while (fabs(xf - xm) > (tol2 - 0.5 * (b - a))) {
        int gs = 1;
        if (fabs(e) > tol1) {
            gs = 0;
            double r = (xf - w) * (fx - fv);
            double q = (xf - v) * (fx - fw);
            double pp = (xf - v) * q - (xf - w) * r;
            q = 2.0 * (q - r);
            if (q > 0.0) pp = -pp;
            q = fabs(q);
            r = e;
            e = d;
            if (fabs(pp) < fabs(0.5 * q * r) && pp > q * (a - xf) && pp < q * (b - xf)) {
                d = pp / q;
                x = xf + d;
                if ((x - a) < tol2 || (b - x) < tol2) {
                    double si2 = sgn_dev(xm - xf) + ((xm - xf) == 0);
                    d = tol1 * si2;
                }
            } else {
                gs = 1;
            }
        }
        if (gs) {
            e = (xf >= xm) ? (a - xf) : (b - xf);
            d = cg * e;
        }
        double si2 = sgn_dev(d) + (d == 0);
        x = xf + si2 * fmax(fabs(d), tol1);
        double fu = F(x);
        ++num;
        ++it;
        if (fu <= fx) {
            if (x >= xf) a = xf, sa = sxf;
            else b = xf, sb = sxf;
            v = w; fv = fw;
            w = xf; fw = fx;
            xf = x; fx = fu; sxf = su;
        } else {
            if (x < xf) a = x, sa = su;
            else b = x, sb = su;
            if (fu <= fw || w == xf) {
                v = w; fv = fw;
                w = x; fw = fu;
            } else if (fu <= fv || v == xf || v == w) {
                v = x; fv = fu;
            }
        }
        xm = 0.5 * (a + b);
        tol1 = seps * fabs(xf) + tolx / 3.0;
        tol2 = 2.0 * tol1;
        if (num >= 500 || it >= 500) break;
    }
    *nfev = num;
    return xf;
#undef F
}

__device__ __forceinline__ void node_coords(const KsArgs& A, int n, int& ki, int& Ki, int& si) {
    ki = n % A.nk;
    int r = n / A.nk;
    Ki = r % A.nK;
    si = r / A.nK;
}

__device__ __forceinline__ double improve_node(const KsArgs& A, const KsView& W, int n,
                                               int* nfev) {
    int ki, Ki, si;
    node_coords(A, n, ki, Ki, si);
    const KsSlice sl = A.slice[si * A.nK + Ki];
    double k = W.kg[ki];
    double res = sl.b1 * k + sl.b2;                 // :152-153
    double kpmax = fmin(res, A.k_max);              // :159
    return ks_fminbnd_dev(A, W, sl, si, k, A.k_min, kpmax, nfev);  // :164
}

__device__ __forceinline__ double howard_node(const KsArgs& A, const KsView& W, int n,
                                              double kp) {
    int ki, Ki, si;
    node_coords(A, n, ki, Ki, si);
    const KsSlice sl = A.slice[si * A.nK + Ki];
    return ks_bellman_dev(A, W, sl, si, W.kg[ki], kp, A.seg_hint ? A.seg_hint[n] : -1);
}

// ------------------------------------------------------------------------------ tiled
// Column-shaped launches (x: k tile, y: column, grid-stride): a node's column and row come from
// the block indices, not from integer divisions of a flat node index per thread.
__device__ __forceinline__ int ks_tile_k() { return blockIdx.x * blockDim.x + threadIdx.x; }

__global__ void ks_slopes_kernel(KsArgs A, const double* __restrict__ V, double* __restrict__ dV) {
    const int q = ks_tile_k();
    if (q >= A.nk) return;
    for (int c = blockIdx.y; c < 4 * A.nK; c += gridDim.y) {
        const size_t col = (size_t)c * A.nk;
        dV[col + q] = A.kg_tab ? pchip_slope_tab(A.k_grid, V + col, A.nk, q, A.kg_tab)
                               : pchip_slope(A.k_grid, V + col, A.nk, q);
    }
}

__global__ void ks_grid_tables_kernel(const double* __restrict__ kg, int nk, double* __restrict__ tab) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < nk) pchip_grid_tables(kg, nk, q, tab);
}

// slopes for a list of columns only (the columns a shard reads)
__global__ void ks_slopes_cols_kernel(KsArgs A, const int* __restrict__ cols, int ncols,
                                      const double* __restrict__ V, double* __restrict__ dV) {
    const int q = ks_tile_k();
    if (q >= A.nk) return;
    for (int c = blockIdx.y; c < ncols; c += gridDim.y) {
        const size_t col = (size_t)cols[c] * A.nk;
        dV[col + q] = A.kg_tab ? pchip_slope_tab(A.k_grid, V + col, A.nk, q, A.kg_tab)
                               : pchip_slope(A.k_grid, V + col, A.nk, q);
    }
}

__global__ void ks_improve_kernel(KsArgs A, const double* __restrict__ V,
                                  const double* __restrict__ dV, double* __restrict__ k_opt,
                                  int* __restrict__ nfev) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= A.n_local) return;
    int n = A.node0 + blockIdx.y * A.sstride + t;
    KsView W{A.k_grid, V, dV};
    int nf = 0;
    const double kp = improve_node(A, W, n, &nf);
    k_opt[n] = kp;
    if (nfev) nfev[n] = nf;
    if (A.seg_hint)  // the segment Howard's 50 sweeps will evaluate this k_opt in
        A.seg_hint[n] = seg_of_dev(A.k_grid, A.nk, fmax(fmin(kp, A.k_grid[A.nk - 1]), A.k_grid[0]));
}

// Howard sweep over the launch's columns: x = k tile, y = column of an s block (grid-stride),
// z = s block; node n = col·nk + ki with col = s·nK + K — the values of howard_node exactly
__global__ void ks_howard_kernel(KsArgs A, const double* __restrict__ V,
                                 const double* __restrict__ dV, const double* __restrict__ k_opt,
                                 double* __restrict__ Vn) {
    const int ki = ks_tile_k();
    if (ki >= A.nk) return;
    const int nk = A.nk;
    const int col0 = A.node0 / nk + (int)blockIdx.z * (A.sstride / nk);  // block-uniform
    const int ncl = A.n_local / nk;
    KsView W{A.k_grid, V, dV};
    const double k = W.kg[ki];
    for (int y = blockIdx.y; y < ncl; y += gridDim.y) {
        const int col = col0 + y;
        const int si = col / A.nK;
        const int n = col * nk + ki;
        const KsSlice sl = A.slice[col];
        Vn[n] = ks_bellman_dev(A, W, sl, si, k, k_opt[n], A.seg_hint ? A.seg_hint[n] : -1);
    }
}

// Copy of one halo column share: elements i0, i0 + step, ... < n from a peer's buffer (system-
// scope loads: served by the owner's memory) to this device.  Eight loads per thread in flight
// before the stores (global_ address space, so no flat instructions).
template <bool SC1 = false>
__device__ __forceinline__ void halo_copy_share(const double* src, double* dst, int i0, int step,
                                                int n) {
    using gu64 = __attribute__((address_space(1))) unsigned long long;
    const gu64* s = (const gu64*)(const void*)src;
    gu64* d = (gu64*)(void*)dst;
    for (int b = i0; b < n; b += 8 * step) {
        unsigned long long u[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int i = b + j * step;
            u[j] = i < n ? __hip_atomic_load(s + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0ull;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int i = b + j * step;
            if (i < n) {
                if constexpr (SC1)  // write-through: the in-kernel consumer reads it sc1
                    __hip_atomic_store(d + i, u[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else
                    d[i] = u[j];
            }
        }
    }
}

// Howard sweep + the NEXT sweep's pchip slopes in one launch (the .Values refresh of
// :186-191 fused into the sweep that produces the values).  A block owns O consecutive k
// nodes of a column and evaluates the sweep on [q0 − 2, q0 + O + 2) (the neighbours the
// slopes of its own nodes read, end rules included), stages those values in LDS and writes
// value and slope of its own nodes — the same formulas on the same values as
// ks_howard_kernel + ks_slopes_kernel, so bit for bit the two-launch sweep.  Columns of
// length <= blockDim are one block each (O = nk: nothing evaluated twice); longer columns
// evaluate 4 of every 256 nodes twice.
template <bool WT, bool SC1 = false>
__device__ __forceinline__ void howard_slopes_col(const KsArgs& A, const KsView& W, int col,
                                                  const double* __restrict__ k_opt,
                                                  double* __restrict__ Vn,
                                                  double* __restrict__ dVn, double* s_v, int O,
                                                  int tile = -1) {
    const int nk = A.nk;
    const int q0 = (tile >= 0 ? tile : (int)blockIdx.x) * O;
    const int lo = q0 >= 2 ? q0 - 2 : 0;
    const int own_hi = min(nk, q0 + O);
    const int hi = min(nk, q0 + O + 2);
    const int q = lo + (int)threadIdx.x;
    const bool comp = q < hi, mine = q >= q0 && q < own_hi;
    const double k = comp ? W.kg[q] : 0.0;
    const LdsCol yl{s_v, lo};
    const int si = col / A.nK;
    const size_t n = (size_t)col * nk + q;
    double v = 0.0;
    if (comp) {
        const KsSlice sl = A.slice[col];
        v = ks_bellman_dev<SC1>(A, W, sl, si, k, k_opt[n], A.seg_hint ? A.seg_hint[n] : -1);
    }
    s_v[threadIdx.x] = v;
    __syncthreads();
    if (mine) {
        const double d = A.kg_tab ? pchip_slope_tab(A.k_grid, yl, nk, q, A.kg_tab)
                                  : pchip_slope_t(A.k_grid, yl, nk, q);
        if (WT) {  // staged direct schedule: peers copy these columns once the next launch has
            // published — stored write-through (system-scope vector stores), so they are in
            // memory when this kernel ends
            __hip_atomic_store(reinterpret_cast<unsigned long long*>(Vn + n),
                               __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(reinterpret_cast<unsigned long long*>(dVn + n),
                               __builtin_bit_cast(unsigned long long, d), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        } else {
            Vn[n] = v;
            dVn[n] = d;
        }
    }
    __syncthreads();
}

// the node-range sweep (x: k tile, y: column of an s block, grid-stride; z: s block)
__global__ __launch_bounds__(256) void ks_howard_slopes_kernel(KsArgs A, const double* __restrict__ V,
                                                               const double* __restrict__ dV,
                                                               const double* __restrict__ k_opt,
                                                               double* __restrict__ Vn,
                                                               double* __restrict__ dVn, int O) {
    __shared__ double s_v[256];
    const int col0 = A.node0 / A.nk + (int)blockIdx.z * (A.sstride / A.nk);  // block-uniform
    const int ncl = A.n_local / A.nk;
    const KsView W{A.k_grid, V, dV};
    for (int y = blockIdx.y; y < ncl; y += gridDim.y)  // block-uniform trip count
        howard_slopes_col<false>(A, W, col0 + y, k_opt, Vn, dVn, s_v, O);
}

// The same sweep on a 1-D grid dealt by XCD (tile-major): blocks are dealt round-robin over the
// 8 XCDs (observed), so linear block L runs on XCD L mod 8; slot start_x + L / 8 of the
// sequence (tile mod 8, tile, column) is what it computes.  Every column's tile t then runs on
// the XCD that runs tile t of every other column, and the forecast segments those tiles read
// (near the tile's k range: k' ≈ k) are fetched into that XCD's L2 once, not once per XCD.
// Work order only: the same values.  gx tiles per column, C columns (s blocks × ncl).
__global__ __launch_bounds__(256) void ks_howard_slopes_xcd_kernel(KsArgs A,
                                                                   const double* __restrict__ V,
                                                                   const double* __restrict__ dV,
                                                                   const double* __restrict__ k_opt,
                                                                   double* __restrict__ Vn,
                                                                   double* __restrict__ dVn, int O,
                                                                   int gx, int C) {
    __shared__ double s_v[256];
    const int total = gx * C;
    const int L = blockIdx.x, x = L & 7, r = L >> 3;
    int start = 0;
    for (int q = 0; q < x; ++q) start += (total - q + 7) >> 3;
    int slot = start + r, g = 0;
    for (; g < 8; ++g) {  // residue group g: tiles g, g + 8, ... of every column
        const int tg = gx > g ? (gx - g + 7) >> 3 : 0;
        if (slot < tg * C) break;
        slot -= tg * C;
    }
    const int tile = g + 8 * (slot / C), cc = slot % C;
    const int ncl = A.n_local / A.nk;
    const int z = cc / ncl, y = cc - z * ncl;
    const int col = A.node0 / A.nk + z * (A.sstride / A.nk) + y;
    const KsView W{A.k_grid, V, dV};
    howard_slopes_col<false>(A, W, col, k_opt, Vn, dVn, s_v, O, tile);
}

// The staged direct schedule's sweep: ONE launch per sweep.
// Block rows, in dispatch order:
//   copy rows      [0, n_copy_rows): block (0, 0) waits (one wave) for the neighbours' slots
//                  >= wait_v in the host page — the versions this sweep reads — and passes that
//                  on through a device word (`go`); the other copy blocks poll the device word.
//                  Then each copies its share of halo column q from the owner's buffer (system-
//                  scope loads) with sc1 stores and adds 1 to copy_cnt (the guide's first-row
//                  hand-off: every storing wave waits for its stores, a barrier, one lane's
//                  agent-scope add).  With no halo but neighbours: one wait-only row.
//   interior rows  col_list: columns whose four forecast columns are all own — no wait at all.
//   boundary rows  bnd_list: thread 0 polls copy_cnt (sc1 loads) up to copy_target, a barrier,
//                  then the sweep reads every column with sc1 loads (no L1 line from an older
//                  halo can serve them).
// Block (0, 0) first publishes pub_v (the previous launch on the stream, which produced version
// pub_v, has completed; its write-through stores are in memory) with a system-scope release.
// Copy rows come first so that the copies start with the launch; boundary rows last, so a
// spinning boundary block never holds back the dispatch of a block it waits for (blocks of one
// XCD are dispatched in order; copy blocks wait only on other ranks) — and measured: boundary
// rows right after the copy rows spin while the copies run and hold slots the interior needs
// (one-GPU model, worst shard: 54.8 vs 30.9 us per sweep, profiles/r06_g03_ks_staged_probe.txt).  Write-after-read on the
// three buffers (ks_dev_direct_sweeps): a launch writes the buffer its neighbours read two
// versions ago, and they published that they had finished with it before this launch's
// predecessor's copy rows could pass their wait — so the interior rows need no wait.
constexpr int kCopyX = 16;  // working copy blocks per copy row (strided copy)
__global__ __launch_bounds__(256) void ks_staged_sweep_kernel(KsArgs A, const double* __restrict__ V,
                                                              const double* __restrict__ dV,
                                                              const double* __restrict__ k_opt,
                                                              double* __restrict__ Vn,
                                                              double* __restrict__ dVn, int O) {
    __shared__ double s_v[256];
    const int tid = threadIdx.x;
    const bool first = blockIdx.x == 0 && blockIdx.y == 0;
    if (A.pub_flag && first && tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(A.pub_flag, A.pub_v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    int y = blockIdx.y;
    if (y < A.n_copy_rows) {  // a copy (or wait-only) row: block-uniform branch
        if ((int)blockIdx.x >= A.copy_x) return;
        if (A.wait_flags) {
            if (first) {  // the one poller of the host page
                if (tid < 64) {
                    wave_wait_flags(A.wait_flags, A.wait_mask, A.wait_v, A.timeout_ticks, A.err);
                    if (tid == 0)
                        __hip_atomic_store(A.go, A.go_token, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            } else if (A.n_halo > 0 && tid == 0) {
                while (__hip_atomic_load(A.go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < A.go_token)
                    __builtin_amdgcn_s_sleep(4);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: peers' data
            }
            __syncthreads();
        }
        if (A.n_halo == 0) return;
        halo_copy_share<true>(A.halo_src[y], A.halo_dst[y], blockIdx.x * blockDim.x + tid,
                              A.copy_x * (int)blockDim.x, A.nk);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its stores done
        __syncthreads();
        if (tid == 0)
            __hip_atomic_fetch_add(A.copy_cnt, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    y -= A.n_copy_rows;
    const KsView W{A.k_grid, V, dV};
    if (y < A.n_list) {
        howard_slopes_col<true, false>(A, W, A.col_list[y], k_opt, Vn, dVn, s_v, O);
        return;
    }
    if (A.n_halo > 0) {  // wait for every copy block of this launch
        if (tid == 0)
            while (__hip_atomic_load(A.copy_cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
                   A.copy_target)
                __builtin_amdgcn_s_sleep(8);
        __syncthreads();
    }
    howard_slopes_col<true, true>(A, W, A.bnd_list[y - A.n_list], k_opt, Vn, dVn, s_v, O);
}

// The staged direct schedule's halo refresh: column q (nk doubles) from src[q] (a peer's buffer,
// mapped through IPC) to dst[q] (this device).  The reads are system-scope loads, so they are
// served coherently from the owner's memory, not from lines this device's caches kept from an
// earlier copy of the same buffer; one launch for every column of the sweep.
__global__ __launch_bounds__(256) void ks_halo_copy_kernel(const double* const* __restrict__ src,
                                                           double* const* __restrict__ dst,
                                                           int nk) {
    halo_copy_share(src[blockIdx.y], dst[blockIdx.y], blockIdx.x * 256 + threadIdx.x,
                    gridDim.x * 256, nk);
}
int launch_ks_halo_copy(const double* const* src, double* const* dst, int ncols, int nk,
                        hipStream_t st) {
    if (ncols <= 0) return AIY_OK;
    if (ncols > 65535 || nk < 1) return fail(AIY_BAD_SHAPE, "halo copy: 1 <= columns <= 65535");
    ks_halo_copy_kernel<<<dim3((unsigned)std::min((nk + 255) / 256, 64), (unsigned)ncols), 256, 0, st>>>(
        src, dst, nk);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}

// the segment hints of the shard's nodes from k_opt (what ks_improve_kernel stores), for nodes
// whose k_opt arrived from another rank (ks_dist.py ghost columns)
__global__ void ks_hints_kernel(KsArgs A, const double* __restrict__ k_opt) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= A.n_local) return;
    int n = A.node0 + blockIdx.y * A.sstride + t;
    const double kp = k_opt[n];
    A.seg_hint[n] = seg_of_dev(A.k_grid, A.nk, fmax(fmin(kp, A.k_grid[A.nk - 1]), A.k_grid[0]));
}

// max |v - v_old| / (|v_old| + 1e-10) ignoring NaN (:195)
__global__ void ks_reldiff_kernel(KsArgs A, const double* __restrict__ V,
                                  const double* __restrict__ Vold,
                                  unsigned long long* __restrict__ slots) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    bool ok = false;
    double d = 0;
    if (t < A.n_local) {
        int n = A.node0 + blockIdx.y * A.sstride + t;
        d = fabs(V[n] - Vold[n]) / (fabs(Vold[n]) + 1e-10);
        ok = d == d;
    }
    block_max_to_slots(ok, d, slots);
}

// ------------------------------------------------------------------------------ fused
// One workgroup, everything in LDS: kg | V | dV | Vn ; k_opt and v_old stay in registers.
constexpr int kFusedThreads = 1024;
constexpr int kFusedMaxPerThread = 4;  // nodes per thread

__global__ __launch_bounds__(kFusedThreads) void ks_fused_vfi_kernel(KsArgs A, double* V_io,
                                                                     double* kopt_io,
                                                                     int* nfev_io, KsOut* out) {
    extern __shared__ double lds[];
    const int nk = A.nk, n_all = A.nk * A.nK * 4;
    double* kg = lds;
    double* V = kg + nk;
    double* dV = V + n_all;
    double* Vn = dV + n_all;
    __shared__ double s_red[kFusedThreads / 64];
    __shared__ int s_flag;
    const int tid = threadIdx.x;
    for (int q = tid; q < nk; q += blockDim.x) kg[q] = A.k_grid[q];
    for (int q = tid; q < n_all; q += blockDim.x) V[q] = V_io[q];
    double kopt[kFusedMaxPerThread], vold[kFusedMaxPerThread];
#pragma unroll
    for (int r = 0; r < kFusedMaxPerThread; ++r) {
        int n = tid + r * kFusedThreads;
        kopt[r] = n < n_all ? kopt_io[n] : 0.0;
        vold[r] = 0.0;
    }
    __syncthreads();
    auto slopes = [&]() {
        for (int q = tid; q < n_all; q += blockDim.x)
            dV[q] = pchip_slope(kg, V + (q / nk) * nk, nk, q % nk);
        __syncthreads();
    };
    int it = 0;
    double rel = __builtin_nan("");
    for (it = 1; it <= A.max_vfi; ++it) {
#pragma unroll
        for (int r = 0; r < kFusedMaxPerThread; ++r) {
            int n = tid + r * kFusedThreads;
            if (n < n_all) vold[r] = V[n];  // value_old = value (:145)
        }
        KsView W{kg, V, dV};
        if ((it - 1) % 5 == 0) {  // policy improvement (:148-168)
            slopes();
#pragma unroll
            for (int r = 0; r < kFusedMaxPerThread; ++r) {
                int n = tid + r * kFusedThreads;
                if (n < n_all) {
                    int nf = 0;
                    kopt[r] = improve_node(A, W, n, &nf);
                    if (nfev_io) nfev_io[n] = nf;
                }
            }
            __syncthreads();
        }
        for (int h = 0; h < A.howard; ++h) {  // Jacobi Howard sweeps (:172-192)
            slopes();
            KsView Wh{kg, V, dV};
#pragma unroll
            for (int r = 0; r < kFusedMaxPerThread; ++r) {
                int n = tid + r * kFusedThreads;
                if (n < n_all) Vn[n] = howard_node(A, Wh, n, kopt[r]);
            }
            __syncthreads();
            for (int q = tid; q < n_all; q += blockDim.x) V[q] = Vn[q];
            __syncthreads();
        }
        // relative difference, NaN ignored (:195)
        double m = -1.0;
#pragma unroll
        for (int r = 0; r < kFusedMaxPerThread; ++r) {
            int n = tid + r * kFusedThreads;
            if (n < n_all) {
                double d = fabs(V[n] - vold[r]) / (fabs(vold[r]) + 1e-10);
                if (d == d) m = fmax(m, d);
            }
        }
        for (int off = 32; off > 0; off >>= 1) m = fmax(m, __shfl_xor(m, off));
        if ((tid & 63) == 0) s_red[tid >> 6] = m;
        __syncthreads();
        if (tid == 0) {
            double mm = -1.0;
            for (int q = 0; q < kFusedThreads / 64; ++q) mm = fmax(mm, s_red[q]);
            rel = mm < 0 ? __builtin_nan("") : mm;
            s_flag = (rel < A.tol) ? 1 : 0;
            s_red[0] = rel;
        }
        __syncthreads();
        rel = s_red[0];
        if (s_flag) break;
        __syncthreads();
    }
    if (it > A.max_vfi) it = A.max_vfi;
    for (int q = tid; q < n_all; q += blockDim.x) V_io[q] = V[q];
#pragma unroll
    for (int r = 0; r < kFusedMaxPerThread; ++r) {
        int n = tid + r * kFusedThreads;
        if (n < n_all) kopt_io[n] = kopt[r];
    }
    if (tid == 0) {
        out->iters = it;
        out->rel = rel;
    }
}

// ------------------------------------------------------------------------------ launchers
static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

size_t ks_fused_lds_bytes(int nk, int nK) { return sizeof(double) * ((size_t)nk + 3ull * nk * nK * 4); }
bool ks_fused_fits(int nk, int nK) {
    return (long long)nk * nK * 4 <= (long long)kFusedThreads * kFusedMaxPerThread &&
           ks_fused_lds_bytes(nk, nK) <= 150 * 1024;
}

int launch_ks_fused(const KsArgs& A, double* V, double* kopt, int* nfev, KsOut* out,
                    hipStream_t st) {
    KsArgs F = A;
    F.seg_hint = nullptr;  // k_opt lives in registers here; the search runs in LDS anyway
    F.colV = F.coldV = nullptr;  // (everything in LDS)
    ks_fused_vfi_kernel<<<1, kFusedThreads, ks_fused_lds_bytes(A.nk, A.nK), st>>>(F, V, kopt,
                                                                                  nfev, out);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}
// column-shaped grid: block of 64·ceil(nk / 64) <= 256 lanes along k, columns along y
static dim3 ks_col_block(int nk) { return dim3(std::min(256, (nk + 63) / 64 * 64)); }
static dim3 ks_col_grid(int nk, long long ncols, int nz = 1) {
    const int bx = (int)ks_col_block(nk).x;
    return dim3(cdiv(nk, bx), (unsigned)std::max<long long>(1, std::min<long long>(ncols, 65535)),
                std::max(nz, 1));
}
int launch_ks_slopes(const KsArgs& A, const double* V, double* dV, hipStream_t st) {
    ks_slopes_kernel<<<ks_col_grid(A.nk, 4ll * A.nK), ks_col_block(A.nk), 0, st>>>(A, V, dV);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}
int launch_ks_grid_tables(const double* kg, int nk, double* tab, hipStream_t st) {
    ks_grid_tables_kernel<<<(nk + 255) / 256, 256, 0, st>>>(kg, nk, tab);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}
int launch_ks_slopes_cols(const KsArgs& A, const int* cols, int ncols, const double* V,
                          double* dV, hipStream_t st) {
    if (ncols <= 0) return AIY_OK;
    ks_slopes_cols_kernel<<<ks_col_grid(A.nk, ncols), ks_col_block(A.nk), 0, st>>>(A, cols, ncols, V, dV);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}
int launch_ks_improve(const KsArgs& A, const double* V, const double* dV, double* kopt,
                      int* nfev, hipStream_t st) {
    ks_improve_kernel<<<dim3(cdiv(A.n_local, 128), std::max(A.ns, 1)), 128, 0, st>>>(A, V, dV, kopt, nfev);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}
int launch_ks_howard(const KsArgs& A, const double* V, const double* dV, const double* kopt,
                     double* Vn, hipStream_t st) {
    if (A.node0 % A.nk || A.n_local % A.nk || (A.ns > 1 && A.sstride % A.nk))
        return fail(AIY_BAD_SHAPE, "Howard launch: node range must be whole columns");
    ks_howard_kernel<<<ks_col_grid(A.nk, A.n_local / A.nk, A.ns), ks_col_block(A.nk), 0, st>>>(
        A, V, dV, kopt, Vn);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}
static int ks_fused_geometry(int nk, int* B) {
    *B = (int)ks_col_block(nk).x;  // 64 .. 256
    return nk <= *B ? nk : *B - 4;
}
int launch_ks_howard_slopes(const KsArgs& A, const double* V, const double* dV,
                            const double* kopt, double* Vn, double* dVn, hipStream_t st) {
    if (A.node0 % A.nk || A.n_local % A.nk || (A.ns > 1 && A.sstride % A.nk))
        return fail(AIY_BAD_SHAPE, "Howard launch: node range must be whole columns");
    int B;
    const int O = ks_fused_geometry(A.nk, &B);
    const dim3 g(cdiv(A.nk, O), (unsigned)std::max(1, std::min(A.n_local / A.nk, 65535)),
                 std::max(A.ns, 1));
    // dealt tile-major by XCD (ks_howard_slopes_xcd_kernel): 200 -> 194 us per sweep at
    // k = 32,768, K = 64 (profiles/r06_g07_ks_xcd_ab.txt); the 3-D grid beyond 65,535 columns
    if ((long long)g.x * g.y * g.z < (1ll << 31) && A.n_local / A.nk <= 65535) {
        const int C = (int)g.y * (int)g.z;
        ks_howard_slopes_xcd_kernel<<<dim3(g.x * C), B, 0, st>>>(A, V, dV, kopt, Vn, dVn, O,
                                                                  (int)g.x, C);
        AIY_HIP(hipGetLastError());
        return AIY_OK;
    }
    ks_howard_slopes_kernel<<<g, B, 0, st>>>(A, V, dV, kopt, Vn, dVn, O);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}
int ks_staged_copy_blocks(int nk) {
    int B;
    const int O = ks_fused_geometry(nk, &B);
    return std::min(cdiv(nk, O), kCopyX);
}
int launch_ks_staged_sweep(const KsArgs& A, const double* V, const double* dV,
                           const double* kopt, double* Vn, double* dVn, hipStream_t st) {
    int B;
    const int O = ks_fused_geometry(A.nk, &B);
    const long long rows = (long long)A.n_copy_rows + A.n_list + A.n_bnd;
    if (rows > 65535) return fail(AIY_BAD_SHAPE, "staged sweep: at most 65,535 block rows");
    if (rows == 0) return AIY_OK;
    if ((A.n_list && !A.col_list) || (A.n_bnd && !A.bnd_list) ||
        (A.n_halo && (!A.halo_src || !A.halo_dst || !A.copy_cnt)))
        return fail(AIY_BAD_ARG, "staged sweep: missing list or halo pointers");
    ks_staged_sweep_kernel<<<dim3(cdiv(A.nk, O), (unsigned)rows), B, 0, st>>>(A, V, dV, kopt, Vn,
                                                                           dVn, O);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}
int launch_ks_hints(const KsArgs& A, const double* kopt, hipStream_t st) {
    if (!A.seg_hint) return AIY_OK;
    ks_hints_kernel<<<dim3(cdiv(A.n_local, 256), std::max(A.ns, 1)), 256, 0, st>>>(A, kopt);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}
int launch_ks_reldiff(const KsArgs& A, const double* V, const double* Vold,
                      unsigned long long* slots, hipStream_t st) {
    ks_reldiff_kernel<<<dim3(cdiv(A.n_local, 256), std::max(A.ns, 1)), 256, 0, st>>>(A, V, Vold, slots);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}

}  // namespace aiy
