// A1/A2 and A3 — exhaustive Bellman sweeps on gfx950.
//   A1: Aiyagari_VFI.m:70-83 (GE copy :152-165)           max over a'          (Nl = 1)
//   A3: Aiyagari_Endogenous_Labor_VFI.m:69-112 (GE :176-219) max over (l, a') column-major
// A1 is the Nl = 1 case of A3 with L = 1 and no disutility term: the cash-on-hand and value
// expressions then coincide operation for operation, so one kernel family serves both.
//
// Four launches per sweep on the caller's stream:
//   1. table   EV(i,k) = Σ_m (β·P(i,m))·V(m,k), m ascending (:79 / Labor :69), and the
//              screening key D(i,k) = n·EV + 1 + τ(|n·EV| + 1), stored as (a_k, D) pairs.
//   2. init    per state: an exact starting candidate — the hint (last sweep's argmax), a
//              coarse scan of every feasible prefix (stride S) and a bracket refinement
//              (steps S/2, S/4, ..., 1) around the best point of each labour level.  For a
//              unimodal objective this IS the maximiser; it only sets the screening bar.
//   3. screen  every feasible candidate.  Work item = one wave × (64·R states × LB labour
//              levels) × CK candidates a', so all waves carry equal work.  Per candidate 6
//              fp64 VALU ops: c = coh − a_k, q = c^n, t = (D_k − B)·q, test t ≥ 1 − 2^-48
//              where B = n·(best + dis_l) − slack.  The test is TRUE for every candidate whose
//              exact value reaches the running best (DESIGN.md §A1 bounds the rounding), so
//              evaluating exactly only the candidates that pass, and merging with the
//              (max value, first column-major index) rule, reproduces the plain exhaustive
//              scan bit for bit.
//              Mixed precision: each work item first screens in packed fp32 (v_pk_* — two
//              candidates per VALU op) against a chunk-relative table rounded OUTWARD
//              (a' rounded down, D' up, coh' up, B' down) with threshold 1 − 2^-19, which
//              bounds every fp32 rounding of the product; a passing 16-candidate block is
//              re-screened in fp64 and evaluated exactly, so the fp32 stage only ever adds
//              work, never drops a candidate.
//   4. merge   per state: init ⊕ every chunk's improvement → v_new, index, policy_k = a(k),
//              policy_l = L(l), policy_c = c(l,k), and max|v_new − v_old| ignoring NaN via an
//              order-independent atomicMax on IEEE bits.
// Non-integer σ (or σ > 9) runs a plain exhaustive kernel (device pow/log).
#include <hip/hip_ext.h>

#include <algorithm>
#include <type_traits>

#include "aiy_common.hpp"
#include "bell_dev.hpp"
#include "bellman.hpp"

namespace aiy {

// ------------------------------------------------------------------------------ batches
// Config 4 (BASELINE configs[3]): C candidate interest rates in one launch.  Every per-state
// array is a [C] block of its single-candidate layout; candidate c sees BellArgs shifted to its
// block, its own r and w, and its own diff slots (two parities, so sweep g's table kernel can
// read sweep g-1's slots while the tree kernel of g writes the other set).
__device__ __forceinline__ BellArgs bell_cand(const BellArgs& A, int c) {
    BellArgs B = A;
    const size_t o = (size_t)c * A.N * A.Na;
    B.r = A.rv[c];
    B.w = A.wv[c];
    B.v_old += o;
    B.EV += o;
    if (B.Dt) B.Dt += o;
    if (B.Dm8) B.Dm8 += (size_t)c * A.N * A.nb8;
    if (B.Dm512) B.Dm512 += (size_t)c * A.N * A.nb512;
    B.kf += o * A.Nl;
    B.best0 += o;
    B.idx0 += o;
    if (B.hint) B.hint += o;
    if (B.mom) B.mom += o;
    B.v_new += o;
    B.idx += o;
    if (B.pk) B.pk += o;
    if (B.pc) B.pc += o;
    B.diff += ((size_t)c * 2 + A.parity) * 2 * kDiffSlots;
    B.C = 1;
    return B;
}

// ------------------------------------------------------------------------------ 0. EV by MFMA
// EV = (βP)·V on the fp64 matrix cores (v_mfma_f64_16x16x4_f64) when Nz is large enough for
// the expectation to be a real contraction (north star).  A wave owns a 16 (i) x 16 (k) tile of
// EV and walks m in steps of 4: A = βP[i][m] (lane l: row l & 15, m = l >> 4 — the product βP
// formed first, as the reference's (beta * P) * v_old associates), B = V[m][k] (lane l: m =
// l >> 4, column l & 15), C/D in the f64 layout (column l & 15, row (l >> 4) + 4·reg).  Four
// waves per block cover 64 consecutive k; blockIdx.y = 16-row tile, blockIdx.z = candidate
// (config 4 batches; candidates stopped at an earlier sweep are skipped — one that stops at
// this sweep, decided by the table kernel after this pass, gets one unused pass, and its EV
// buffer is scratch from then on).  Out-of-range rows/columns/m are zero.
typedef double aiy_v4d __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void bell_ev_mfma_kernel(int N, int Na,
                                                           const double* __restrict__ P,
                                                           const double* __restrict__ V,
                                                           double beta, double* __restrict__ EV,
                                                           const int* __restrict__ stop) {
    const int c = blockIdx.z;
    if (stop && stop[c]) return;  // block-uniform
    const size_t o = (size_t)c * N * Na;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int i0 = blockIdx.y * 16, k0 = blockIdx.x * 64 + wave * 16;
    const int r = lane & 15, q = lane >> 4;
    const int ia = i0 + r, kb = k0 + r;
    aiy_v4d acc = {0.0, 0.0, 0.0, 0.0};
    for (int m0 = 0; m0 < N; m0 += 4) {
        const int m = m0 + q;
        const double av = (ia < N && m < N) ? beta * P[ia * N + m] : 0.0;
        const double bv = (m < N && kb < Na) ? V[o + (size_t)m * Na + kb] : 0.0;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
    }
    const int kc = k0 + r;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int i = i0 + q + 4 * g;
        if (i < N && kc < Na) EV[o + (size_t)i * Na + kc] = acc[g];
    }
}

// ------------------------------------------------------------------------------ 1. table
// 2-D grid (x: 512 candidates of a row, y: row i).  Besides EV and the (a_k, D_k) pairs the
// kernel writes the screening bounds: the maxima of D over aligned 8-, 64- and 512-candidate
// blocks of the row (lane butterflies, then LDS across the block's 8 waves).  Block (0, 0)
// clears the diff slots of the coming sweep — after folding the previous sweep's slots into
// fold[0..1] when asked (the speculative solve's per-sweep diff, without a reduce launch).
constexpr int kTableBlock = 512;
__global__ __launch_bounds__(kTableBlock) void bell_table_kernel(
    int N, int Na, const double* __restrict__ P, const double* __restrict__ V, double beta,
    int np, const double* __restrict__ a, double* __restrict__ EV, double2* __restrict__ T,
    float* __restrict__ T32, int CK, double* __restrict__ Dm, double* __restrict__ Dm8,
    double* __restrict__ Dm512, int nb, int nb8, int nb512,
    unsigned long long* __restrict__ diff, double* __restrict__ Dt,
    unsigned long long* __restrict__ fold, bool ev_in, bool xcd) {
    __shared__ double s_max[kTableBlock / 64];
    // xcd: the (chunk, row) of this block is dealt like the tree kernel's items (xcd_remap over
    // the row-major order), so the XCD that writes a row's table chunk is the one whose tree
    // tiles read it first (the hint window, the climb, the 8-block bounds near the optimum):
    // those first touches hit that XCD's L2 instead of the MALL.  Work order only.
    int i = blockIdx.y, cx = blockIdx.x;
    if (xcd) {
        const int p = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
        i = p / gridDim.x;
        cx = p - i * gridDim.x;
    }
    const int k = cx * kTableBlock + threadIdx.x;
    if (diff && blockIdx.x == 0 && blockIdx.y == 0) {  // block-uniform branch
        if (fold && threadIdx.x < 64) {  // same fold as reduce_slots_kernel
            const int l = threadIdx.x;
            unsigned long long m = diff[2 * l];
            const int any = __ballot((diff[2 * l + 1] & 1ull) != 0ull) != 0ull;
            for (int off = 32; off > 0; off >>= 1) {
                unsigned long long o = __shfl_xor(m, off);
                m = o > m ? o : m;
            }
            if (l == 0) {
                fold[0] = m;
                fold[1] = any ? 1ull : 0ull;
            }
        }
        __syncthreads();
        if (threadIdx.x < 2 * kDiffSlots) diff[threadIdx.x] = 0ull;
    }
    const bool ok = k < Na;
    double D = -__builtin_inf();
    if (ok) {
        const size_t t = (size_t)i * Na + k;
        double acc;
        if (ev_in) {  // EV already written by bell_ev_mfma_kernel
            acc = EV[t];
        } else {
            acc = table_ev(N, Na, P, V, beta, i, k);
            EV[t] = acc;
        }
        if (T || Dt) {
            D = table_D(acc, np);
            if (T) T[t] = make_double2(a[k], D);
            if (Dt) Dt[t] = D;
            if (T32) {  // relative to the chunk origin (a, D at k0): small magnitudes, fine ulps
                int k0 = k - k % CK;
                double D0 = table_D(ev_in ? EV[(size_t)i * Na + k0]
                                          : table_ev(N, Na, P, V, beta, i, k0), np);
                float* pr = T32 + 2 * (size_t)i * (Na + (Na & 1)) + 2 * (k & ~1) + (k & 1);
                pr[0] = f32_dn(a[k] - a[k0]);  // pair layout {a_k, a_k+1, D_k, D_k+1}
                pr[2] = f32_up(D - D0);
            }
        }
    }
    if (!T && !Dt) return;  // uniform per launch
    // block maxima (NaN keys drop out of fmax: a NaN candidate is never a maximiser), by DPP
    // lane moves: lane ^ 1, lane ^ 2, lane + 4 give the 8-block maximum at lanes 8j; the
    // reduction ladder gives the wave's 64-block maximum at lane 63
    {
        double d8 = fmax(D, dpp_d<0xB1>(D));
        d8 = fmax(d8, dpp_d<0x4E>(d8));
        d8 = fmax(d8, dpp_d<0x104>(d8));
        if (Dm8 && ok && (k & 7) == 0) Dm8[(size_t)i * nb8 + (k >> 3)] = d8;
    }
    D = fmax(D, dpp_d<0xB1>(D));
    D = fmax(D, dpp_d<0x4E>(D));
    D = fmax(D, dpp_d<0x141>(D));         // row half-mirror: max of 8
    D = fmax(D, dpp_d<0x140>(D));         // row mirror: max of 16
    D = fmax(D, dpp_d<0x142, 0xa>(D));    // row_bcast:15: max of 32 in rows 1, 3
    D = fmax(D, dpp_d<0x143, 0xc>(D));    // row_bcast:31: max of 64 in row 3
    D = readlane_d(D, 63);
    if (Dm && ok && (k & 63) == 0) Dm[(size_t)i * nb + (k >> 6)] = D;
    if (Dm512) {
        if ((threadIdx.x & 63) == 0) s_max[threadIdx.x >> 6] = D;
        __syncthreads();
        if (threadIdx.x == 0) {
            double m = s_max[0];
            for (int q = 1; q < kTableBlock / 64; ++q) m = fmax(m, s_max[q]);
            Dm512[(size_t)i * nb512 + cx] = m;
        }
    }
}

// Batched table (config 4): grid (x: 512 candidates of a row, y: C·N rows).  Besides the
// single-candidate table it runs candidate c's stopping rule (Aiyagari_VFI.m:85-86): it folds
// the diff slots the previous sweep's tree kernel left for c and, below tol, marks c stopped at
// that sweep (stop[c] = sweep - 1) — then neither this sweep's table nor tree touches c again,
// so c's buffers keep v_new, v_old and the policies of its stopping sweep (break semantics),
// while the other candidates go on.  Every block of c takes the same decision from the same
// slots; block (0, row 0 of c) records it and clears this sweep's slot set.
__global__ __launch_bounds__(kTableBlock) void bell_table_batch_kernel(
    int N, int Na, const double* __restrict__ P, const double* __restrict__ V, double beta,
    int np, const double* __restrict__ a, double* __restrict__ EV, double* __restrict__ Dt,
    double* __restrict__ Dm8, double* __restrict__ Dm512, int nb8, int nb512,
    unsigned long long* __restrict__ slots, int* __restrict__ stop, int sweep, double tol,
    bool ev_in, bool xcd) {
    __shared__ double s_max[kTableBlock / 64];
    __shared__ int s_stop;
    int cy = blockIdx.y, cx = blockIdx.x;  // (xcd: dealt as the tree's items, bell_table_kernel)
    if (xcd) {
        const int p = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
        cy = p / gridDim.x;
        cx = p - cy * gridDim.x;
    }
    const int c = cy / N, i = cy - c * N;
    if (stop[c]) return;  // block-uniform
    if (sweep > 1) {
        if (threadIdx.x < 64) {
            const int l = threadIdx.x;
            const unsigned long long* sl = slots + ((size_t)c * 2 + ((sweep - 1) & 1)) * 2 * kDiffSlots;
            unsigned long long m = sl[2 * l];
            const int any = __ballot((sl[2 * l + 1] & 1ull) != 0ull) != 0ull;
            for (int off = 32; off > 0; off >>= 1) {
                const unsigned long long o = __shfl_xor(m, off);
                m = o > m ? o : m;
            }
            if (l == 0) s_stop = any && aiy_bitsd(m) < tol;  // NaN-only: no stop (:85)
        }
        __syncthreads();
        if (s_stop) {
            if (cx == 0 && i == 0 && threadIdx.x == 0) stop[c] = sweep - 1;
            return;
        }
    }
    if (cx == 0 && i == 0 && threadIdx.x < 2 * kDiffSlots)
        slots[((size_t)c * 2 + (sweep & 1)) * 2 * kDiffSlots + threadIdx.x] = 0ull;
    const size_t o = (size_t)c * N * Na;
    const int k = cx * kTableBlock + threadIdx.x;
    const bool ok = k < Na;
    double D = -__builtin_inf();
    if (ok) {
        const size_t t = o + (size_t)i * Na + k;
        double acc;
        if (ev_in) {
            acc = EV[t];
        } else {
            acc = table_ev(N, Na, P, V + o, beta, i, k);
            EV[t] = acc;
        }
        D = table_D(acc, np);
        Dt[t] = D;
    }
    const size_t rb8 = ((size_t)c * N + i) * nb8, rb512 = ((size_t)c * N + i) * nb512;
    {  // DPP maxima, as bell_table_kernel
        double d8 = fmax(D, dpp_d<0xB1>(D));
        d8 = fmax(d8, dpp_d<0x4E>(d8));
        d8 = fmax(d8, dpp_d<0x104>(d8));
        if (ok && (k & 7) == 0) Dm8[rb8 + (k >> 3)] = d8;
    }
    D = fmax(D, dpp_d<0xB1>(D));
    D = fmax(D, dpp_d<0x4E>(D));
    D = fmax(D, dpp_d<0x141>(D));
    D = fmax(D, dpp_d<0x140>(D));
    D = fmax(D, dpp_d<0x142, 0xa>(D));
    D = fmax(D, dpp_d<0x143, 0xc>(D));
    D = readlane_d(D, 63);
    if ((threadIdx.x & 63) == 0) s_max[threadIdx.x >> 6] = D;
    __syncthreads();
    if (threadIdx.x == 0) {
        double m = s_max[0];
        for (int q = 1; q < kTableBlock / 64; ++q) m = fmax(m, s_max[q]);
        Dm512[rb512 + cx] = m;
    }
}

int launch_bell_table_batch(const BellArgs& A, unsigned long long* slots, int sweep, double tol,
                            hipStream_t st) {
    dim3 grid((A.Na + kTableBlock - 1) / kTableBlock, A.C * A.N);
    bell_table_batch_kernel<<<grid, kTableBlock, 0, st>>>(
        A.N, A.Na, A.P, A.v_old, A.beta, A.np, A.a, A.EV, A.Dt, A.Dm8, A.Dm512, A.nb8, A.nb512,
        slots, const_cast<int*>(A.stop), sweep, tol, A.ev_mfma, (A.variant & 16) != 0);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}

// ------------------------------------------------------------------------------ 1b. kf
// feasible prefix per (l, i, j): depends on (r, w, a, s, L) only, so a solve computes it once
template <bool LAB>
__global__ void bell_kf_kernel(BellArgs A0) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    int n = A0.N * A0.Na;
    BellArgs A = A0;
    if (A0.C > 1) {  // batched: t spans C blocks of (l, i, j)
        const int c = t / (n * A0.Nl);
        if (c >= A0.C) return;
        A = bell_cand(A0, c);
        t -= c * n * A0.Nl;
    }
    if (t >= n * A.Nl) return;
    int l = t / n, ij = t - l * n;
    int i = ij / A.Na, j = ij - i * A.Na;
    double coh = cash<LAB>((1 + A.r) * A.a[j], A.w * A.s[i], LAB ? A.L[l] : 1.0);
    A.kf[t] = lower_bound_dev(A.a, A.Na, coh);
}

// ------------------------------------------------------------------------------ 2. init
template <int NP, bool LAB>
__global__ void bell_init_kernel(BellArgs A0) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    BellArgs A = A0;
    if (A0.C > 1) {
        const int c = t / (A0.N * A0.Na);
        if (c >= A0.C || A0.stop[c]) return;
        A = bell_cand(A0, c);
        t -= c * A0.N * A0.Na;
    }
    if (t >= A.N * A.Na) return;
    const int Na = A.Na, Nl = A.Nl;
    int i = t / Na, j = t - i * Na;
    const double* __restrict__ a = A.a;
    const double* __restrict__ ev = A.EV + (size_t)i * Na;
    double x = (1 + A.r) * a[j];
    double y = A.w * A.s[i];
    double best = __builtin_nan("");
    int idx = -1;
    bool anyfeas = false;
    auto eval = [&](int l, int k, double coh) {
        double dis = LAB ? A.dis[l] : 0.0;
        return bell_val<NP, LAB>(coh - a[k], ev[k], A.sigma, dis);
    };
    const int n_all = A.N * Na;
    const int S = A.coarse;
    int hl = -1, hk = -1;
    if (A.hint) {
        int h = A.hint[t];
        if (h >= 0 && h % Nl < Nl) {
            hl = h % Nl;
            int kf = A.kf[hl * n_all + t];
            if (kf > 0) {
                hk = min(h / Nl, kf - 1);
                double coh = cash<LAB>(x, y, LAB ? A.L[hl] : 1.0);
                lexi_take(eval(hl, hk, coh), hl + Nl * hk, best, idx);
            }
        }
    }
    for (int l = 0; l < Nl; ++l) {
        int kf = A.kf[l * n_all + t];
        if (kf == 0) continue;
        anyfeas = true;
        double coh = cash<LAB>(x, y, LAB ? A.L[l] : 1.0);
        double lb = __builtin_nan("");
        int lk = -1;
        // with a hint only its labour level is searched: one good candidate sets the bar
        if (A.hint && hk >= 0 && l != hl) continue;
        if (S > 0 && hk < 0) {  // cold start: coarse scan of the feasible prefix
            int k = 0;
            for (; k + 3 * S < kf; k += 4 * S) {  // 4 independent evaluations in flight
                double v0 = eval(l, k, coh), v1 = eval(l, k + S, coh);
                double v2 = eval(l, k + 2 * S, coh), v3 = eval(l, k + 3 * S, coh);
                lexi_take(v0, k, lb, lk);
                lexi_take(v1, k + S, lb, lk);
                lexi_take(v2, k + 2 * S, lb, lk);
                lexi_take(v3, k + 3 * S, lb, lk);
            }
            for (; k < kf; k += S) lexi_take(eval(l, k, coh), k, lb, lk);
            lexi_take(eval(l, kf - 1, coh), kf - 1, lb, lk);
        }
        if (A.hint && hk >= 0) {  // warm start: last sweep's argmax
            int k = hk < kf ? hk : kf - 1;
            lexi_take(eval(l, k, coh), k, lb, lk);
        }
        if (lk < 0) lexi_take(eval(l, 0, coh), 0, lb, lk);
        int step0 = S > 0 ? (S >> 1) : 64;
        if (lk < 0 || lb != lb) continue;
        // bracket refinement: for a unimodal objective this lands on the maximiser
        for (int step = step0; step >= 1; step >>= 1) {
            int c0 = lk;
            if (c0 - step >= 0) lexi_take(eval(l, c0 - step, coh), c0 - step, lb, lk);
            if (c0 + step < kf) lexi_take(eval(l, c0 + step, coh), c0 + step, lb, lk);
        }
        lexi_take(lb, l + Nl * lk, best, idx);
    }
    A.best0[t] = best;
    A.idx0[t] = anyfeas ? idx : -2;  // -2: no feasible choice at all
}

// ------------------------------------------------------------------------------ 3. screen
template <int NP, bool LAB, int R, int LB, int KB, int MINW>
__global__ __launch_bounds__(256, MINW) void bell_screen_kernel(BellArgs A, int ntile, int nlb,
                                                                int nchunk) {
    const int wave = readfirst(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int item = readfirst(blockIdx.x * 4 + wave);
    const int chunk = item % nchunk;
    int rest = item / nchunk;
    const int lbk = rest % nlb;
    rest /= nlb;
    const int tile = rest % ntile;
    const int i = rest / ntile;
    const int N = A.N, Na = A.Na, Nl = A.Nl, CK = A.CK;
    if (i >= N) return;
    const double* __restrict__ a = A.a;
    const int jbase = tile * (64 * R);
    const int jlast = min(jbase + 64 * R, Na) - 1;
    const int l0 = lbk * LB;
    const int l1 = min(l0 + LB, Nl);
    const double y = A.w * A.s[i];
    // wave-uniform feasible range from the cached prefixes (kf is monotone in j)
    int kmax = 0, kmin = 0x7fffffff;
    {
        const size_t nall = (size_t)N * Na;
        for (int l = l0; l < l1; ++l) {
            kmax = max(kmax, A.kf[l * nall + (size_t)i * Na + jlast]);
            kmin = min(kmin, A.kf[l * nall + (size_t)i * Na + jbase]);
        }
        kmax = readfirst(kmax);
        kmin = readfirst(kmin);
    }
    const int k_lo = chunk * CK;
    if (k_lo >= kmax) return;
    const int k_hi = min(k_lo + CK, kmax);

    double coh[R][LB], B[R][LB], best[R], dis[LB];
    int idx[R], imp[R];
#pragma unroll
    for (int q = 0; q < LB; ++q) dis[q] = (LAB && l0 + q < l1) ? A.dis[l0 + q] : 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        int j = jbase + r * 64 + lane;
        imp[r] = -1;
        bool ok = j < Na;
        size_t ij = (size_t)i * Na + (ok ? j : 0);
        best[r] = ok ? A.best0[ij] : 0.0;
        idx[r] = ok ? A.idx0[ij] : 0x7fffffff;
        if (idx[r] == -2) idx[r] = -1;
        double x = ok ? (1 + A.r) * a[j] : 0.0;
#pragma unroll
        for (int q = 0; q < LB; ++q) {
            bool okq = ok && (l0 + q < l1);
            // invalid sub-states get a NaN bar: every screen test on them is false
            coh[r][q] = okq ? cash<LAB>(x, y, LAB ? A.L[l0 + q] : 1.0) : 0.0;
            B[r][q] = okq ? screen_B(best[r], idx[r], dis[q], NP) : __builtin_nan("");
        }
    }
    const double2* __restrict__ Trow = A.T + (size_t)i * Na;
    const double* __restrict__ ev = A.EV + (size_t)i * Na;
    unsigned nhits = 0, nfine = 0;

    auto exact_block = [&](int k0, int kend) __attribute__((always_inline)) {
        for (int k = k0; k < kend; ++k) {
            const double2 tk = Trow[k];
#pragma unroll
            for (int r = 0; r < R; ++r) {
#pragma unroll
                for (int q = 0; q < LB; ++q) {
                    double c = coh[r][q] - tk.x;
                    int lin = (l0 + q) + Nl * k;
                    // the running best itself always passes; its value is already known
                    if (lin != idx[r] && c > 0 && (tk.y - B[r][q]) * aiy_ipow(c, NP) >= kThr) {
                        ++nhits;
                        double val = bell_val<NP, LAB>(c, ev[k], A.sigma, dis[q]);
                        if (lexi_take(val, lin, best[r], idx[r])) {
                            imp[r] = lin;
#pragma unroll
                            for (int q2 = 0; q2 < LB; ++q2)
                                if (B[r][q2] == B[r][q2])
                                    B[r][q2] = screen_B(best[r], idx[r], dis[q2], NP);
                        }
                    }
                }
            }
        }
    };

    // region 1: every sub-state feasible (k < kmin); region 2: c clamped at 0 so that
    // infeasible candidates (NaN / -Inf in the reference) never pass the screen
    auto run = [&](auto guard, int kb, int ke) __attribute__((always_inline)) {
        int k = kb;
        for (; k + KB <= ke; k += KB) {
            // max of t over the block (NaN from invalid sub-states drops out of fmax)
            double tm = -__builtin_inf();
#pragma unroll
            for (int kk = 0; kk < KB; ++kk) {
                const double2 tk = Trow[k + kk];  // wave-uniform address → scalar loads
#pragma unroll
                for (int r = 0; r < R; ++r) {
#pragma unroll
                    for (int q = 0; q < LB; ++q) {
                        double c = coh[r][q] - tk.x;
                        if constexpr (decltype(guard)::value) c = fmax(c, 0.0);
                        tm = fmax(tm, (tk.y - B[r][q]) * aiy_ipow(c, NP));
                    }
                }
            }
            if (__any(tm >= kThr)) exact_block(k, k + KB);
        }
        if (k < ke) {
            double tm = -__builtin_inf();
            for (int kk = k; kk < ke; ++kk) {
                const double2 tk = Trow[kk];
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int q = 0; q < LB; ++q)
                        tm = fmax(tm, (tk.y - B[r][q]) * aiy_ipow(fmax(coh[r][q] - tk.x, 0.0), NP));
            }
            if (__any(tm >= kThr)) exact_block(k, ke);
        }
    };

    // ---- packed fp32 pre-screen (all quantities relative to the chunk origin k_lo), set up
    // lazily: most work items never reach the candidate level
    int st32 = A.T32 != nullptr ? 0 : -1;  // 0 = not set up, 1 = on, -1 = off
    float cp[R][LB], bp[R][LB];
    const float* __restrict__ T32row = A.T32 ? A.T32 + 2 * (size_t)i * (Na + (Na & 1)) : nullptr;
    double S0 = 0.0;
    auto set_bp = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int q = 0; q < LB; ++q)
                bp[r][q] = (B[r][q] == B[r][q]) ? f32_dn(B[r][q] - S0) : __builtin_nanf("");
    };
    auto setup32 = [&]() __attribute__((always_inline)) {
        const double A0 = a[k_lo];
        S0 = Trow[k_lo].y;
        bool ok = true;
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int q = 0; q < LB; ++q) cp[r][q] = f32_up(coh[r][q] - A0);
        set_bp();
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int q = 0; q < LB; ++q) {
                ok = ok && fabsf(cp[r][q]) <= kBig32;
                ok = ok && (bp[r][q] != bp[r][q] || fabsf(bp[r][q]) <= kBig32);
            }
        // the chunk's table must be finite and moderate (else t = inf·0 could hide a pass)
        for (int k = k_lo + lane; k < k_hi; k += 64)  // no short circuit: loads overlap
            ok &= fabsf(T32row[2 * (k & ~1) + 2 + (k & 1)]) <= kBig32;
        st32 = __all(ok) ? 1 : -1;
    };
    auto run32 = [&](auto guard, int kb, int ke) __attribute__((always_inline)) {
        int k = kb;
        for (; k + KB <= ke; k += KB) {
            float tm = -__builtin_inff();
#pragma unroll
            for (int kk = 0; kk < KB; kk += 2) {
                // pair layout {a_k, a_k+1, D_k, D_k+1}: 64-bit scalar operands as loaded
                const float4 tq = *reinterpret_cast<const float4*>(T32row + 2 * (k + kk));
                const f32x2 av = {tq.x, tq.y}, dv = {tq.z, tq.w};
                f32x2 tt[R][LB];
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int q = 0; q < LB; ++q) {
                        f32x2 c = f32x2{cp[r][q], cp[r][q]} - av;
                        if constexpr (decltype(guard)::value) {
                            c.x = fmaxf(c.x, 0.0f);
                            c.y = fmaxf(c.y, 0.0f);
                        }
                        tt[r][q] = (dv - f32x2{bp[r][q], bp[r][q]}) * ipow2<NP>(c);
                    }
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int q = 0; q < LB; ++q) tm = fmaxf(fmaxf(tm, tt[r][q].x), tt[r][q].y);
            }
            if (__any(tm >= kThr32)) {
                exact_block(k, k + KB);  // fp64 screen + exact values on this block
                set_bp();
            }
        }
        if (k < ke) run(guard, k, ke);  // ragged tail: fp64
    };
    // one whole 64-candidate block in packed fp32 with a single wave vote: no branch between
    // the table loads, so they are all in flight together (a pass re-screens per 8 in fp64)
    auto block32 = [&](auto guard, int b0) __attribute__((always_inline)) {
        float tm = -__builtin_inff();
#pragma unroll 8
        for (int kk = 0; kk < 64; kk += 2) {
            const float4 tq = *reinterpret_cast<const float4*>(T32row + 2 * (b0 + kk));
            const f32x2 av = {tq.x, tq.y}, dv = {tq.z, tq.w};
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int q = 0; q < LB; ++q) {
                    f32x2 c = f32x2{cp[r][q], cp[r][q]} - av;
                    if constexpr (decltype(guard)::value) {
                        c.x = fmaxf(c.x, 0.0f);
                        c.y = fmaxf(c.y, 0.0f);
                    }
                    const f32x2 tt = (dv - f32x2{bp[r][q], bp[r][q]}) * ipow2<NP>(c);
                    tm = fmaxf(fmaxf(tm, tt.x), tt.y);
                }
        }
        if (__any(tm >= kThr32)) {
            run(guard, b0, b0 + 64);
            set_bp();
        }
    };
    // candidate level on [b0, b1): b0 is 64-aligned, so the fp32 pair layout lines up
    auto fine = [&](int b0, int b1) __attribute__((always_inline)) {
        if (st32 == 0) setup32();
        if (A.hitcount) nfine += b1 - b0;
        const bool guard = b1 > kmin;  // some sub-state's feasible prefix ends inside
        if (st32 == 1) {
            if (!LAB && b1 - b0 == 64) {  // (labour: 5 sub-states per lane, per-8 votes)
                if (guard) block32(std::true_type{}, b0);
                else block32(std::false_type{}, b0);
            } else {
                if (guard) run32(std::true_type{}, b0, b1);
                else run32(std::false_type{}, b0, b1);
            }
        } else {
            if (guard) run(std::true_type{}, b0, b1);
            else run(std::false_type{}, b0, b1);
        }
    };
    // block bound: for k in [b0, b1) the reference's own ordering gives c_k <= c_b0 and
    // D_k <= Dmax exactly (fp subtraction/multiplication are monotone), so
    // t_k = (D_k - B)·c_k^n <= (Dmax - B)·max(c_b0, 0)^n in floating point: a block whose
    // bound fails the threshold holds no candidate that can reach the running best.
    auto bound_pass = [&](double dmax, double a0) __attribute__((always_inline)) {
        double tm = -__builtin_inf();
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int q = 0; q < LB; ++q)
                tm = fmax(tm, (dmax - B[r][q]) * aiy_ipow(fmax(coh[r][q] - a0, 0.0), NP));
        return __any(tm >= kThr);
    };
    // the chunk's block bounds (Dmax, a at the block start) are fetched one block per lane in
    // a single round trip; superblock (8-block) maxima by butterfly; tests read them back with
    // v_readlane — the search itself never waits on memory
    const double* __restrict__ Dmrow = A.Dm + (size_t)i * A.nb;
    unsigned nsup = 0, nblk = 0;
    const int nbk = (k_hi - k_lo + 63) >> 6;
    for (int g = 0; g < nbk; g += 64) {
        const int gb = (k_lo >> 6) + g + lane;
        const bool okb = g + lane < nbk;
        const double dmv = okb ? Dmrow[gb] : -__builtin_inf();
        const double a0v = okb ? a[gb << 6] : 0.0;
        double smv = dmv;
        smv = fmax(smv, __shfl_xor(smv, 1));
        smv = fmax(smv, __shfl_xor(smv, 2));
        smv = fmax(smv, __shfl_xor(smv, 4));
        const int ng = min(64, nbk - g);
        for (int sb = 0; sb < ng; sb += 8) {
            ++nsup;
            if (!bound_pass(readlane_d(smv, sb), readlane_d(a0v, sb))) continue;
            const int se = min(sb + 8, ng);
            for (int b = sb; b < se; ++b) {
                if (se - sb > 1) {
                    ++nblk;
                    if (!bound_pass(readlane_d(dmv, b), readlane_d(a0v, b))) continue;
                }
                const int b0 = k_lo + ((g + b) << 6);
                fine(b0, min(b0 + 64, k_hi));
            }
        }
    }
    if (A.hitcount) {
        const unsigned ns = 64 * R * (l1 - l0);
        nsup *= ns;
        nblk *= ns;
    }

    const size_t slab = ((size_t)lbk * nchunk + chunk) * N + i;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        int j = jbase + r * 64 + lane;
        if (j < Na && imp[r] >= 0) {  // rare: the merge reads and resets only touched states
            A.partial[slab * Na + j] = imp[r];
            A.touched[(size_t)i * Na + j] = 1;
        }
    }
    if (A.hitcount) {  // instrumentation (aiy_ws_set_timing bit 1): 64 spread slot groups
        unsigned long long* hc = A.hitcount + 4 * (item % kDiffSlots);
        if (nhits) atomicAdd(hc, (unsigned long long)nhits);
        if (lane == 0) {
            atomicAdd(hc + 1, (unsigned long long)nsup);
            atomicAdd(hc + 2, (unsigned long long)nblk);
            if (nfine) atomicAdd(hc + 3, (unsigned long long)nfine * 64 * R * (l1 - l0));
        }
    }
}

// ------------------------------------------------------------------------------ 3'. tree
// The default screened sweep.  One workgroup of W waves owns 64·R consecutive states of row i
// and searches all their candidates (every labour level, the whole feasible prefix) through a
// bound tree, then writes the final outputs itself (no per-chunk partials, no merge pass).
//   level 0: 512-candidate superblocks — bounds (Dmax512, a at the block start) fetched one
//            superblock per lane in a single round trip and read back with v_readlane
//   level 1/2: inside a passing superblock, one round trip fetches its 64 sub-block maxima
//            (Dmax8) and sub-block starts; 64-blocks are their 8-lane butterfly maxima
//   level 3: the candidates of every passing 64-block are staged in LDS together (one round
//            trip); each candidate of a passing sub-block gets the exact fp64 screen test, and
//            the candidates that pass get their exact value in the literal MATLAB order
// Every bound is t_blk = (Dmax − B)·max(c_start, 0)^n ≥ t_k for all k in the block, exactly in
// floating point (monotone rounding), so no candidate that can reach a wave's running best is
// ever skipped; the (max value, first index) merge is order-independent, hence the result
// equals the plain exhaustive scan bit for bit, whatever the split of work between waves.
// Cooperation: the W waves first split the blocks of the superblock holding the current argmax
// (best first), exchange their bests through LDS so that all hold the same near-optimal bar,
// then take the remaining superblocks round-robin; a last exchange folds the results.
// The starting bar is the hint (last sweep's argmax) and its two neighbours, or — on a cold
// start — the init kernel's candidate (best0/idx0).
// INS: the instrumented build (per-state work counters, per-item trace); the production
// instantiation compiles every counter and time stamp out
// The body of one work item (tile of row i); block_id / nblocks are the launch coordinates.
// PK > 1 (W = 1, variant bits 16-17): PK independent one-wave tiles share a workgroup (fewer
// dispatches); each wave is its own item, `lw` its LDS slice, and no workgroup barrier runs.
// HY (bell_tree_hybrid_kernel, variant bit 26): a two-wave workgroup runs either two one-wave
// tiles (PK = 2) or one heavy tile with both waves (W = 2, with the one-wave pipelines: the
// launch keeps the W = 1 register budget); s_cand / s_pass are the kernel's LDS, shared by both.
template <int NP, bool LAB, int R, int LB, int W, bool INS, int PK, bool HY = false>
__device__ __forceinline__ void bell_tree_item(const BellArgs& A0, int ntile, int block_id,
                                               int nblocks, double2 (*s_cand)[512],
                                               unsigned long long* s_pass) {
    static_assert(PK == 1 || W == 1, "packed workgroups hold one-wave tiles");
    const int lane = threadIdx.x & 63;
    const int lw = readfirst(threadIdx.x >> 6);  // this wave's LDS slice
    const int wave = PK > 1 ? 0 : lw;            // its rank among the tile's cooperating waves
    // every kernel argument the start-up reads, in one batch of scalar loads (otherwise the
    // compiler fetches them in dependent rounds as the control flow reaches each use)
    asm volatile("" ::"s"(A0.a), "s"(A0.Dt), "s"(A0.EV), "s"(A0.kf), "s"(A0.hint), "s"(A0.v_old),
                 "s"(A0.Dm512), "s"(A0.s), "s"(A0.r), "s"(A0.w), "s"(A0.N), "s"(A0.Na),
                 "s"(A0.variant), "s"(A0.C), "s"(A0.nb512), "s"(A0.sigma), "s"(A0.trace),
                 "s"(A0.best0), "s"(A0.idx0), "s"(A0.tw), "s"(ntile), "s"(nblocks), "s"(A0.mom),
                 "s"(A0.idx), "s"(A0.pk), "s"(A0.pc), "s"(A0.v_new), "s"(A0.diff));
    const long long t_boot = (INS && A0.trace) ? (long long)wall_clock64() : 0;  // (instrumentation)
    const long long c_boot = (INS && A0.trace) ? (long long)__builtin_amdgcn_s_memtime() : 0;
    int item = A0.perm ? A0.perm[block_id]
                       : ((A0.variant & 16) ? xcd_remap(block_id, nblocks) : block_id);
    if (PK > 1 && item < 0) return;  // (the last workgroup's unused slots)
    BellArgs A = A0;
    if (A0.C > 1) {  // batched candidates: blocks [c·N·ntile, (c+1)·N·ntile) are candidate c's
        const int c = item / (A0.N * ntile);
        if (A0.stop[c]) return;  // converged at an earlier sweep: its buffers stay as they are
        A = bell_cand(A0, c);
        item -= c * A0.N * ntile;
    }
    const int tile = item % ntile;
    const int i = item / ntile;
    const int N = A.N, Na = A.Na, Nl = LAB ? A.Nl : 1;  // (A1: one "labour level")
    const size_t nall = (size_t)N * Na;
    const double* __restrict__ a = A.a;
    const double* __restrict__ Drow = A.Dt + (size_t)i * Na;
    const double* __restrict__ ev = A.EV + (size_t)i * Na;
    const double y = A.w * A.s[i];
    // states per tile: 64·R, or A.tw (< 64, R = 1: lanes tw..63 idle) — see bell_tile_width
    const int TW = (R == 1 && A0.tw > 0) ? A0.tw : 64 * R;
    const int jbase = tile * TW;
    // s_cand[W·PK][512]: each wave's current superblock (a_k, D_k); s_pass[W]: (first
    // superblock, bit 12) per-wave pass masks
    // W >= 2 (cooperating waves): registers were budgeted for 5 waves per SIMD, so the staging
    // and fine-screen software pipelines (two register sets each) are off and the screen
    // stages four chains at a time; the best exchange reuses each wave's idle s_cand slice
    constexpr bool LEAN = (W >= 2 && !HY) || LAB;  // (labour: keeps 3 waves per SIMD)

    // loads that do not depend on the start-up below, issued first so that their latency
    // overlaps it: the level-0 bounds of the first 64 superblocks (first labour group) and v_old
    double dm0_pre, a0_pre;
    {
        const bool oks = lane < A.nb512;
        dm0_pre = oks ? A.Dm512[(size_t)i * A.nb512 + lane] : -__builtin_inf();
        a0_pre = oks ? a[lane << 9] : 0.0;
    }
    double vo_pre[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int j = jbase + r * 64 + lane;
        vo_pre[r] = (j < Na && r * 64 + lane < TW && wave == 0) ? A.v_old[(size_t)i * Na + j] : 0.0;
    }

    double x[R], best[R];
    int idx[R], hk0[R], mlast[R];  // mlast: the last sweep's shift (packed into mom's high half)
    bool okr[R], feas[R];
    // momentum (variant bit 9 clear): the argmax's shift over the last hinted sweep, so the
    // start-up also tries hint + shift — in the early sweeps of a solve the optimum drifts by
    // tens of candidates per sweep and a climb from the stale hint costs a dependent round
    // trip per step.  Only the screening bar depends on it, never the result.
    int* __restrict__ mom = (A.variant & 512) ? nullptr : A.mom;
    unsigned nsu = 0;  // (instrumentation) the start-up's exact evaluations: window + climb
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int j = jbase + r * 64 + lane;
        okr[r] = j < Na && r * 64 + lane < TW;
        const size_t t = (size_t)i * Na + (okr[r] ? j : 0);
        x[r] = okr[r] ? (1 + A.r) * a[j] : 0.0;
        best[r] = __builtin_nan("");
        idx[r] = -1;
        hk0[r] = -1;
        mlast[r] = 0;
        feas[r] = false;
        if (!okr[r]) continue;
        for (int l = 0; l < Nl; ++l) feas[r] = feas[r] || A.kf[l * nall + t] > 0;
        if (A.hint) {
            const int h = A.hint[t];
            // mom packs two shifts: low 16 bits the last sweep's, high 16 the one before; with
            // variant bit 21 the start extrapolates the drift linearly (2·last − previous)
            const int mraw = (mom && h >= 0) ? mom[t] : 0;
            const int ms0 = (int)(short)(mraw & 0xffff), ms1 = (int)(short)(mraw >> 16);
            mlast[r] = ms0;
            const int mv = max(-Na, min(Na, (A.variant & (1 << 21)) ? 2 * ms0 - ms1 : ms0));
            if (h >= 0) {
                const int hl = h % Nl;
                const int kf = A.kf[hl * nall + t];
                if (kf > 0) {
                    const int hk = min(h / Nl, kf - 1);
                    const double coh = cash<LAB>(x[r], y, LAB ? A.L[hl] : 1.0);
                    const double dis = LAB ? A.dis[hl] : 0.0;
                    auto take = [&](int k) __attribute__((always_inline)) {
                        if (INS) ++nsu;
                        return lexi_take(bell_val<NP, LAB>(coh - a[k], ev[k], A.sigma, dis),
                                         hl + Nl * k, best[r], idx[r]);
                    };
                    // Window: the hint and its wn neighbours on each side (wn = 1, 2, 4 or 8:
                    // variant bits 7-8), all loads in flight together, then their exact values
                    // (independent chains).  Indices are clamped into the feasible prefix; a
                    // repeated candidate merges as a no-op.
                    const int wn = 1 << ((A.variant >> 7) & 3);
                    hk0[r] = hk;
                    // the extrapolated start hm = hint + last shift and its two neighbours,
                    // when that window does not touch the hint's own
                    const int hm = min(max(hk + mv, 0), kf - 1);
                    // bit 23: when the extrapolated window is used, the hint's window is the
                    // hint alone (the drift predictor is usually right: three fewer evaluations)
                    constexpr int mw = 1;
                    const bool usem = hm > hk + wn + mw || hm < hk - wn - mw;
                    const int wnh = (usem && (A.variant & (1 << 23))) ? 0 : wn;
                    // bit 24 (with 23): not even the hint itself — the extrapolated window
                    // and the climb from it carry the start alone
                    const bool skiph = usem && (A.variant & (1 << 24));
                    constexpr int WM = 8;
                    double wa[2 * WM + 1], we[2 * WM + 1], ma[3], me[3];
#pragma unroll
                    for (int d = -WM; d <= WM; ++d) {
                        if (d < -wnh || d > wnh || skiph) continue;  // (per lane: bits 23-24)
                        const int kc = min(max(hk + d, 0), kf - 1);
                        wa[d + WM] = a[kc];
                        we[d + WM] = ev[kc];
                    }
                    if (usem) {
#pragma unroll
                        for (int d = -1; d <= 1; ++d) {
                            const int kc = min(max(hm + d, 0), kf - 1);
                            ma[d + 1] = a[kc];
                            me[d + 1] = ev[kc];
                        }
                    }
#pragma unroll
                    for (int d = -WM; d <= WM; ++d) {
                        if (d < -wnh || d > wnh || skiph) continue;
                        const int kc = min(max(hk + d, 0), kf - 1);
                        if (INS) ++nsu;
                        lexi_take(bell_val<NP, LAB>(coh - wa[d + WM], we[d + WM], A.sigma, dis),
                                  hl + Nl * kc, best[r], idx[r]);
                    }
                    if (usem) {
#pragma unroll
                        for (int d = -1; d <= 1; ++d) {
                            const int kc = min(max(hm + d, 0), kf - 1);
                            if (INS) ++nsu;
                            lexi_take(bell_val<NP, LAB>(coh - ma[d + 1], me[d + 1], A.sigma, dis),
                                      hl + Nl * kc, best[r], idx[r]);
                        }
                    }
                    // Climb: when the best of the window sits on its edge, the optimum has moved
                    // further (early sweeps; the sweep after a cold start moves it by thousands
                    // of candidates).  Doubling steps while the value improves, then halving
                    // steps around the best point: for a unimodal objective this lands on the
                    // maximiser in O(log distance) exact evaluations instead of the tree raising
                    // the bar one passing candidate at a time.  Any candidate is a valid bar, so
                    // the result does not depend on it (the tree below still proves the maximum).
                    const int kb = idx[r] >= 0 ? idx[r] / Nl : hk;
                    int dir = kb >= hk + wnh ? 1 : (kb <= hk - wnh ? -1 : 0);
                    if (usem && kb >= hm - mw && kb <= hm + mw)  // best in the extrapolated window
                        dir = kb == hm + mw ? 1 : (kb == hm - mw ? -1 : 0);
                    if (dir != 0 && !(A.variant & 32)) {
                        int k = kb, step = 2;
                        for (;;) {
                            const int kn = min(max(k + dir * step, 0), kf - 1);
                            if (kn == k || !take(kn)) break;
                            k = kn;
                            step <<= 1;
                        }
                        for (int s2 = step >> 1; s2 >= 1; s2 >>= 1) {
                            const int c0 = idx[r] / Nl;
                            if (c0 + s2 < kf) take(c0 + s2);
                            if (c0 - s2 >= 0) take(c0 - s2);
                        }
                    }
                }
            }
        } else {
            best[r] = A.best0[t];
            idx[r] = A.idx0[t] == -2 ? -1 : A.idx0[t];
        }
    }
    // the start-up's argmax and its a_k, loaded now: the output needs a(argmax) for policy_k,
    // and the tree rarely moves the argmax once the start-up has climbed to it, so the output
    // phase usually skips that dependent load (it reloads when some lane's argmax moved)
    int q_su[R];
    double kp_su[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        q_su[r] = idx[r];
        kp_su[r] = a[idx[r] >= 0 ? idx[r] / Nl : 0];
    }
    // nhits counts every exact evaluation of the launch: the start-up's (hint window,
    // extrapolated window, climb) and the screen's (VERDICT r4 "do this" 1)
    unsigned nhits = nsu, nsup = 0, nblk = 0, nfine = 0, lane_pairs = 0;
    const long long t_start = (INS && A.trace) ? (long long)wall_clock64() : 0;
    // phase cycle counters (trace mode): startup, superblock() calls, fine screens, exact paths
    long long cyc[4] = {0, 0, 0, 0}, c_mark = (INS && A.trace) ? (long long)__builtin_amdgcn_s_memtime() : 0;
    const long long c_mark0 = c_mark;
    auto stamp = [&](int ph) __attribute__((always_inline)) {
        if (INS && A.trace) {
            const long long now = (long long)__builtin_amdgcn_s_memtime();
            cyc[ph] += now - c_mark;
            c_mark = now;
        }
    };
    stamp(0);

    // every wave leaves with the (max value, first index) of all waves' bests
    auto exchange = [&]() __attribute__((always_inline)) {
        if constexpr (W > 1) {
#pragma unroll
            for (int r = 0; r < R; ++r)  // (index exact as a double)
                s_cand[lw][r * 64 + lane] = make_double2(best[r], (double)idx[r]);
            __syncthreads();
            for (int v = 0; v < W; ++v)
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const double2 e = s_cand[v][r * 64 + lane];
                    if (v != wave && (int)e.y >= 0) lexi_take(e.x, (int)e.y, best[r], idx[r]);
                }
            __syncthreads();
        }
    };

    for (int l0 = 0; l0 < Nl; l0 += LB) {  // labour levels in groups of LB sub-states per lane
        double coh[R][LB], B[R][LB], dis[LB];
        int kg = 0;  // the group's feasible range over the tile (identical in every wave)
#pragma unroll
        for (int q = 0; q < LB; ++q) dis[q] = (LAB && l0 + q < Nl) ? A.dis[l0 + q] : 0.0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const size_t t = (size_t)i * Na + (okr[r] ? jbase + r * 64 + lane : 0);
#pragma unroll
            for (int q = 0; q < LB; ++q) {
                const bool okq = okr[r] && l0 + q < Nl;
                coh[r][q] = okq ? cash<LAB>(x[r], y, LAB ? A.L[l0 + q] : 1.0) : 0.0;
                if (okq) kg = max(kg, A.kf[(l0 + q) * nall + t]);
            }
        }
        if (A.r > -1.0) {
            // coh is increasing in j when 1 + r > 0, so every feasible prefix kf is
            // non-decreasing along the tile: the maximum sits in the last valid lane
            const int jl = min(Na - 1, jbase + TW - 1);  // the tile's last state
            kg = readlane_i(kg, (jl - jbase) & 63);
        } else {
            for (int off = 32; off > 0; off >>= 1) kg = max(kg, __shfl_xor(kg, off));
            kg = readfirst(kg);
        }
        if (kg == 0) continue;
        if (l0 > 0) exchange();  // the previous group left per-wave bests
        auto set_B = [&]() __attribute__((always_inline)) {
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int q = 0; q < LB; ++q)  // invalid sub-states: NaN bar, every test false
                    B[r][q] = (okr[r] && l0 + q < Nl) ? screen_B(best[r], idx[r], dis[q], NP)
                                                      : __builtin_nan("");
        };
        set_B();

        // eight block bounds at once (independent dependency chains, so their latencies
        // overlap): lanes l0 + stride*u of (dv, av) hold (Dmax, a at the block start); bit u
        // of the result is set when some sub-state passes bound u (u < cnt)
        constexpr int RL = R * LB, G = LEAN ? (RL <= 2 ? 4 : 1) : StageGroup<RL>::G;
        auto mask8 = [&](double dv, double av, int l0, int stride, int cnt, bool sub = false)
                         __attribute__((always_inline)) {
            double dmax[8], a0[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int ln = min(l0 + stride * u, 63);
                dmax[u] = readlane_d(dv, ln);
                a0[u] = readlane_d(av, ln);
            }
            bool pu[8];
#pragma unroll
            for (int g0 = 0; g0 < 8; g0 += G) {
                double cx[G * RL], dd[G * RL], t[G * RL];
#pragma unroll
                for (int gu = 0; gu < G; ++gu)
#pragma unroll
                    for (int r = 0; r < R; ++r)
#pragma unroll
                        for (int q = 0; q < LB; ++q) {
                            const int m = (gu * R + r) * LB + q;
                            cx[m] = coh[r][q] - a0[g0 + gu];
                            dd[m] = dmax[g0 + gu] - B[r][q];
                        }
                AIY_SCHED_BARRIER();
                screen_t<NP, G * RL>(t, cx, dd);
#pragma unroll
                for (int gu = 0; gu < G; ++gu) {
                    bool pass = false;
#pragma unroll
                    for (int m = gu * RL; m < (gu + 1) * RL; ++m) pass = pass || t[m] >= kThr;
                    pu[g0 + gu] = pass;
                }
            }
            unsigned m = 0;
#pragma unroll
            for (int u = 0; u < 8; ++u) m |= (__any(pu[u]) ? 1u : 0u) << u;
            if (INS && A.trace && sub)  // (instrumentation) this lane's own passing sub-blocks
#pragma unroll
                for (int u = 0; u < 8; ++u) lane_pairs += (u < cnt && pu[u]) ? 1u : 0u;
            return m & ((1u << cnt) - 1u);
        };
        // candidates [k0, k1), k1 - k0 <= 8, of superblock sbase staged in LDS.  The exact
        // screen test on all of them without a branch (the current argmax itself is masked:
        // its value is known) gives one vote per candidate; only voted candidates take the
        // exact path: re-test per lane, exact value in the literal MATLAB order, merge
        // the eight staged candidates of 8-block `bit` (broadcast LDS reads, all in flight);
        // the whole 64-block is staged, candidates past the feasible range are masked by fine()
        auto load_tk = [&](int bit, double2 (&tk)[8]) __attribute__((always_inline)) {
#pragma unroll
            for (int kk = 0; kk < 8; ++kk) tk[kk] = s_cand[lw][(bit << 3) + kk];
        };
        auto fine = [&](int sbase, int k0, int k1, const double2 (&tk)[8])
                        __attribute__((always_inline)) {
            if (INS && (A.hitcount || A.trace)) nfine += k1 - k0;
            bool pk[8];
#pragma unroll
            for (int g0 = 0; g0 < 8; g0 += G) {
                double cx[G * RL], dd[G * RL], t[G * RL];
#pragma unroll
                for (int gk = 0; gk < G; ++gk)
#pragma unroll
                    for (int r = 0; r < R; ++r)
#pragma unroll
                        for (int q = 0; q < LB; ++q) {
                            const int m = (gk * R + r) * LB + q;
                            cx[m] = coh[r][q] - tk[g0 + gk].x;
                            dd[m] = tk[g0 + gk].y - B[r][q];
                        }
                AIY_SCHED_BARRIER();
                screen_t<NP, G * RL>(t, cx, dd);
#pragma unroll
                for (int gk = 0; gk < G; ++gk) {
                    bool pass = false;
#pragma unroll
                    for (int r = 0; r < R; ++r)
#pragma unroll
                        for (int q = 0; q < LB; ++q) {
                            const int lin = (l0 + q) + Nl * (k0 + g0 + gk);
                            pass = pass || (t[(gk * R + r) * LB + q] >= kThr && lin != idx[r]);
                        }
                    pk[g0 + gk] = pass;
                }
            }
            {  // one wave vote first: almost always no candidate passes
                bool pall = false;
#pragma unroll
                for (int kk = 0; kk < 8; ++kk) pall = pall || pk[kk];
                if (!__any(pall)) return;
            }
            unsigned vote = 0;
#pragma unroll
            for (int kk = 0; kk < 8; ++kk) vote |= (__any(pk[kk]) ? 1u : 0u) << kk;
            vote &= (1u << (k1 - k0)) - 1u;
            if (!vote) return;
            stamp(2);
            while (vote) {
                const int kk = __builtin_ctz(vote);
                vote &= vote - 1;
                const int k = k0 + kk;
                const double2 tkk = s_cand[lw][k - sbase];
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int q = 0; q < LB; ++q) {
                        const double c = coh[r][q] - tkk.x;
                        const int lin = (l0 + q) + Nl * k;
                        if (lin != idx[r] && c > 0 &&
                            (tkk.y - B[r][q]) * aiy_ipow(c, NP) >= kThr) {
                            ++nhits;
                            const double val =
                                bell_val<NP, LAB>(c, ev[k], A.sigma, dis[q]);
                            if (lexi_take(val, lin, best[r], idx[r])) {
#pragma unroll
                                for (int q2 = 0; q2 < LB; ++q2)
                                    if (B[r][q2] == B[r][q2])
                                        B[r][q2] = screen_B(best[r], idx[r], dis[q2], NP);
                            }
                        }
                    }
            }
            stamp(3);
        };
        // one superblock, blocks b with b % bstep == bsel: one round trip for the 64 sub-block
        // bounds, then all bound tests (v_readlane, no memory), then ONE round trip staging the
        // candidates of every passing block in LDS
        // the 64 sub-block bounds of superblock sb, one per lane (issued ahead of their use)
        auto load8 = [&](int sb, double& dm8, double& a8) __attribute__((always_inline)) {
            const int sub = (sb << 6) + lane;
            const bool oku = sub < A.nb8;
            dm8 = oku ? A.Dm8[(size_t)i * A.nb8 + sub] : -__builtin_inf();
            a8 = oku ? a[sub << 3] : 0.0;
        };
        // one superblock, blocks b with b % bstep == bsel, in two halves.  prep: the bound tests
        // of its 64-blocks and 8-blocks (v_readlane of the sub-block bounds, no memory) and the
        // loads of the candidates of every passing 64-block into registers.  finish: those
        // registers to LDS, then the fine screen of every passing 8-block.  The main loop runs
        // prep of superblock n+1 before finish of superblock n, so the candidate loads of n+1
        // are in flight while n is screened (a bar raised by n's exact path only makes n+1's
        // bound tests, done against the older bar, pass more: never fewer candidates).
        auto prep = [&](int sb, int bsel, int bstep, double dm8, double a8, double2 (&st)[8],
                        bool subsplit = false)
                        __attribute__((always_inline)) -> unsigned long long {
            stamp(0);
            const int sbase = sb << 9;  // first candidate of the superblock
            // 64-block maxima at lanes 8b (the only lanes read): lane ^ 1, lane ^ 2, lane + 4
            double dm64 = dm8;
            dm64 = fmax(dm64, dpp_d<0xB1>(dm64));
            dm64 = fmax(dm64, dpp_d<0x4E>(dm64));
            dm64 = fmax(dm64, dpp_d<0x104>(dm64));
            // blocks inside the feasible range and owned by this wave.  subsplit: every wave
            // bound-tests every block and keeps the passing 8-blocks i with i % bstep == bsel —
            // the passing 8-blocks cluster around the optima, so a split by 64-block leaves
            // one wave with most of the fine screens and the others waiting at the exchange
            const int nblock = min(8, (kg - sbase + 63) >> 6);
            unsigned own = 0;
            for (int b = subsplit ? 0 : bsel; b < nblock; b += subsplit ? 1 : bstep) own |= 1u << b;
            if (INS && (A.hitcount || A.trace)) nblk += __builtin_popcount(own);
            const unsigned bpass = mask8(dm64, a8, 0, 8, nblock) & own;
            unsigned long long pass = 0;  // bit 8b+u: sub-block u of block b passes
            const bool deal = subsplit && bstep > 1;
            int ord = 0;
            for (unsigned bm = bpass; bm; bm &= bm - 1, ++ord) {
                // deal: the passing 64-blocks' 8-block tests go round-robin over the waves too
                if (deal && ord % bstep != bsel) continue;
                const int b = __builtin_ctz(bm);
                const int nsub = min(8, (kg - (sbase + (b << 6)) + 7) >> 3);
                if (INS && (A.hitcount || A.trace)) nblk += nsub;
                pass |= (unsigned long long)mask8(dm8, a8, 8 * b, 1, nsub, true) << (8 * b);
            }
            if constexpr (W > 1) {
                if (deal) {  // the union of the waves' masks, then 8-blocks bsel, bsel + W, ...
                    s_pass[bsel] = pass;
                    __syncthreads();
                    unsigned long long all = 0;
                    for (int v = 0; v < bstep; ++v) all |= s_pass[v];
                    __syncthreads();
                    const unsigned long long pat = bstep == 2 ? 0x5555555555555555ull
                                                 : (bstep == 4 ? 0x1111111111111111ull
                                                               : 0x0101010101010101ull);
                    pass = all & (pat << bsel);
                }
            }
            if constexpr (LEAN) {
                // no register set for all eight: the passing 64-blocks two at a time, both
                // loads issued before either LDS write (a load and its write in one guarded
                // block would cost one L2 round trip per block)
                unsigned bm = 0;
#pragma unroll
                for (int b = 0; b < 8; ++b) bm |= ((pass >> (8 * b)) & 0xffull) ? 1u << b : 0u;
                while (bm) {
                    const int b0 = __builtin_ctz(bm);
                    bm &= bm - 1;
                    const int b1 = bm ? __builtin_ctz(bm) : -1;
                    if (bm) bm &= bm - 1;
                    const int k0 = min(sbase + (b0 << 6) + lane, Na - 1);
                    const double2 v0 = make_double2(a[k0], Drow[k0]);
                    double2 v1 = make_double2(0.0, 0.0);
                    if (b1 >= 0) {
                        const int k1 = min(sbase + (b1 << 6) + lane, Na - 1);
                        v1 = make_double2(a[k1], Drow[k1]);
                    }
                    s_cand[lw][(b0 << 6) + lane] = v0;
                    if (b1 >= 0) s_cand[lw][(b1 << 6) + lane] = v1;
                }
            } else {
#pragma unroll
                for (int b = 0; b < 8; ++b)  // all loads issued before any is used
                    if ((pass >> (8 * b)) & 0xffull) {
                        const int k = min(sbase + (b << 6) + lane, Na - 1);
                        st[b] = make_double2(a[k], Drow[k]);
                    }
            }
            stamp(1);
            return pass;
        };
        auto finish = [&](int sb, unsigned long long pass, const double2 (&st)[8])
                          __attribute__((always_inline)) {
            const int sbase = sb << 9;
            if constexpr (!LEAN)
#pragma unroll
                for (int b = 0; b < 8; ++b)
                    if ((pass >> (8 * b)) & 0xffull) s_cand[lw][(b << 6) + lane] = st[b];
            __builtin_amdgcn_wave_barrier();  // a wave reads only its own slice
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            stamp(1);
            // the next 8-block's candidates are read from LDS while this one is screened (two
            // register sets, unrolled by two: no copies)
            double2 tkA[8], tkB[8];
            unsigned long long pm = pass;
            if constexpr (LEAN) {
                for (; pm; pm &= pm - 1) {
                    const int b0 = __builtin_ctzll(pm);
                    load_tk(b0, tkA);
                    fine(sbase, sbase + (b0 << 3), min(sbase + (b0 << 3) + 8, kg), tkA);
                }
            }
            if (pm) load_tk(__builtin_ctzll(pm), tkA);
            while (pm) {
                const int b0 = __builtin_ctzll(pm);
                pm &= pm - 1;
                if (pm) load_tk(__builtin_ctzll(pm), tkB);
                fine(sbase, sbase + (b0 << 3), min(sbase + (b0 << 3) + 8, kg), tkA);
                if (!pm) break;
                const int b1 = __builtin_ctzll(pm);
                pm &= pm - 1;
                if (pm) load_tk(__builtin_ctzll(pm), tkA);
                fine(sbase, sbase + (b1 << 3), min(sbase + (b1 << 3) + 8, kg), tkB);
            }
            stamp(2);
            __builtin_amdgcn_wave_barrier();  // reads done before the next superblock's writes
        };

        const int nsb = (kg + 511) >> 9;
        // best first: the superblock holding the tile's current argmax, its blocks split over
        // the waves; then one exchange gives every wave the same near-optimal bar
        int sfirst = -1;
        {
            int hk = -1;
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (idx[r] >= 0) hk = idx[r] / Nl;
            const unsigned long long m = __ballot(hk >= 0);
            if (m) sfirst = min(readlane_i(hk, __builtin_ctzll(m)) >> 9, nsb - 1);
        }
        double2 st_cur[8], st_prev[8];
        if (sfirst >= 0) {  // (its bound would pass: it holds the bar's candidate)
            if (INS) ++nsup;
            double d8, a8;
            load8(sfirst, d8, a8);
            const unsigned long long p = prep(sfirst, wave, W, d8, a8, st_cur,
                                              (A.variant & 4096) != 0);
            if (p) finish(sfirst, p, st_cur);
            exchange();
            set_B();
        }
        // level-0 bounds of the first 64 superblocks
        double dm0, a0;
        auto load512 = [&](int g) __attribute__((always_inline)) {
            const int sbl = g + lane;
            const bool oks = sbl < nsb;
            dm0 = oks ? A.Dm512[(size_t)i * A.nb512 + sbl] : -__builtin_inf();
            a0 = oks ? a[sbl << 9] : 0.0;
        };
        if (l0 == 0) {  // prefetched (lanes past nsb are masked by the bound counts below)
            dm0 = dm0_pre;
            a0 = a0_pre;
        } else {
            load512(0);
        }
        // the passing superblocks in order: level-0 tests eight at a time, on demand
        int g = 0, s8 = -8;
        unsigned sm = 0;
        auto next_sb = [&]() __attribute__((always_inline)) -> int {
            for (;;) {
                if (sm) {
                    const int u = __builtin_ctz(sm);
                    sm &= sm - 1;
                    return g + s8 + u;
                }
                s8 += 8;
                if (s8 >= min(64, nsb - g)) {
                    g += 64;
                    s8 = 0;
                    if (g >= nsb) return -1;
                    load512(g);
                }
                const int cnt = min(8, min(64, nsb - g) - s8);
                unsigned own = 0;
                for (int u = 0; u < cnt; ++u) {
                    const int sb = g + s8 + u;
                    if (sb != sfirst && sb % W == wave) own |= 1u << u;
                }
                if (!own) continue;
                if (INS) nsup += __builtin_popcount(own);
                sm = mask8(dm0, a0, s8, 1, cnt) & own;
            }
        };
        // software pipeline: load8 two superblocks ahead, the candidate loads one ahead
        int cur = nsb > 0 ? next_sb() : -1;
        double pd = 0.0, pa = 0.0;
        if (cur >= 0) load8(cur, pd, pa);
        unsigned long long pass_prev = 0;
        int sb_prev = -1;
        while (cur >= 0) {
            const double d8 = pd, a8 = pa;
            const int nxt = next_sb();
            if (nxt >= 0) load8(nxt, pd, pa);
            const unsigned long long pc = prep(cur, 0, 1, d8, a8, st_cur);
            if constexpr (LEAN) {  // staged straight to LDS: screen it now
                if (pc) finish(cur, pc, st_cur);
                cur = nxt;
                continue;
            }
            if (pass_prev) finish(sb_prev, pass_prev, st_prev);
#pragma unroll
            for (int b = 0; b < 8; ++b) st_prev[b] = st_cur[b];
            pass_prev = pc;
            sb_prev = cur;
            cur = nxt;
        }
        if (pass_prev) finish(sb_prev, pass_prev, st_prev);
    }

    exchange();
    const long long c_end = (INS && A.trace) ? (long long)__builtin_amdgcn_s_memtime() : 0;

    // final outputs, wave 0 (the merge kernel's rules: Aiyagari_VFI.m:79-81,
    // Labor_VFI.m:85,106-109)
    bool okd = false;
    double dmax = 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (!okr[r] || wave != 0) continue;
        const size_t t = (size_t)i * Na + jbase + r * 64 + lane;
        double b = best[r];
        int q = idx[r];
        const double vo = vo_pre[r];
        if (!feas[r] && LAB) {
            b = A.keep_incoming ? A.v_new[t] : vo;
        } else {
            if (q < 0) {  // all candidates NaN: max returns NaN at index 1
                q = 0;
                b = __builtin_nan("");
            }
            const int l = q % Nl, k = q / Nl;
            double kp = kp_su[r];
            if (__ballot(q != q_su[r]) != 0ull) kp = a[k];  // (wave-uniform: usually skipped)
            A.idx[t] = q;
            if (A.pk) A.pk[t] = kp;
            if (A.pc) A.pc[t] = cash<LAB>(x[r], y, LAB ? A.L[l] : 1.0) - kp;
            if (LAB && A.pl) A.pl[t] = A.L[l];
        }
        A.v_new[t] = b;
        if (mom && A.hint) {  // this sweep's shift of the argmax, for the next sweep's start
            const int sh = (hk0[r] >= 0 && idx[r] >= 0) ? idx[r] / Nl - hk0[r] : 0;
            const int shc = max(-32767, min(32767, sh));
            mom[t] = (int)(((unsigned)shc & 0xffffu) | ((unsigned)mlast[r] << 16));
        }
        const double d = fabs(b - vo);
        if (d == d) {
            dmax = okd ? fmax(dmax, d) : d;
            okd = true;
        }
    }
    if constexpr (W == 1) wave_max_to_slots(okd, dmax, A.diff);
    else block_max_to_slots(okd, dmax, A.diff);
    if (INS && A.trace) {  // instrumentation (aiy_ws_set_timing bit 2): per-wave sums into wave 0
        __shared__ unsigned s_cnt[W][4];
        __shared__ unsigned s_pairs;
        unsigned pairs = lane_pairs, sums[4] = {nsup, nblk, nfine, nhits};
        if constexpr (W == 1) {  // one wave: a shuffle sum, no barrier (packed workgroups)
            for (int o = 32; o > 0; o >>= 1) pairs += __shfl_xor(pairs, o);
        } else {
            if (threadIdx.x == 0) s_pairs = 0;
            __syncthreads();
            atomicAdd(&s_pairs, lane_pairs);
            if (lane == 0) {
                s_cnt[wave][0] = nsup; s_cnt[wave][1] = nblk; s_cnt[wave][2] = nfine; s_cnt[wave][3] = nhits;
            }
            __syncthreads();
            pairs = s_pairs;
            for (int c = 0; c < 4; ++c) {
                unsigned sum = 0;
                for (int v = 0; v < W; ++v) sum += s_cnt[v][c];
                sums[c] = sum;
            }
        }
        if (W == 1 ? lane == 0 : threadIdx.x == 0) {
            long long* tr = A.trace + 16 * (size_t)item;
            tr[0] = t_start;
            tr[1] = (long long)wall_clock64();
            // HW_REG_XCC_ID (bits 0-31) | HW_REG_HW_ID << 32 (wave, SIMD, CU, SH, SE of this wave)
            tr[2] = (long long)(unsigned)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11)) |
                    ((long long)(unsigned)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11))
                     << 32);
            for (int c = 0; c < 4; ++c) tr[3 + c] = sums[c];
            tr[7] = block_id;
            for (int c = 0; c < 4; ++c) tr[8 + c] = cyc[c];
            tr[12] = t_boot;                                   // kernel entry (wall clock)
            tr[13] = c_mark0 - c_boot;                         // start-up cycles (hint, climb)
            tr[14] = (long long)__builtin_amdgcn_s_memtime() - c_end;  // output cycles
            tr[15] = pairs;  // (state, sub-block) pairs passing the 8-block bound
        }
    }
    if (INS && A.hitcount) {  // instrumentation (aiy_ws_set_timing bit 1)
        unsigned long long* hc = A.hitcount + 4 * (blockIdx.x % kDiffSlots);
        if (nhits) atomicAdd(hc, (unsigned long long)nhits);
        if (lane == 0) {
            const unsigned long long ns = 64ull * R * LB;
            atomicAdd(hc + 1, nsup * ns);
            atomicAdd(hc + 2, nblk * ns);
            if (nfine) atomicAdd(hc + 3, nfine * ns);
        }
    }
}

template <int NP, bool LAB, int R, int LB, int W, bool INS, int PK>
// min waves per SIMD 3 (168 VGPRs): every item of Na = 20,000 is resident at W = 1; the
// cooperative tiles (W >= 2) serve small grids and labour, where a few hundred waves run and
// latency, not occupancy, bounds them — a budget of 5 (and of 4) made those builds spill
__global__ __launch_bounds__(64 * W * PK, 3) void bell_tree_kernel(BellArgs A0, int ntile) {
    __shared__ double2 s_cand[W * PK][512];
    __shared__ unsigned long long s_pass[W];
    const int lw = PK > 1 ? readfirst(threadIdx.x >> 6) : 0;
    bell_tree_item<NP, LAB, R, LB, W, INS, PK>(A0, ntile, (int)blockIdx.x * PK + lw,
                                               (int)gridDim.x * PK, s_cand, s_pass);
}

// Heavy tiles on two waves (variant bit 26, A1 with a dispatch permutation): workgroup b holds
// perm[2b], perm[2b + 1]; perm[2b + 1] == -2 marks a cooperative tile (both waves on perm[2b]),
// otherwise the two slots are one-wave tiles as in the packed launch (PK = 2).  ws_tree_perm
// picks the heaviest tiles of each XCD's range for the cooperative workgroups and deals them
// first.  Work split only: the (max value, first index) merge makes the result identical.
template <int NP, bool INS>
__global__ __launch_bounds__(128, 3) void bell_tree_hybrid_kernel(BellArgs A0, int ntile) {
    __shared__ double2 s_cand[2][512];
    __shared__ unsigned long long s_pass[2];
    const int b = (int)blockIdx.x;
    if (A0.perm[2 * b + 1] == -2) {
        bell_tree_item<NP, false, 1, 1, 2, INS, 1, true>(A0, ntile, 2 * b, 2 * (int)gridDim.x,
                                                        s_cand, s_pass);
    } else {
        const int lw = readfirst(threadIdx.x >> 6);
        bell_tree_item<NP, false, 1, 1, 1, INS, 2, true>(A0, ntile, 2 * b + lw,
                                                        2 * (int)gridDim.x, s_cand, s_pass);
    }
}

// ------------------------------------------------------------------------------ 4. merge
template <int NP, bool LAB, int LB>
__global__ void bell_merge_kernel(BellArgs A, int use_partial, int nlb, int nchunk) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    bool ok = false;
    double d = 0.0;
    const int N = A.N, Na = A.Na, Nl = A.Nl;
    if (t < N * Na) {
        int i = t / Na, j = t - i * Na;
        const double* __restrict__ a = A.a;
        double x = (1 + A.r) * a[j];
        double y = A.w * A.s[i];
        double best = A.best0[t];
        int idx = A.idx0[t];
        if (use_partial && A.touched[t]) {
            A.touched[t] = 0;
            const double* __restrict__ ev = A.EV + (size_t)i * Na;
            for (int lbk = 0; lbk < nlb; ++lbk) {
                int kfm = 0;
                for (int l = lbk * LB; l < min(lbk * LB + LB, Nl); ++l)
                    kfm = max(kfm, A.kf[(size_t)l * N * Na + t]);
                int nch = (kfm + A.CK - 1) / A.CK;
                for (int c = 0; c < nch; ++c) {
                    int* pq = A.partial + (((size_t)lbk * nchunk + c) * N + i) * Na + j;
                    int q = *pq;
                    if (q >= 0) {
                        *pq = -1;
                        int l = q % Nl, k = q / Nl;
                        double coh = cash<LAB>(x, y, LAB ? A.L[l] : 1.0);
                        lexi_take(bell_val<NP, LAB>(coh - a[k], ev[k], A.sigma,
                                                    LAB ? A.dis[l] : 0.0),
                                  q, best, idx);
                    }
                }
            }
        }
        double vo = A.v_old[t];
        if (idx == -2 && LAB) {
            // Labor_VFI.m:85: no feasible choice → v_new keeps its value: the incoming v_new
            // on a first sweep, == v_old on later sweeps of a solve (:120 v_old = v_new)
            best = A.keep_incoming ? A.v_new[t] : vo;
        } else {
            if (idx < 0) {  // all candidates NaN: max returns NaN at index 1
                idx = 0;
                best = __builtin_nan("");
            }
            int l = idx % Nl, k = idx / Nl;
            double kp = a[k];
            double coh = cash<LAB>(x, y, LAB ? A.L[l] : 1.0);
            A.idx[t] = idx;
            if (A.pk) A.pk[t] = kp;
            if (A.pc) A.pc[t] = coh - kp;
            if (LAB && A.pl) A.pl[t] = A.L[l];
        }
        A.v_new[t] = best;
        d = fabs(best - vo);
        ok = (d == d);
    }
    block_max_to_slots(ok, d, A.diff);
}

// ------------------------------------------------------------------------------ plain
template <int NP, bool LAB>
__global__ __launch_bounds__(256) void bell_plain_kernel(BellArgs A) {
    // The exhaustive scan (mode 2, or variant bit 10): every feasible candidate evaluated
    // exactly, writing the sweep's outputs itself (no init or merge launch), in the literal
    // MATLAB order, merged with the (max value, first column-major index) rule.  A block owns
    // 64 consecutive states of one row (one per lane) and its four waves split the candidate
    // range into quarters (four times the waves of one wave per tile: the scan is bound by
    // dependent fp64 divisions, so it needs the occupancy); the candidate index is
    // wave-uniform, so a_k and EV_ik arrive by scalar loads, and each lane evaluates 8
    // candidates per step as independent chains before merging them.  The quarters' partial
    // maxima are merged through LDS; the merge rule is order-independent, so the result is the
    // sequential scan's bit for bit.
    constexpr int W = 4, U = 8;
    __shared__ double s_best[W][64];
    __shared__ int s_idx[W][64];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int Na = A.Na, Nl = A.Nl;
    const int i = blockIdx.y;
    const int j = blockIdx.x * 64 + lane;
    const bool okj = j < Na;
    const size_t t = (size_t)i * Na + (okj ? j : 0);
    const double* __restrict__ a = A.a;
    const double* __restrict__ ev = A.EV + (size_t)i * Na;
    const double x = okj ? (1 + A.r) * a[j] : 0.0, y = A.w * A.s[i];
    double best = __builtin_nan("");
    int idx = -1;
    bool anyfeas = false;
    for (int l = 0; l < Nl; ++l) {
        const double coh = cash<LAB>(x, y, LAB ? A.L[l] : 1.0);
        const double dis = LAB ? A.dis[l] : 0.0;
        const int kf = okj ? A.kf[(size_t)l * A.N * Na + t] : 0;
        anyfeas = anyfeas || kf > 0;
        int km = kf;
        for (int off = 32; off > 0; off >>= 1) km = max(km, __shfl_xor(km, off));
        const int kmax = __builtin_amdgcn_readfirstlane(km);
        const int kc = (kmax + W * U - 1) / (W * U) * U;  // quarter length, a multiple of U
        const int k_lo = wave * kc, k_hi = min(kmax, k_lo + kc);
        for (int k = k_lo; k < k_hi; k += U) {
            double v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int kk = min(k + u, Na - 1);
                const double val = bell_val<NP, LAB>(coh - a[kk], ev[kk], A.sigma, dis);
                v[u] = (k + u < kf) ? val : __builtin_nan("");
            }
            AIY_SCHED_BARRIER();
#pragma unroll
            for (int u = 0; u < U; ++u) lexi_take_sel(v[u], l + Nl * (k + u), best, idx);
        }
    }
    s_best[wave][lane] = best;
    s_idx[wave][lane] = idx;
    __syncthreads();
    // wave 0 writes the sweep's outputs (the merge kernel's rules: Aiyagari_VFI.m:79-81,
    // Labor_VFI.m:85,106-109) and the block's max|v_new - v_old|
    bool okd = false;
    double dd = 0.0;
    if (wave == 0 && okj) {
#pragma unroll
        for (int w = 1; w < W; ++w) lexi_take(s_best[w][lane], s_idx[w][lane], best, idx);
        const double vo = A.v_old[t];
        if (!anyfeas && LAB) {  // no feasible (l, a'): v_new keeps its value (:85)
            best = A.keep_incoming ? A.v_new[t] : vo;
        } else {
            if (idx < 0) {  // all candidates NaN: max returns NaN at index 1
                idx = 0;
                best = __builtin_nan("");
            }
            const int l = idx % Nl, k = idx / Nl;
            const double kp = a[k];
            A.idx[t] = idx;
            if (A.pk) A.pk[t] = kp;
            if (A.pc) A.pc[t] = cash<LAB>(x, y, LAB ? A.L[l] : 1.0) - kp;
            if (LAB && A.pl) A.pl[t] = A.L[l];
        }
        A.v_new[t] = best;
        dd = fabs(best - vo);
        okd = dd == dd;
    }
    block_max_to_slots(okd, dd, A.diff);
}

// ------------------------------------------------------------------------------ launchers
static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

thread_local DispatchEvents g_dispatch_ev;  // (dispatch.hpp)

int launch_bell_ev_mfma(const BellArgs& A, hipStream_t st) {
    const dim3 grid(cdiv(A.Na, 64), cdiv(A.N, 16), std::max(A.C, 1));
    bell_ev_mfma_kernel<<<grid, 256, 0, st>>>(A.N, A.Na, A.P, A.v_old, A.beta, A.EV,
                                              A.C > 1 ? A.stop : nullptr);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}

int launch_bell_table(const BellArgs& A, hipStream_t st) {
    static_assert(2 * kDiffSlots <= kTableBlock, "table block clears the diff slots");
    dim3 grid(cdiv(A.Na, kTableBlock), A.N);
    const bool scr = A.np > 0;
    if (A.ev_mfma) AIY_TRY(launch_bell_ev_mfma(A, st));
    bell_table_kernel<<<grid, kTableBlock, 0, st>>>(
        A.N, A.Na, A.P, A.v_old, A.beta, A.np, A.a, A.EV, (scr && !A.tree) ? A.T : nullptr,
        scr ? A.T32 : nullptr, A.CK, scr ? A.Dm : nullptr, scr ? A.Dm8 : nullptr,
        scr ? A.Dm512 : nullptr, A.nb, A.nb8, A.nb512, A.diff, scr ? A.Dt : nullptr, A.fold,
        A.ev_mfma, (A.variant & 16) != 0);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}

int launch_bell_kf(const BellArgs& A, hipStream_t st) {
    int n = std::max(A.C, 1) * A.N * A.Na * A.Nl;
    if (A.labor) bell_kf_kernel<true><<<cdiv(n, 256), 256, 0, st>>>(A);
    else bell_kf_kernel<false><<<cdiv(n, 256), 256, 0, st>>>(A);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}

// kf of each tile's last state: out[row][t] = kf[row][min(Na-1, t·TW + TW-1)] for the Nl·N rows
// (the host-side dispatch order needs only these: ws_tree_perm)
__global__ void kf_tile_last_kernel(const int* __restrict__ kf, int rows, int Na, int TW,
                                    int ntile, int* __restrict__ out) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= rows * ntile) return;
    const int row = g / ntile, t = g - row * ntile;
    out[g] = kf[(size_t)row * Na + min(Na - 1, t * TW + TW - 1)];
}
int launch_kf_tile_last(const int* kf, int rows, int Na, int TW, int ntile, int* out,
                        hipStream_t st) {
    kf_tile_last_kernel<<<cdiv((long long)rows * ntile, 256), 256, 0, st>>>(kf, rows, Na, TW,
                                                                             ntile, out);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}

#ifndef AIY_BELL_R
#define AIY_BELL_R 2
#endif
template <int NP, bool LAB>
struct Geo {
    static constexpr int R = LAB ? 1 : AIY_BELL_R;
    static constexpr int LB = LAB ? 5 : 1;
};

template <int NP, bool LAB>
static void run_init(const BellArgs& A, hipStream_t st) {
    bell_init_kernel<NP, LAB><<<cdiv((long long)std::max(A.C, 1) * A.N * A.Na, 128), 128, 0, st>>>(A);
}
template <int NP, bool LAB, int R, int MINW>
static void screen_geo(const BellArgs& A, hipStream_t st) {
    constexpr int LB = LAB ? 5 : 1;
    int ntile = cdiv(A.Na, 64 * R), nlb = cdiv(A.Nl, LB), nchunk = cdiv(A.Na, A.CK);
    long long items = (long long)A.N * ntile * nlb * nchunk;
    bell_screen_kernel<NP, LAB, R, LB, 8, MINW><<<cdiv(items, 4), 256, 0, st>>>(A, ntile, nlb, nchunk);
}
template <int NP, bool LAB>
static void run_screen(const BellArgs& A, hipStream_t st) {
    if constexpr (NP > 0) {
        if constexpr (LAB) {
            screen_geo<NP, LAB, 1, 1>(A, st);
        } else {
            // variant: bit 0 → 4 states per lane (else 2); bit 1 → cap registers for 8 waves/SIMD
            switch (A.variant & 3) {
                case 1: screen_geo<NP, LAB, 4, 1>(A, st); break;
                case 2: screen_geo<NP, LAB, 2, 8>(A, st); break;
                case 3: screen_geo<NP, LAB, 4, 8>(A, st); break;
                default: screen_geo<NP, LAB, 2, 1>(A, st); break;
            }
        }
    }
}
template <int NP, bool LAB, int R, int W, int PK = 1>
static void tree_geo(const BellArgs& A, hipStream_t st) {
    constexpr int LB = LAB ? 5 : 1;
    const int ntile = cdiv(A.Na, bell_tile_width(A, R));
    const int grid = cdiv(std::max(A.C, 1) * A.N * ntile, PK);
    if (A.trace || A.hitcount)
        launch_dispatch_timed(bell_tree_kernel<NP, LAB, R, LB, W, true, PK>, dim3(grid),
                              dim3(64 * W * PK), 0, st, A, ntile);
    else
        launch_dispatch_timed(bell_tree_kernel<NP, LAB, R, LB, W, false, PK>, dim3(grid),
                              dim3(64 * W * PK), 0, st, A, ntile);
}
// variant bit 0: 2 states per lane (A1 only); bits 1-2: waves per tile 1 (default), 2, 4, 8;
// one-wave tiles with a dispatch permutation: bell_tree_pack waves per workgroup
template <int NP, bool LAB, int R>
static void tree_w(const BellArgs& A, hipStream_t st) {
    switch ((A.variant >> 1) & 3) {
        case 1: tree_geo<NP, LAB, R, 2>(A, st); break;
        case 2: tree_geo<NP, LAB, R, 4>(A, st); break;
        case 3: tree_geo<NP, LAB, R, 8>(A, st); break;
        default:
            if constexpr (!LAB && R == 1) {
                if (A.perm && bell_tree_hybrid(A)) {
                    const int ntile = cdiv(A.Na, bell_tile_width(A, 1));
                    const int grid = A.perm_slots / 2;
                    if (A.trace || A.hitcount)
                        launch_dispatch_timed(bell_tree_hybrid_kernel<NP, true>, dim3(grid),
                                              dim3(128), 0, st, A, ntile);
                    else
                        launch_dispatch_timed(bell_tree_hybrid_kernel<NP, false>, dim3(grid),
                                              dim3(128), 0, st, A, ntile);
                    return;
                }
                switch (A.perm ? bell_tree_pack(A) : 1) {
                    case 2: tree_geo<NP, LAB, R, 1, 2>(A, st); return;
                    case 4: tree_geo<NP, LAB, R, 1, 4>(A, st); return;
                    case 8: tree_geo<NP, LAB, R, 1, 8>(A, st); return;
                    default: break;
                }
            }
            tree_geo<NP, LAB, R, 1>(A, st);
            break;
    }
}
template <int NP, bool LAB>
static void run_tree(const BellArgs& A, hipStream_t st) {
    if constexpr (NP > 0) {
        // the tuning geometries are instantiated for the reference sigma = 5 (NP = 4) only
        if constexpr (!LAB && NP == 4) {
            if (A.variant & 1) tree_w<NP, LAB, 2>(A, st);
            else tree_w<NP, LAB, 1>(A, st);
        } else if constexpr (LAB && NP == 4) {  // labour: cooperating waves per tile (bits 1-2)
            tree_w<NP, LAB, 1>(A, st);
        } else {
            tree_geo<NP, LAB, 1, 1>(A, st);
        }
    }
}
template <int NP, bool LAB>
static void run_plain(const BellArgs& A, hipStream_t st) {
    bell_plain_kernel<NP, LAB><<<dim3(cdiv(A.Na, 64), A.N), 256, 0, st>>>(A);
}
template <int NP, bool LAB>
static void run_merge(const BellArgs& A, int use_partial, hipStream_t st) {
    constexpr int LB = Geo<NP, LAB>::LB;
    bell_merge_kernel<NP, LAB, LB><<<cdiv(A.N * A.Na, 256), 256, 0, st>>>(
        A, use_partial, cdiv(A.Nl, LB), cdiv(A.Na, A.CK));
}

template <template <int, bool> class F, class... Args>
static int dispatch(int np, bool lab, Args&&... args) {
#define AIY_CASE(n)                                              \
    case n:                                                      \
        if (lab) F<n, true>::go(args...);                        \
        else F<n, false>::go(args...);                           \
        break;
    switch (np) {
        AIY_CASE(1) AIY_CASE(2) AIY_CASE(3) AIY_CASE(4) AIY_CASE(5) AIY_CASE(6) AIY_CASE(7)
        AIY_CASE(8)
        default:
            if (lab) F<0, true>::go(args...);
            else F<0, false>::go(args...);
    }
#undef AIY_CASE
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}
template <int NP, bool LAB>
struct InitF { static void go(const BellArgs& A, hipStream_t st) { run_init<NP, LAB>(A, st); } };
template <int NP, bool LAB>
struct ScreenF { static void go(const BellArgs& A, hipStream_t st) { run_screen<NP, LAB>(A, st); } };
template <int NP, bool LAB>
struct TreeF { static void go(const BellArgs& A, hipStream_t st) { run_tree<NP, LAB>(A, st); } };
template <int NP, bool LAB>
struct PlainF { static void go(const BellArgs& A, hipStream_t st) { run_plain<NP, LAB>(A, st); } };
template <int NP, bool LAB>
struct MergeF {
    static void go(const BellArgs& A, int u, hipStream_t st) { run_merge<NP, LAB>(A, u, st); }
};

int launch_bell_init(const BellArgs& A, hipStream_t st) { return dispatch<InitF>(A.np, A.labor, A, st); }
int launch_bell_screen(const BellArgs& A, hipStream_t st) {
    if (A.np < 1 || A.np > 8) return fail(AIY_BAD_ARG, "screened sweep needs integer sigma in [2, 9]");
    return dispatch<ScreenF>(A.np, A.labor, A, st);
}
int launch_bell_tree(const BellArgs& A, hipStream_t st) {
    if (A.np < 1 || A.np > 8) return fail(AIY_BAD_ARG, "screened sweep needs integer sigma in [2, 9]");
    return dispatch<TreeF>(A.np, A.labor, A, st);
}
int launch_bell_plain(const BellArgs& A, hipStream_t st) { return dispatch<PlainF>(A.np, A.labor, A, st); }
int launch_bell_merge(const BellArgs& A, int use_partial, hipStream_t st) {
    return dispatch<MergeF>(A.np, A.labor, A, use_partial, st);
}

size_t bell_partial_slots(const BellArgs& A) {
    int LB = A.labor ? 5 : 1;  // independent of the per-lane state count R (indexed by j)
    return (size_t)cdiv(A.Nl, LB) * cdiv(A.Na, A.CK) * A.N * A.Na;
}

}  // namespace aiy

namespace aiy {
// dis_l = psi * L_l^(1+eta) / (1+eta)   (Aiyagari_Endogenous_Labor_VFI.m:96)
__global__ void disutility_kernel(const double* __restrict__ L, int Nl, double psi, double eta,
                                  double* __restrict__ dis) {
    int l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= Nl) return;
    double Lp = aiy_pow(L[l], 1 + eta);
    dis[l] = psi * Lp / (1 + eta);
}
int launch_disutility(const double* L, int Nl, double psi, double eta, double* dis,
                      hipStream_t st) {
    disutility_kernel<<<(Nl + 63) / 64, 64, 0, st>>>(L, Nl, psi, eta, dis);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}
}  // namespace aiy

namespace aiy {
// fold the kDiffSlots {max bits, any} slots into one {max bits, any} pair (device → device)
__global__ void reduce_slots_kernel(const unsigned long long* __restrict__ slots,
                                   unsigned long long* __restrict__ out) {
    int l = threadIdx.x;
    unsigned long long k = slots[2 * l];
    int any = __ballot((slots[2 * l + 1] & 1ull) != 0ull) != 0ull;
    for (int off = 32; off > 0; off >>= 1) {
        unsigned long long o = __shfl_xor(k, off);
        k = o > k ? o : k;
    }
    if (l == 0) {
        out[0] = k;
        out[1] = any ? 1ull : 0ull;
    }
}
int launch_reduce_slots(const unsigned long long* slots, void* out, hipStream_t st) {
    static_assert(kDiffSlots == 64, "one wave folds the slots");
    reduce_slots_kernel<<<1, 64, 0, st>>>(slots, (unsigned long long*)out);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}
// host-side fold of slots copied back (pinned)
double fold_slots_host(const unsigned long long* h) {
    unsigned long long k = 0;
    bool any = false;
    for (int q = 0; q < kDiffSlots; ++q) {
        if (h[2 * q + 1] & 1ull) any = true;  // (bit 1: EGM non-monotone flag)
        k = h[2 * q] > k ? h[2 * q] : k;
    }
    if (!any) return __builtin_nan("");
    return aiy_bitsd(k);
}
}  // namespace aiy
