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
#include <type_traits>

#include "aiy_common.hpp"
#include "bellman.hpp"

namespace aiy {

constexpr double kTau = 9.094947017729282e-13;  // 2^-40
constexpr double kThr = 0.99999999999999644729;  // 1 - 2^-48
constexpr float kThr32 = 0.999998092651367f;      // 1 - 2^-19 (exact in fp32)
constexpr float kBig32 = 1.152921504606847e18f;   // 2^60: fp32-path range guard

typedef float f32x2 __attribute__((ext_vector_type(2)));

// fp64 → fp32 rounded outward by one step past round-to-nearest: a rigorous upper (lower)
// bound of the real value even with the fp64 rounding of x's own computation
__device__ __forceinline__ float f32_up(double x) { return nextafterf((float)x, __builtin_inff()); }
__device__ __forceinline__ float f32_dn(double x) { return nextafterf((float)x, -__builtin_inff()); }

template <int NP>
__device__ __forceinline__ f32x2 ipow2(f32x2 c) {
    static_assert(NP >= 1 && NP <= 8, "screen exponent");
    if constexpr (NP == 1) return c;
    f32x2 c2 = c * c;
    if constexpr (NP == 2) return c2;
    if constexpr (NP == 3) return c2 * c;
    f32x2 c4 = c2 * c2;
    if constexpr (NP == 4) return c4;
    if constexpr (NP == 5) return c4 * c;
    if constexpr (NP == 6) return c4 * c2;
    if constexpr (NP == 7) return (c4 * c2) * c;
    return c4 * c4;
}

// exact value of candidate (c, l, k) in the literal MATLAB order
template <int NP, bool LAB>
__device__ __forceinline__ double bell_val(double c, double ev, double sigma, double dis) {
    double u;
    if constexpr (NP > 0) {
        double p = 1.0 / aiy_ipow(c, NP);  // c.^(1-sigma), sigma = NP + 1
        u = (p - 1) / (1 - sigma);
    } else {
        if (!LAB && sigma == 1.0) u = aiy_log(c);  // Aiyagari_VFI.m:74-75 (labour script: no branch)
        else u = (aiy_pow(c, 1.0 - sigma) - 1) / (1 - sigma);
    }
    if constexpr (LAB) return (u - dis) + ev;  // Labor_VFI.m:95-99
    else return u + ev;                        // Aiyagari_VFI.m:79
}

// (max value, first index) merge; NaN never enters (MATLAB max omits NaN)
__device__ __forceinline__ bool lexi_take(double val, int q, double& best, int& idx) {
    if (val != val) return false;
    if (idx < 0 || val > best || (val == best && q < idx)) {
        best = val;
        idx = q;
        return true;
    }
    return false;
}

// screening bar of (best, dis_l):  n·(best + dis) − τ·n·(|best| + |dis|)
__device__ __forceinline__ double screen_B(double best, int idx, double dis, int np) {
    if (idx < 0) return -__builtin_inf();
    double nd = (double)np;
    return nd * (best + dis) - kTau * nd * (fabs(best) + fabs(dis));
}

template <bool LAB>
__device__ __forceinline__ double cash(double x, double y, double Ll) {
    if constexpr (LAB) return x + y * Ll;  // (1+r)a_j + (w s_i) L_l   (Labor_VFI.m:81)
    else return x + y;                     // (1+r)a_j + w s_i          (Aiyagari_VFI.m:72)
}

// ------------------------------------------------------------------------------ 1. table
__device__ __forceinline__ double table_ev(int N, int Na, const double* __restrict__ P,
                                           const double* __restrict__ V, double beta, int i,
                                           int k) {
    double acc = 0.0;
    for (int m = 0; m < N; ++m) acc = acc + (beta * P[i * N + m]) * V[m * Na + k];
    return acc;
}
__device__ __forceinline__ double table_D(double ev, int np) {
    double ne = (double)np * ev;
    return (ne + 1.0) + kTau * (fabs(ne) + 1.0);
}

__global__ void bell_table_kernel(int N, int Na, const double* __restrict__ P,
                                  const double* __restrict__ V, double beta, int np,
                                  const double* __restrict__ a, double* __restrict__ EV,
                                  double2* __restrict__ T, float* __restrict__ T32, int CK) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= N * Na) return;
    int i = t / Na, k = t - i * Na;
    double acc = table_ev(N, Na, P, V, beta, i, k);
    EV[t] = acc;
    if (T) {
        double D = table_D(acc, np);
        T[t] = make_double2(a[k], D);
        if (T32) {  // relative to the chunk origin (a, D at k0): small magnitudes, fine ulps
            int k0 = k - k % CK;
            double D0 = table_D(table_ev(N, Na, P, V, beta, i, k0), np);
            float* pr = T32 + 2 * (size_t)i * (Na + (Na & 1)) + 2 * (k & ~1) + (k & 1);
            pr[0] = f32_dn(a[k] - a[k0]);  // pair layout {a_k, a_k+1, D_k, D_k+1}
            pr[2] = f32_up(D - D0);
        }
    }
}

// ------------------------------------------------------------------------------ 1b. kf
// feasible prefix per (l, i, j): depends on (r, w, a, s, L) only, so a solve computes it once
template <bool LAB>
__global__ void bell_kf_kernel(BellArgs A) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    int n = A.N * A.Na;
    if (t >= n * A.Nl) return;
    int l = t / n, ij = t - l * n;
    int i = ij / A.Na, j = ij - i * A.Na;
    double coh = cash<LAB>((1 + A.r) * A.a[j], A.w * A.s[i], LAB ? A.L[l] : 1.0);
    A.kf[t] = lower_bound_dev(A.a, A.Na, coh);
}

// ------------------------------------------------------------------------------ 2. init
template <int NP, bool LAB>
__global__ void bell_init_kernel(BellArgs A) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
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
        if (S > 0) {  // coarse scan of the feasible prefix (robust when the policy moved far)
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
    unsigned nhits = 0;

    auto exact_block = [&](int k0, int kend) {
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
    auto run = [&](auto guard, int kb, int ke) {
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
    const int r1_end = min(k_hi, max(k_lo, kmin));

    // ---- packed fp32 pre-screen (all quantities relative to the chunk origin k_lo)
    bool use32 = A.T32 != nullptr;
    float cp[R][LB], bp[R][LB];
    const float* __restrict__ T32row = use32 ? A.T32 + 2 * (size_t)i * (Na + (Na & 1)) : nullptr;
    double A0 = 0.0, S0 = 0.0;
    auto set_bp = [&]() {
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int q = 0; q < LB; ++q)
                bp[r][q] = (B[r][q] == B[r][q]) ? f32_dn(B[r][q] - S0) : __builtin_nanf("");
    };
    if (use32) {
        A0 = a[k_lo];
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
        for (int k = k_lo + lane; k < k_hi; k += 64)
            ok = ok && fabsf(T32row[2 * (k & ~1) + 2 + (k & 1)]) <= kBig32;
        use32 = __all(ok);
    }
    auto run32 = [&](auto guard, int kb, int ke) {
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
    if (use32) {
        // the pair layout needs even block starts: move the region split down to even
        // (the guarded loop is valid for feasible candidates too)
        const int r1_even = max(k_lo, r1_end & ~1);
        run32(std::false_type{}, k_lo, r1_even);
        run32(std::true_type{}, r1_even, k_hi);
    } else {
        run(std::false_type{}, k_lo, r1_end);
        run(std::true_type{}, r1_end, k_hi);
    }

    const size_t slab = ((size_t)lbk * nchunk + chunk) * N + i;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        int j = jbase + r * 64 + lane;
        if (j < Na) A.partial[slab * Na + j] = imp[r];
    }
    if (A.hitcount && nhits) atomicAdd(A.hitcount, (unsigned long long)nhits);
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
        if (use_partial && idx != -2) {
            const double* __restrict__ ev = A.EV + (size_t)i * Na;
            for (int lbk = 0; lbk < nlb; ++lbk) {
                int kfm = 0;
                for (int l = lbk * LB; l < min(lbk * LB + LB, Nl); ++l)
                    kfm = max(kfm, A.kf[(size_t)l * N * Na + t]);
                int nch = (kfm + A.CK - 1) / A.CK;
                for (int c = 0; c < nch; ++c) {
                    int q = A.partial[(((size_t)lbk * nchunk + c) * N + i) * Na + j];
                    if (q >= 0) {
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
__global__ void bell_plain_kernel(BellArgs A) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= A.N * A.Na) return;
    if (A.idx0[t] == -2) return;
    const int Na = A.Na, Nl = A.Nl;
    int i = t / Na, j = t - i * Na;
    const double* __restrict__ a = A.a;
    const double* __restrict__ ev = A.EV + (size_t)i * Na;
    double x = (1 + A.r) * a[j], y = A.w * A.s[i];
    double best = __builtin_nan("");
    int idx = -1;
    for (int l = 0; l < Nl; ++l) {
        double coh = cash<LAB>(x, y, LAB ? A.L[l] : 1.0);
        double dis = LAB ? A.dis[l] : 0.0;
        int kf = A.kf[(size_t)l * A.N * Na + t];
        for (int k = 0; k < kf; ++k)
            lexi_take(bell_val<NP, LAB>(coh - a[k], ev[k], A.sigma, dis), l + Nl * k, best, idx);
    }
    A.best0[t] = best;
    A.idx0[t] = idx;
}

// ------------------------------------------------------------------------------ launchers
static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

int launch_bell_table(const BellArgs& A, hipStream_t st) {
    int n = A.N * A.Na;
    bell_table_kernel<<<cdiv(n, 256), 256, 0, st>>>(A.N, A.Na, A.P, A.v_old, A.beta, A.np, A.a,
                                                    A.EV, A.np > 0 ? A.T : nullptr,
                                                    A.np > 0 ? A.T32 : nullptr, A.CK);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}

int launch_bell_kf(const BellArgs& A, hipStream_t st) {
    int n = A.N * A.Na * A.Nl;
    if (A.labor) bell_kf_kernel<true><<<cdiv(n, 256), 256, 0, st>>>(A);
    else bell_kf_kernel<false><<<cdiv(n, 256), 256, 0, st>>>(A);
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
    bell_init_kernel<NP, LAB><<<cdiv(A.N * A.Na, 128), 128, 0, st>>>(A);
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
template <int NP, bool LAB>
static void run_plain(const BellArgs& A, hipStream_t st) {
    bell_plain_kernel<NP, LAB><<<cdiv(A.N * A.Na, 128), 128, 0, st>>>(A);
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
    int any = __ballot(slots[2 * l + 1] != 0ull) != 0ull;
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
        if (h[2 * q + 1]) any = true;
        k = h[2 * q] > k ? h[2 * q] : k;
    }
    if (!any) return __builtin_nan("");
    return aiy_bitsd(k);
}
}  // namespace aiy
