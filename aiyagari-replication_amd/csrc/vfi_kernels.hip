// A1/A2 — Aiyagari VFI Bellman sweep on gfx950 (reference: Aiyagari_VFI.m:65-90; the GE copy
// :147-171).  Four launches per sweep, all on the caller's stream:
//
//   1. table   EV(i,k) = Σ_m (β·P(i,m))·V(m,k) in the reference's order (:79), plus the
//              screening key D(i,k) = n·EV + 1 + slack, stored interleaved with a_k.
//   2. init    per state (i,j): cash on hand coh = (1+r)a_j + w s_i (:72), the feasible
//              prefix kf = #{k : a_k < coh} (c <= 0 is NaN and ignored by max, :73), and an
//              exact starting candidate (the hint = last sweep's argmax, or a coarse scan).
//   3. screen  the exhaustive max over a' (:79).  Work item = one wavefront × (64·R states)
//              × (CK candidates a'), so every wave carries the same work whatever j is
//              (feasible prefixes grow with j).  Each candidate costs 6 fp64 VALU ops: a
//              division-free test  (D_k − n·best)·c^n ≥ 1 − 2^-48  that is TRUE for every
//              candidate whose exact value reaches the running best (rigorous slack, see
//              DESIGN.md §A1).  Candidates that pass are evaluated exactly in the literal
//              MATLAB order and merged with the (max value, first index) rule, so the result
//              equals a plain exhaustive scan bit for bit.
//   4. merge   per state: combine the init candidate with each chunk's improvement, write
//              v_new, policy index, policy_k = a(idx) (:80), policy_c = coh − policy_k
//              (:81), and max|v_new − v_old| ignoring NaN (:85) via an order-independent
//              atomicMax on the IEEE bits (deterministic).
//
// Integer σ ≥ 2 (the reference's σ = 5) uses the screened path with n = σ−1 as a template
// constant; any other σ uses the plain exhaustive kernel (exact evaluation of every feasible
// candidate, pow/log from the device math library).
#include "aiy_common.hpp"
#include "vfi_kernels.hpp"

#include <type_traits>

namespace aiy {

constexpr double kTau = 9.094947017729282e-13;  // 2^-40: slack relative to |n·EV|, |n·best|
constexpr double kThr = 0.99999999999999644729;  // 1 - 2^-48

// exact candidate value in the literal order of Aiyagari_VFI.m:72-79.
template <int NP>
__device__ __forceinline__ double vfi_val(double c, double ev, double sigma) {
    double u;
    if constexpr (NP > 0) {
        double p = 1.0 / aiy_ipow(c, NP);  // c.^(1-sigma), sigma = NP+1
        u = (p - 1) / (1 - sigma);
    } else {
        u = (sigma == 1.0) ? log(c) : (pow(c, 1.0 - sigma) - 1) / (1 - sigma);
    }
    return u + ev;
}

// (max value, first index) merge; NaN values never enter (MATLAB max omits NaN).
__device__ __forceinline__ void lexi_take(double val, int k, double& best, int& idx) {
    if (val != val) return;
    if (idx < 0 || val > best || (val == best && k < idx)) {
        best = val;
        idx = k;
    }
}

// screening key of the running best: B = n·best − τ·n·|best|
__device__ __forceinline__ double screen_B(double best, int idx, int np) {
    if (idx < 0) return -__builtin_inf();
    double nb = (double)np * best;
    return nb - kTau * fabs(nb);
}

// ------------------------------------------------------------------------------ 1. table
__global__ void vfi_table_kernel(int N, int Na, const double* __restrict__ P,
                                 const double* __restrict__ V, double beta, int np,
                                 const double* __restrict__ a, double* __restrict__ EV,
                                 double2* __restrict__ T) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= N * Na) return;
    int i = t / Na, k = t - i * Na;
    double acc = 0.0;
    for (int m = 0; m < N; ++m) acc = acc + (beta * P[i * N + m]) * V[m * Na + k];
    EV[t] = acc;
    if (T) {
        double nd = (double)np;
        double ne = nd * acc;
        double D = (ne + 1.0) + kTau * (fabs(ne) + 1.0);
        T[t] = make_double2(a[k], D);
    }
}

// ------------------------------------------------------------------------------ 2. init
template <int NP>
__global__ void vfi_init_kernel(int N, int Na, const double* __restrict__ a,
                                const double* __restrict__ s, double r, double w, double sigma,
                                const double* __restrict__ EV, const int* __restrict__ hint,
                                int coarse, double* __restrict__ coh_o, int* __restrict__ kf_o,
                                double* __restrict__ best_o, int* __restrict__ idx_o) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= N * Na) return;
    int i = t / Na, j = t - i * Na;
    double coh = (1 + r) * a[j] + w * s[i];  // :72
    int kf = lower_bound_dev(a, Na, coh);    // a_k < coh  <=>  c > 0
    const double* ev = EV + (size_t)i * Na;
    double best = __builtin_nan("");
    int idx = -1;
    if (kf > 0) {
        if (hint) {
            int h = hint[t];
            h = h < 0 ? 0 : (h >= kf ? kf - 1 : h);
            lexi_take(vfi_val<NP>(coh - a[h], ev[h], sigma), h, best, idx);
        }
        if (coarse > 0) {
            for (int k = 0; k < kf; k += coarse)
                lexi_take(vfi_val<NP>(coh - a[k], ev[k], sigma), k, best, idx);
            lexi_take(vfi_val<NP>(coh - a[kf - 1], ev[kf - 1], sigma), kf - 1, best, idx);
        } else if (!hint) {
            lexi_take(vfi_val<NP>(coh - a[0], ev[0], sigma), 0, best, idx);
        }
    }
    coh_o[t] = coh;
    kf_o[t] = kf;
    best_o[t] = best;
    idx_o[t] = idx;
}

// ------------------------------------------------------------------------------ 3. screen
template <int NP, int R, int KB>
__global__ __launch_bounds__(256) void vfi_screen_kernel(
    int N, int Na, int ntile, int nchunk, int CK, const double2* __restrict__ T,
    const double* __restrict__ EV, const double* __restrict__ a,
    const double* __restrict__ coh_g, const int* __restrict__ kf_g,
    const double* __restrict__ best0, const int* __restrict__ idx0, double sigma,
    int* __restrict__ partial, unsigned long long* __restrict__ hitcount) {
    const int wave = readfirst(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int item = readfirst(blockIdx.x * 4 + wave);
    const int chunk = item % nchunk;
    const int rest = item / nchunk;
    const int tile = rest % ntile;
    const int i = rest / ntile;
    if (i >= N) return;
    const int jbase = tile * (64 * R);
    const int jlast = min(jbase + 64 * R, Na) - 1;
    const int kmax = readfirst(kf_g[(size_t)i * Na + jlast]);
    const int k_lo = chunk * CK;
    if (k_lo >= kmax) return;
    const int kmin = readfirst(kf_g[(size_t)i * Na + jbase]);
    const int k_hi = min(k_lo + CK, kmax);

    double coh[R], B[R], best[R];
    int idx[R], imp[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        int j = jbase + r * 64 + lane;
        imp[r] = -1;
        if (j < Na) {
            size_t ij = (size_t)i * Na + j;
            coh[r] = coh_g[ij];
            best[r] = best0[ij];
            idx[r] = idx0[ij];
            B[r] = screen_B(best[r], idx[r], NP);
        } else {
            coh[r] = -__builtin_inf();
            best[r] = 0.0;
            idx[r] = 0x7fffffff;
            B[r] = __builtin_inf();
        }
    }
    const double2* __restrict__ Trow = T + (size_t)i * Na;
    const double* __restrict__ ev = EV + (size_t)i * Na;
    unsigned nhits = 0;

    auto exact_block = [&](int k0, int kend) {
        for (int k = k0; k < kend; ++k) {
            double ak = a[k];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                double c = coh[r] - ak;
                if (c > 0) {
                    double q = aiy_ipow(c, NP);
                    double t = (Trow[k].y - B[r]) * q;
                    if (t >= kThr) {
                        double val = vfi_val<NP>(c, ev[k], sigma);
                        int before = idx[r];
                        lexi_take(val, k, best[r], idx[r]);
                        if (idx[r] != before) {
                            imp[r] = k;
                            B[r] = screen_B(best[r], idx[r], NP);
                        }
                        ++nhits;
                    }
                }
            }
        }
    };

    // region 1: every lane feasible (k < kmin <= kf_j); region 2: guard c by max(c, 0) so
    // infeasible candidates (c <= 0, NaN in the reference) can never pass the screen.
    auto run = [&](auto guard, int kb, int ke) {
        int k = kb;
        for (; k + KB <= ke; k += KB) {
            bool hit = false;
#pragma unroll
            for (int kk = 0; kk < KB; ++kk) {
                const double2 tk = Trow[k + kk];  // wave-uniform address → scalar loads
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    double c = coh[r] - tk.x;
                    if constexpr (decltype(guard)::value) c = fmax(c, 0.0);
                    double q = aiy_ipow(c, NP);
                    double t = (tk.y - B[r]) * q;
                    hit |= (t >= kThr);
                }
            }
            if (__any(hit)) exact_block(k, k + KB);
        }
        if (k < ke) {  // remainder (< KB candidates), always guarded
            bool hit = false;
            for (int kk = k; kk < ke; ++kk) {
                const double2 tk = Trow[kk];
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    double c = fmax(coh[r] - tk.x, 0.0);
                    double q = aiy_ipow(c, NP);
                    hit |= ((tk.y - B[r]) * q >= kThr);
                }
            }
            if (__any(hit)) exact_block(k, ke);
        }
    };
    const int r1_end = min(k_hi, max(k_lo, kmin));
    run(std::false_type{}, k_lo, r1_end);
    run(std::true_type{}, r1_end, k_hi);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        int j = jbase + r * 64 + lane;
        if (j < Na) partial[((size_t)chunk * N + i) * Na + j] = imp[r];
    }
    if (hitcount && nhits) atomicAdd(hitcount, (unsigned long long)nhits);
}

// ------------------------------------------------------------------------------ 4. merge
template <int NP>
__global__ void vfi_merge_kernel(int N, int Na, int CK, int use_partial,
                                 const double* __restrict__ a, const double* __restrict__ coh_g,
                                 const int* __restrict__ kf_g, const double* __restrict__ best0,
                                 const int* __restrict__ idx0, const double* __restrict__ EV,
                                 const int* __restrict__ partial, const double* __restrict__ v_old,
                                 double sigma, double* __restrict__ v_new, int* __restrict__ idx_o,
                                 double* __restrict__ pk, double* __restrict__ pc,
                                 unsigned long long* __restrict__ diff) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    bool ok = false;
    double d = 0.0;
    if (t < N * Na) {
        int i = t / Na;
        double coh = coh_g[t];
        double best = best0[t];
        int idx = idx0[t];
        if (use_partial) {
            int nch = (kf_g[t] + CK - 1) / CK;
            const double* ev = EV + (size_t)i * Na;
            for (int c = 0; c < nch; ++c) {
                int q = partial[((size_t)c * N + i) * Na + (t - i * Na)];
                if (q >= 0) lexi_take(vfi_val<NP>(coh - a[q], ev[q], sigma), q, best, idx);
            }
        }
        if (idx < 0) {  // no feasible a': max of all-NaN is NaN at index 1
            idx = 0;
            best = __builtin_nan("");
        }
        v_new[t] = best;
        idx_o[t] = idx;
        double kp = a[idx];
        if (pk) pk[t] = kp;
        if (pc) pc[t] = coh - kp;
        d = fabs(best - v_old[t]);
        ok = (d == d);
    }
    if (diff) {
        unsigned long long key = ok ? nonneg_key(d) : 0ull;
        unsigned long long anyok = __ballot(ok);
        for (int off = 32; off > 0; off >>= 1) {
            unsigned long long o = __shfl_xor(key, off);
            key = o > key ? o : key;
        }
        if ((threadIdx.x & 63) == 0 && anyok) {
            atomicMax(diff, key);
            atomicOr(diff + 1, 1ull);
        }
    }
}

// ------------------------------------------------------------------------------ plain
// exhaustive (any σ): one thread per state, every feasible candidate evaluated exactly.
template <int NP>
__global__ void vfi_plain_kernel(int N, int Na, const double* __restrict__ a,
                                 const double* __restrict__ coh_g, const int* __restrict__ kf_g,
                                 const double* __restrict__ EV, double sigma,
                                 double* __restrict__ best_o, int* __restrict__ idx_o) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= N * Na) return;
    int i = t / Na;
    const double* ev = EV + (size_t)i * Na;
    double coh = coh_g[t];
    int kf = kf_g[t];
    double best = __builtin_nan("");
    int idx = -1;
    for (int k = 0; k < kf; ++k) lexi_take(vfi_val<NP>(coh - a[k], ev[k], sigma), k, best, idx);
    best_o[t] = best;
    idx_o[t] = idx;
}

// ------------------------------------------------------------------------------ launchers
static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

int launch_vfi_table(const VfiArgs& A, hipStream_t st) {
    int n = A.N * A.Na;
    vfi_table_kernel<<<cdiv(n, 256), 256, 0, st>>>(A.N, A.Na, A.P, A.v_old, A.beta, A.np, A.a,
                                                   A.EV, A.np > 0 ? A.T : nullptr);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}

template <int NP>
static void init_t(const VfiArgs& A, hipStream_t st) {
    int n = A.N * A.Na;
    vfi_init_kernel<NP><<<cdiv(n, 256), 256, 0, st>>>(A.N, A.Na, A.a, A.s, A.r, A.w, A.sigma,
                                                      A.EV, A.hint, A.coarse, A.coh, A.kf,
                                                      A.best0, A.idx0);
}
template <int NP>
static void screen_t(const VfiArgs& A, hipStream_t st) {
    constexpr int R = 2, KB = 8;
    int ntile = cdiv(A.Na, 64 * R);
    int nchunk = cdiv(A.Na, A.CK);
    long long items = (long long)A.N * ntile * nchunk;
    vfi_screen_kernel<NP, R, KB><<<cdiv(items, 4), 256, 0, st>>>(
        A.N, A.Na, ntile, nchunk, A.CK, A.T, A.EV, A.a, A.coh, A.kf, A.best0, A.idx0, A.sigma,
        A.partial, A.hitcount);
}
template <int NP>
static void merge_t(const VfiArgs& A, int use_partial, hipStream_t st) {
    int n = A.N * A.Na;
    vfi_merge_kernel<NP><<<cdiv(n, 256), 256, 0, st>>>(
        A.N, A.Na, A.CK, use_partial, A.a, A.coh, A.kf, A.best0, A.idx0, A.EV, A.partial,
        A.v_old, A.sigma, A.v_new, A.idx, A.pk, A.pc, A.diff);
}
template <int NP>
static void plain_t(const VfiArgs& A, hipStream_t st) {
    int n = A.N * A.Na;
    vfi_plain_kernel<NP><<<cdiv(n, 256), 256, 0, st>>>(A.N, A.Na, A.a, A.coh, A.kf, A.EV,
                                                       A.sigma, A.best0, A.idx0);
}

#define AIY_NP_DISPATCH(np, fn, ...)          \
    switch (np) {                             \
        case 1: fn<1>(__VA_ARGS__); break;    \
        case 2: fn<2>(__VA_ARGS__); break;    \
        case 3: fn<3>(__VA_ARGS__); break;    \
        case 4: fn<4>(__VA_ARGS__); break;    \
        case 5: fn<5>(__VA_ARGS__); break;    \
        case 6: fn<6>(__VA_ARGS__); break;    \
        case 7: fn<7>(__VA_ARGS__); break;    \
        case 8: fn<8>(__VA_ARGS__); break;    \
        default: fn<0>(__VA_ARGS__); break;   \
    }

int launch_vfi_init(const VfiArgs& A, hipStream_t st) {
    AIY_NP_DISPATCH(A.np, init_t, A, st);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}
int launch_vfi_screen(const VfiArgs& A, hipStream_t st) {
    if (A.np < 1 || A.np > 8) return fail(AIY_BAD_ARG, "screened sweep needs integer sigma in [2,9]");
    switch (A.np) {
        case 1: screen_t<1>(A, st); break;
        case 2: screen_t<2>(A, st); break;
        case 3: screen_t<3>(A, st); break;
        case 4: screen_t<4>(A, st); break;
        case 5: screen_t<5>(A, st); break;
        case 6: screen_t<6>(A, st); break;
        case 7: screen_t<7>(A, st); break;
        default: screen_t<8>(A, st); break;
    }
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}
int launch_vfi_plain(const VfiArgs& A, hipStream_t st) {
    AIY_NP_DISPATCH(A.np, plain_t, A, st);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}
int launch_vfi_merge(const VfiArgs& A, int use_partial, hipStream_t st) {
    AIY_NP_DISPATCH(A.np, merge_t, A, use_partial, st);
    AIY_HIP(hipGetLastError());
    return AIY_OK;
}

}  // namespace aiy
