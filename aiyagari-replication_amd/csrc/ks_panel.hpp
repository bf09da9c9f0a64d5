// Launch interface of the Krusell-Smith shock-panel and panel-simulation kernels
// (ks_panel_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace aiy {

constexpr int kPanelBlock = 256;      // lanes per block of the panel kernels
constexpr int kPanelMaxBlocks = 1024;  // cap on blocks (more agents -> more per lane)

// G of the mean(k_population) reduction order (np_oracle.ks_panel_blocks)
inline int panel_blocks(int64_t pop) {
    int64_t g = (pop + kPanelBlock - 1) / kPanelBlock;
    return (int)(g < 1 ? 1 : (g > kPanelMaxBlocks ? kPanelMaxBlocks : g));
}

struct ShockArgs {
    int T, pop;
    double pgg, pbb, ug;
    double thr[8];        // [cur_z][prev_z][prev_e]: Peps(prev_e, 1) of :78-92
    const double* U;      // the rand stream: T-1 aggregate, pop initial, (T-1)*pop (t, i)
    int8_t* zi;           // [T] 0 good / 1 bad
    int8_t* eps;          // element (t, i) at eps[t*ts + i*is]: 0 employed / 1 unemployed
    int64_t ts, is;
};
int launch_ks_shocks(const ShockArgs& A, hipStream_t st);

struct PanelArgs {
    int nk, nK, T, pop, G;
    const double* k_grid;
    const double* K_grid;
    const double* k_opt;   // k x K x S column-major: (ki, Ki, s) at (s*nK + Ki)*nk + ki
    const int8_t* zi;      // [T]
    const int8_t* eps;     // (t, i) at eps[t*ts + i*is]
    int64_t ts, is;
    double* k_pop;         // [pop] in/out
    double* K_ts;          // [T] out
    double* part;          // [2*G] block partial sums (ping-pong per period)
};
int launch_ks_panel(const PanelArgs& A, hipStream_t st);

}  // namespace aiy
