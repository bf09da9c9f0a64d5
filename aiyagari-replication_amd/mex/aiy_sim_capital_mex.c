/* [agg_k_supply, sim_k, sim_z] = aiy_sim_capital_mex(policy_k, a_grid, P, z1, k1, uniforms [, layout])
 * Replaces the simulation loop of Aiyagari_VFI.m:104-129 (GE :174-193) and its copies.
 * policy_k is N x Na (VFI scripts, layout = 1) or Na x N (EGM scripts, layout = 0); without
 * `layout` it is detected from size(P,1), which is ambiguous (an error) when Na == N.
 * uniforms = the T-1 `rand` draws the loop would consume (generate them with rand(T-1,1)). */
#include "mexcommon.h"
void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    aiy_nargs(nrhs, 6, 7, nlhs, 3, "[agg_k_supply,sim_k,sim_z] = aiy_sim_capital_mex(policy_k,a_grid,P,z1,k1,uniforms[,layout])");
    mwSize N = mxGetM(prhs[2]), Na = 0, Tm1 = 0;
    const double* P = aiy_in(prhs[2], "P", N, N);
    const double* pol = aiy_in(prhs[0], "policy_k", 0, 0);
    int vfi;
    if (nrhs > 6) {
        vfi = aiy_scalar(prhs[6], "layout") != 0.0;
    } else {
        if (mxGetM(prhs[0]) == N && mxGetN(prhs[0]) == N)
            aiy_err("aiy:shape", "policy_k is %lu x %lu with N = %lu: pass layout (1 = N x Na, "
                    "0 = Na x N)", (unsigned long)N, (unsigned long)N, (unsigned long)N);
        vfi = (mxGetM(prhs[0]) == N);
    }
    if (vfi && mxGetM(prhs[0]) != N) aiy_err("aiy:shape", "layout 1: policy_k must be N x Na");
    if (!vfi && mxGetN(prhs[0]) != N)
        aiy_err("aiy:shape", "policy_k must be N x Na or Na x N with N = size(P,1)");
    Na = vfi ? mxGetN(prhs[0]) : mxGetM(prhs[0]);
    const double* a = aiy_vec(prhs[1], "a_grid", Na, NULL);
    double z1 = aiy_scalar(prhs[3], "z1"), k1 = aiy_scalar(prhs[4], "k1");
    const double* U = aiy_vec(prhs[5], "uniforms", 0, &Tm1);
    int64_t T = (int64_t)Tm1 + 1;
    double K = 0;
    mxArray* sk = nlhs > 1 ? aiy_out(T, 1) : NULL;
    int32_t* sz = nlhs > 2 ? (int32_t*)malloc(sizeof(int32_t) * T) : NULL;
    aiy_begin();
    int rc = aiy_sim_capital(pol, vfi, a, P, (int64_t)N, (int64_t)Na, (int64_t)z1, k1, T, U, &K,
                             sk ? mxGetPr(sk) : NULL, sz);
    if (rc == AIY_OK && sz) {
        plhs[2] = aiy_out(T, 1);
        for (int64_t t = 0; t < T; ++t) mxGetPr(plhs[2])[t] = sz[t];
    }
    free(sz);
    if (rc != AIY_OK && sk) mxDestroyArray(sk);
    aiy_check(rc);
    plhs[0] = mxCreateDoubleScalar(K);
    if (sk) plhs[1] = sk;
}
