/* [v_new, policy_k, policy_c, idx] = aiy_vfi_sweep_mex(v_old, a_grid, s, P, r, w, beta, sigma)
 * Replaces the body of the sweep in Aiyagari_VFI.m:68-83 (idx: 1-based, as max returns). */
#include "mexcommon.h"
void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    aiy_nargs(nrhs, 8, 8, nlhs, 4, "[v_new,policy_k,policy_c,idx] = aiy_vfi_sweep_mex(v_old,a_grid,s,P,r,w,beta,sigma)");
    mwSize N = mxGetM(prhs[0]), Na = mxGetN(prhs[0]);
    const double* v = aiy_in(prhs[0], "v_old", 0, 0);
    const double* a = aiy_vec(prhs[1], "a_grid", Na, NULL);
    const double* s = aiy_vec(prhs[2], "s", N, NULL);
    const double* P = aiy_in(prhs[3], "P", N, N);
    double r = aiy_scalar(prhs[4], "r"), w = aiy_scalar(prhs[5], "w");
    double beta = aiy_scalar(prhs[6], "beta"), sigma = aiy_scalar(prhs[7], "sigma");
    plhs[0] = aiy_out(N, Na);
    mxArray* pk = aiy_out(N, Na);
    mxArray* pc = aiy_out(N, Na);
    int32_t* idx = (int32_t*)malloc(sizeof(int32_t) * N * Na);
    aiy_begin();
    int rc = aiy_vfi_sweep(v, a, s, P, (int64_t)N, (int64_t)Na, r, w, beta, sigma, mxGetPr(plhs[0]),
                           mxGetPr(pk), mxGetPr(pc), idx);
    if (rc == AIY_OK && nlhs > 3) {
        plhs[3] = aiy_out(N, Na);
        double* o = mxGetPr(plhs[3]);
        for (mwSize q = 0; q < N * Na; ++q) o[q] = idx[q];
    }
    free(idx);
    aiy_check(rc);
    if (nlhs > 1) plhs[1] = pk; else mxDestroyArray(pk);
    if (nlhs > 2) plhs[2] = pc; else mxDestroyArray(pc);
}
