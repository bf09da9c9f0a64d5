/* [lambda, K, iter, dist] = aiy_dist_stationary_mex(policy, a_grid, P, lambda0, tol, max_iter,
 *                                                   on_grid)
 * New (no reference counterpart): stationary distribution by histogram iteration.
 * on_grid = 1: policy holds 1-based grid indices (the idx of max, VFI); 0: policy_k values
 * (EGM), mass split between bracketing grid nodes.  N x Na (VFI) or Na x N (EGM) layout. */
#include "mexcommon.h"
void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    aiy_nargs(nrhs, 7, 7, nlhs, 4, "[lambda,K,iter,dist] = aiy_dist_stationary_mex(policy,a_grid,P,lambda0,tol,max_iter,on_grid)");
    mwSize N = mxGetM(prhs[2]);
    const double* P = aiy_in(prhs[2], "P", N, N);
    const double* pol = aiy_in(prhs[0], "policy", 0, 0);
    int vfi = (mxGetM(prhs[0]) == N);
    mwSize Na = vfi ? mxGetN(prhs[0]) : mxGetM(prhs[0]);
    const double* a = aiy_vec(prhs[1], "a_grid", Na, NULL);
    aiy_in(prhs[3], "lambda0", mxGetM(prhs[0]), mxGetN(prhs[0]));
    double tol = aiy_scalar(prhs[4], "tol");
    int64_t max_iter = (int64_t)aiy_scalar(prhs[5], "max_iter");
    int on_grid = aiy_scalar(prhs[6], "on_grid") != 0;
    plhs[0] = aiy_copy(prhs[3]);
    int32_t* idx = NULL;
    if (on_grid) {
        idx = (int32_t*)malloc(sizeof(int32_t) * N * Na);
        for (mwSize q = 0; q < N * Na; ++q) idx[q] = (int32_t)pol[q];
    }
    double K = 0, dist = 0;
    int64_t it = 0;
    aiy_begin();
    int rc = aiy_dist_stationary(idx, on_grid ? NULL : pol, vfi, a, P, (int64_t)N, (int64_t)Na,
                                 tol, max_iter, mxGetPr(plhs[0]), &K, &it, &dist);
    free(idx);
    aiy_check(rc);
    if (nlhs > 1) plhs[1] = mxCreateDoubleScalar(K);
    if (nlhs > 2) plhs[2] = mxCreateDoubleScalar((double)it);
    if (nlhs > 3) plhs[3] = mxCreateDoubleScalar(dist);
}
