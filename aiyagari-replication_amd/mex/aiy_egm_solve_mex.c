/* [policy_c, policy_k, dist, iter] =
 *     aiy_egm_solve_mex(policy_c, a_grid, s, P, r, w, beta, sigma, amin, tol, max_iter)
 * Replaces the EGM while loop of Aiyagari_EGM.m:71-110 (GE copy :172-212).  policy_c: Na x N. */
#include "mexcommon.h"
void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    aiy_nargs(nrhs, 11, 11, nlhs, 4, "[policy_c,policy_k,dist,iter] = aiy_egm_solve_mex(policy_c,a_grid,s,P,r,w,beta,sigma,amin,tol,max_iter)");
    mwSize Na = mxGetM(prhs[0]), N = mxGetN(prhs[0]);
    aiy_in(prhs[0], "policy_c", 0, 0);
    const double* a = aiy_vec(prhs[1], "a_grid", Na, NULL);
    const double* s = aiy_vec(prhs[2], "s", N, NULL);
    const double* P = aiy_in(prhs[3], "P", N, N);
    double r = aiy_scalar(prhs[4], "r"), w = aiy_scalar(prhs[5], "w");
    double beta = aiy_scalar(prhs[6], "beta"), sigma = aiy_scalar(prhs[7], "sigma");
    double amin = aiy_scalar(prhs[8], "amin"), tol = aiy_scalar(prhs[9], "tol");
    int64_t max_iter = (int64_t)aiy_scalar(prhs[10], "max_iter");
    plhs[0] = aiy_copy(prhs[0]);
    mxArray* pk = aiy_out(Na, N);
    double dist = 0;
    int64_t it = 0;
    aiy_begin();
    aiy_check(aiy_egm_solve(mxGetPr(plhs[0]), a, s, P, (int64_t)N, (int64_t)Na, r, w, beta, sigma,
                            amin, tol, max_iter, mxGetPr(pk), &dist, &it));
    if (nlhs > 1) plhs[1] = pk; else mxDestroyArray(pk);
    if (nlhs > 2) plhs[2] = mxCreateDoubleScalar(dist);
    if (nlhs > 3) plhs[3] = mxCreateDoubleScalar((double)it);
}
