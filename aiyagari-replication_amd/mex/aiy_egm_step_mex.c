/* [policy_c_next, policy_k, dist] = aiy_egm_step_mex(policy_c, a_grid, s, P, r, w, beta, sigma, amin)
 * One pass of the EGM loop body, Aiyagari_EGM.m:77-107 (GE copy :179-210): the Euler RHS, the
 * endogenous grid, interp1 with linear extrapolation, the borrowing clamp, and
 * dist = max|policy_c_next - policy_c| (:106).  The script keeps its own while loop
 * (:74 `while dist > tol && iter < max_iter`) and `policy_c = policy_c_next` (:107).
 * policy_c, policy_c_next, policy_k: Na x N (the script's layout). */
#include "mexcommon.h"
void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    aiy_nargs(nrhs, 9, 9, nlhs, 3, "[policy_c_next,policy_k,dist] = aiy_egm_step_mex(policy_c,a_grid,s,P,r,w,beta,sigma,amin)");
    mwSize Na = mxGetM(prhs[0]), N = mxGetN(prhs[0]);
    const double* c = aiy_in(prhs[0], "policy_c", 0, 0);
    const double* a = aiy_vec(prhs[1], "a_grid", Na, NULL);
    const double* s = aiy_vec(prhs[2], "s", N, NULL);
    const double* P = aiy_in(prhs[3], "P", N, N);
    double r = aiy_scalar(prhs[4], "r"), w = aiy_scalar(prhs[5], "w");
    double beta = aiy_scalar(prhs[6], "beta"), sigma = aiy_scalar(prhs[7], "sigma");
    double amin = aiy_scalar(prhs[8], "amin");
    plhs[0] = aiy_out(Na, N);
    mxArray* pk = aiy_out(Na, N);
    double dist = 0;
    aiy_begin();
    aiy_check(aiy_egm_step(c, a, s, P, (int64_t)N, (int64_t)Na, r, w, beta, sigma, amin,
                           mxGetPr(plhs[0]), mxGetPr(pk), &dist));
    if (nlhs > 1) plhs[1] = pk; else mxDestroyArray(pk);
    if (nlhs > 2) plhs[2] = mxCreateDoubleScalar(dist);
}
