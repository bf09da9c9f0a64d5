/* [v_new, v_old, policy_k, policy_l, policy_c, iter] = aiy_labor_vfi_solve_mex(v_old, a_grid,
 *     s, P, labor_choice, r, w, beta, sigma, psi, eta, tol, max_iter [, v_new, policy_k,
 *     policy_l, policy_c])
 * Replaces Aiyagari_Endogenous_Labor_VFI.m:64-122 (GE copy :171-228).  The optional trailing
 * arrays are the values the script's workspace holds from the previous solve (kept for states
 * with no feasible choice, :85). */
#include "mexcommon.h"
void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    aiy_nargs(nrhs, 13, 17, nlhs, 6, "[v_new,v_old,policy_k,policy_l,policy_c,iter] = aiy_labor_vfi_solve_mex(v_old,a_grid,s,P,labor_choice,r,w,beta,sigma,psi,eta,tol,max_iter[,v_new,policy_k,policy_l,policy_c])");
    mwSize N = mxGetM(prhs[0]), Na = mxGetN(prhs[0]), Nl = 0;
    aiy_in(prhs[0], "v_old", 0, 0);
    const double* a = aiy_vec(prhs[1], "a_grid", Na, NULL);
    const double* s = aiy_vec(prhs[2], "s", N, NULL);
    const double* P = aiy_in(prhs[3], "P", N, N);
    const double* L = aiy_vec(prhs[4], "labor_choice", 0, &Nl);
    double r = aiy_scalar(prhs[5], "r"), w = aiy_scalar(prhs[6], "w");
    double beta = aiy_scalar(prhs[7], "beta"), sigma = aiy_scalar(prhs[8], "sigma");
    double psi = aiy_scalar(prhs[9], "psi"), eta = aiy_scalar(prhs[10], "eta");
    double tol = aiy_scalar(prhs[11], "tol");
    int64_t max_iter = (int64_t)aiy_scalar(prhs[12], "max_iter");
    mxArray* vo = aiy_copy(prhs[0]);
    mxArray* outs[4];
    const char* names[4] = {"v_new", "policy_k", "policy_l", "policy_c"};
    for (int q = 0; q < 4; ++q) {
        if (nrhs > 13 + q) {
            aiy_in(prhs[13 + q], names[q], N, Na);
            outs[q] = aiy_copy(prhs[13 + q]);
        } else {
            outs[q] = aiy_out(N, Na);
        }
    }
    int64_t it = 0;
    aiy_begin();
    int rc = aiy_labor_vfi_solve(mxGetPr(vo), a, s, P, L, (int64_t)N, (int64_t)Na, (int64_t)Nl, r, w,
                                 beta, sigma, psi, eta, tol, max_iter, mxGetPr(outs[0]),
                                 mxGetPr(outs[1]), mxGetPr(outs[2]), mxGetPr(outs[3]), NULL, &it);
    aiy_check(rc);
    plhs[0] = outs[0];
    if (nlhs > 1) plhs[1] = vo; else mxDestroyArray(vo);
    for (int q = 1; q < 4; ++q) {
        if (nlhs > q + 1) plhs[q + 1] = outs[q]; else mxDestroyArray(outs[q]);
    }
    if (nlhs > 5) plhs[5] = mxCreateDoubleScalar((double)it);
}
