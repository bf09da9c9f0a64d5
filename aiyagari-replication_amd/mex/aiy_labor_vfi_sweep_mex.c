/* [v_new, policy_k, policy_l, policy_c, idx] = aiy_labor_vfi_sweep_mex(v_old, a_grid, s, P,
 *     labor_choice, r, w, beta, sigma, psi, eta [, v_new, policy_k, policy_l, policy_c])
 * One sweep of Aiyagari_Endogenous_Labor_VFI.m:69-112 (GE copy :176-219): EV = beta*P*v_old,
 * the joint max over (labour level, a') in column-major order, the policies.  The optional
 * trailing arrays are the script's workspace values from the previous sweep: states with no
 * feasible choice keep them (:85).  idx (optional): the 1-based linear index into the
 * Nl x Na (labour, a') matrix, as max(total(:)) returns it (:102). */
#include "mexcommon.h"
void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    aiy_nargs(nrhs, 11, 15, nlhs, 5, "[v_new,policy_k,policy_l,policy_c,idx] = aiy_labor_vfi_sweep_mex(v_old,a_grid,s,P,labor_choice,r,w,beta,sigma,psi,eta[,v_new,policy_k,policy_l,policy_c])");
    mwSize N = mxGetM(prhs[0]), Na = mxGetN(prhs[0]), Nl = 0;
    const double* v = aiy_in(prhs[0], "v_old", 0, 0);
    const double* a = aiy_vec(prhs[1], "a_grid", Na, NULL);
    const double* s = aiy_vec(prhs[2], "s", N, NULL);
    const double* P = aiy_in(prhs[3], "P", N, N);
    const double* L = aiy_vec(prhs[4], "labor_choice", 0, &Nl);
    double r = aiy_scalar(prhs[5], "r"), w = aiy_scalar(prhs[6], "w");
    double beta = aiy_scalar(prhs[7], "beta"), sigma = aiy_scalar(prhs[8], "sigma");
    double psi = aiy_scalar(prhs[9], "psi"), eta = aiy_scalar(prhs[10], "eta");
    mxArray* outs[4];
    const char* names[4] = {"v_new", "policy_k", "policy_l", "policy_c"};
    for (int q = 0; q < 4; ++q) {
        if (nrhs > 11 + q) {
            aiy_in(prhs[11 + q], names[q], N, Na);
            outs[q] = aiy_copy(prhs[11 + q]);
        } else {
            outs[q] = aiy_out(N, Na);
        }
    }
    int32_t* lin = (int32_t*)malloc(sizeof(int32_t) * N * Na);
    aiy_begin();
    int rc = aiy_labor_vfi_sweep(v, a, s, P, L, (int64_t)N, (int64_t)Na, (int64_t)Nl, r, w, beta,
                                 sigma, psi, eta, mxGetPr(outs[0]), mxGetPr(outs[1]),
                                 mxGetPr(outs[2]), mxGetPr(outs[3]), lin);
    if (rc == AIY_OK && nlhs > 4) {
        plhs[4] = aiy_out(N, Na);
        double* o = mxGetPr(plhs[4]);
        for (mwSize q = 0; q < N * Na; ++q) o[q] = lin[q];
    }
    free(lin);
    aiy_check(rc);
    plhs[0] = outs[0];
    for (int q = 1; q < 4; ++q) {
        if (nlhs > q) plhs[q] = outs[q]; else mxDestroyArray(outs[q]);
    }
}
