/* Shared validation for the MEX / mkoctfile gateways.  Every gateway: validates class, shape and
 * real-ness of its inputs on the interpreter thread, allocates outputs with the layout of the
 * variables the call replaces, calls the C ABI (include/aiyagari_hip.h) and maps a non-OK status
 * to mexErrMsgIdAndTxt("aiy:<STATUS>", ...).  No C++ objects are alive when mexErrMsgIdAndTxt
 * longjmps: the gateways are plain C and the library frees its own scratch before returning. */
#ifndef AIY_MEXCOMMON_H
#define AIY_MEXCOMMON_H
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "aiyagari_hip.h"
#include "mex.h"

static const char* aiy_status_id(int rc) {
    switch (rc) {
        case AIY_BAD_SHAPE: return "aiy:BAD_SHAPE";
        case AIY_NON_FINITE: return "aiy:NON_FINITE";
        case AIY_HIP_ERROR: return "aiy:HIP_ERROR";
        case AIY_RCCL_ERROR: return "aiy:RCCL_ERROR";
        case AIY_NO_DEVICE: return "aiy:NO_DEVICE";
        case AIY_BAD_ARG: return "aiy:BAD_ARG";
        case AIY_FIND_EMPTY: return "aiy:FIND_EMPTY";
        case AIY_NO_MEMORY: return "aiy:NO_MEMORY";
        default: return "aiy:ERROR";
    }
}
/* Lifecycle.  The library keeps device buffers across calls; every gateway
 * registers aiy_release_all with mexAtExit on its first call, so `clear all` / `clear mex`
 * (Krusell_Smith_VFI.m:2) frees them, and holds mexLock while a library call runs (aiy_begin ..
 * aiy_check), so the file cannot be cleared under a solve.  Every error path unlocks first:
 * mexErrMsgIdAndTxt longjmps. */
static int aiy_locked = 0;
static void aiy_mex_release(void) { (void)aiy_release_all(); }
static void aiy_unlock(void) {
    if (aiy_locked) {
        mexUnlock();
        aiy_locked = 0;
    }
}
static void aiy_err(const char* id, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    aiy_unlock();
    mexErrMsgIdAndTxt(id, "%s", buf);
}
static void aiy_begin(void) {
    static int registered = 0;
    if (!registered) {
        mexAtExit(aiy_mex_release);
        registered = 1;
    }
    if (!aiy_locked) {
        mexLock();
        aiy_locked = 1;
    }
}
static void aiy_check(int rc) {
    aiy_unlock();
    if (rc != AIY_OK) mexErrMsgIdAndTxt(aiy_status_id(rc), "%s", aiy_last_error());
}
static void aiy_nargs(int nrhs, int lo, int hi, int nlhs, int maxl, const char* usage) {
    if (nrhs < lo || nrhs > hi || nlhs > maxl) aiy_err("aiy:usage", "usage: %s", usage);
}
/* real double array; m, n = required rows/cols (0 = any); returns data */
static const double* aiy_in(const mxArray* a, const char* name, mwSize m, mwSize n) {
    if (!mxIsDouble(a) || mxIsComplex(a) || mxIsSparse(a))
        aiy_err("aiy:type", "%s must be a real, full double array", name);
    if ((m && mxGetM(a) != m) || (n && mxGetN(a) != n))
        aiy_err("aiy:shape", "%s must be %lu x %lu (got %lu x %lu)", name,
                          (unsigned long)m, (unsigned long)n, (unsigned long)mxGetM(a),
                          (unsigned long)mxGetN(a));
    return mxGetPr(a);
}
/* vector (row or column) of length n (0 = any); *len receives the length */
static const double* aiy_vec(const mxArray* a, const char* name, mwSize n, mwSize* len) {
    if (!mxIsDouble(a) || mxIsComplex(a) || mxIsSparse(a))
        aiy_err("aiy:type", "%s must be a real, full double vector", name);
    mwSize m = mxGetM(a), k = mxGetN(a);
    if (m != 1 && k != 1) aiy_err("aiy:shape", "%s must be a vector", name);
    mwSize l = m * k;
    if (n && l != n)
        aiy_err("aiy:shape", "%s must have %lu elements (got %lu)", name,
                          (unsigned long)n, (unsigned long)l);
    if (len) *len = l;
    return mxGetPr(a);
}
static double aiy_scalar(const mxArray* a, const char* name) {
    if (!mxIsDouble(a) || mxIsComplex(a) || mxGetNumberOfElements(a) != 1)
        aiy_err("aiy:type", "%s must be a real double scalar", name);
    return mxGetScalar(a);
}
static mxArray* aiy_out(mwSize m, mwSize n) { return mxCreateDoubleMatrix(m, n, mxREAL); }
static mxArray* aiy_copy(const mxArray* a) {
    mxArray* o = mxCreateDoubleMatrix(mxGetM(a), mxGetN(a), mxREAL);
    memcpy(mxGetPr(o), mxGetPr(a), sizeof(double) * mxGetNumberOfElements(a));
    return o;
}
#endif
