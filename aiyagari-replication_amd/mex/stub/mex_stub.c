/* Test-only implementation of the stub mx API (see mex.h).  mexErrMsgIdAndTxt longjmps back
 * to stub_call(), like MATLAB unwinding to the prompt, so gateway argument validation can be
 * unit-tested.  Arrays are column-major, as in MATLAB. */
#include <setjmp.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mex.h"

struct mxArray_tag {
    mxClassID cls;
    mwSize ndim;
    mwSize dims[4];
    void* data;
};

static jmp_buf g_jmp;
static char g_err_id[128], g_err_msg[1024];

static size_t esize(mxClassID c) { return c == mxINT32_CLASS ? 4 : 8; }

mxArray* mxCreateNumericArray(mwSize ndim, const mwSize* dims, mxClassID cls, mxComplexity c) {
    (void)c;
    mxArray* a = (mxArray*)calloc(1, sizeof *a);
    a->cls = cls;
    a->ndim = ndim < 2 ? 2 : ndim;
    size_t n = 1;
    for (mwSize q = 0; q < 4; ++q) a->dims[q] = 1;
    for (mwSize q = 0; q < ndim && q < 4; ++q) {
        a->dims[q] = dims[q];
        n *= dims[q];
    }
    a->data = calloc(n ? n : 1, esize(cls));
    return a;
}
mxArray* mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity c) {
    mwSize d[2] = {m, n};
    return mxCreateNumericArray(2, d, mxDOUBLE_CLASS, c);
}
mxArray* mxCreateDoubleScalar(double v) {
    mxArray* a = mxCreateDoubleMatrix(1, 1, mxREAL);
    ((double*)a->data)[0] = v;
    return a;
}
void mxDestroyArray(mxArray* a) {
    if (!a) return;
    free(a->data);
    free(a);
}
double* mxGetPr(const mxArray* a) { return (double*)a->data; }
void* mxGetData(const mxArray* a) { return a->data; }
mwSize mxGetM(const mxArray* a) { return a->dims[0]; }
mwSize mxGetN(const mxArray* a) {
    mwSize n = 1;
    for (mwSize q = 1; q < a->ndim; ++q) n *= a->dims[q];
    return n;
}
mwSize mxGetNumberOfElements(const mxArray* a) { return a->dims[0] * mxGetN(a); }
mwSize mxGetNumberOfDimensions(const mxArray* a) { return a->ndim; }
const mwSize* mxGetDimensions(const mxArray* a) { return a->dims; }
int mxIsDouble(const mxArray* a) { return a->cls == mxDOUBLE_CLASS; }
int mxIsComplex(const mxArray* a) { (void)a; return 0; }
int mxIsSparse(const mxArray* a) { (void)a; return 0; }
double mxGetScalar(const mxArray* a) {
    return a->cls == mxINT32_CLASS ? (double)((int*)a->data)[0] : ((double*)a->data)[0];
}
void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err_msg, sizeof g_err_msg, fmt, ap);
    va_end(ap);
    snprintf(g_err_id, sizeof g_err_id, "%s", id);
    longjmp(g_jmp, 1);
}
/* MATLAB keeps one exit function and one lock count per MEX file; the stub links every
 * gateway into one library, so it keeps a list of the registered exit functions (one per
 * gateway) and one lock count, which the tests read to check that calls are balanced. */
static void (*g_atexit[64])(void);
static int g_natexit = 0, g_lock = 0;
int mexAtExit(void (*fn)(void)) {
    if (g_natexit < 64) g_atexit[g_natexit++] = fn;
    return 0;
}
void mexLock(void) { ++g_lock; }
void mexUnlock(void) { --g_lock; }

/* ---- harness entry points (ctypes) ---- */
typedef void (*mexfn)(int, mxArray**, int, const mxArray**);
int stub_call(mexfn fn, int nlhs, mxArray** plhs, int nrhs, const mxArray** prhs) {
    g_err_id[0] = g_err_msg[0] = 0;
    if (setjmp(g_jmp)) return 1;
    fn(nlhs, plhs, nrhs, prhs);
    return 0;
}
const char* stub_err_id(void) { return g_err_id; }
const char* stub_err_msg(void) { return g_err_msg; }
mxArray* stub_int32_matrix(mwSize m, mwSize n) {
    mwSize d[2] = {m, n};
    return mxCreateNumericArray(2, d, mxINT32_CLASS, mxREAL);
}
mxArray* stub_double_array3(mwSize a, mwSize b, mwSize c) {
    mwSize d[3] = {a, b, c};
    return mxCreateNumericArray(3, d, mxDOUBLE_CLASS, mxREAL);
}
/* `clear mex`: run every registered exit function once (MATLAB does so when it unloads the
 * files), then forget them; returns how many ran */
int stub_clear_mex(void) {
    int n = g_natexit;
    for (int q = 0; q < n; ++q) g_atexit[q]();
    g_natexit = 0;
    return n;
}
int stub_lock_depth(void) { return g_lock; }
