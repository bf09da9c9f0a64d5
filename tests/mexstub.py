"""ctypes driver for the MEX gateways compiled against the stub mx API
(aiyagari-replication_amd/mex/libmexstub.so).  Calls mexFunction_<name> exactly as MATLAB would
(nlhs, plhs, nrhs, prhs); mexErrMsgIdAndTxt comes back as MexError(id, message)."""
import ctypes as C
from pathlib import Path

import numpy as np

LIB = Path(__file__).resolve().parents[1] / "aiyagari-replication_amd" / "mex" / "libmexstub.so"


class MexError(RuntimeError):
    def __init__(self, ident, msg):
        super().__init__(f"{ident}: {msg}")
        self.id = ident


_L = None


def lib():
    global _L
    if _L is None:
        L = C.CDLL(str(LIB))
        L.mxCreateDoubleMatrix.restype = C.c_void_p
        L.mxCreateDoubleMatrix.argtypes = [C.c_size_t, C.c_size_t, C.c_int]
        L.stub_double_array3.restype = C.c_void_p
        L.stub_double_array3.argtypes = [C.c_size_t, C.c_size_t, C.c_size_t]
        L.mxGetPr.restype = C.c_void_p
        L.mxGetPr.argtypes = [C.c_void_p]
        for f in ("mxGetM", "mxGetN", "mxGetNumberOfElements"):
            getattr(L, f).restype = C.c_size_t
            getattr(L, f).argtypes = [C.c_void_p]
        L.mxDestroyArray.argtypes = [C.c_void_p]
        L.stub_err_id.restype = C.c_char_p
        L.stub_err_msg.restype = C.c_char_p
        L.stub_call.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p]
        _L = L
    return _L


def to_mx(x):
    x = np.asarray(x, dtype=np.float64)
    L = lib()
    if x.ndim == 3:
        a = L.stub_double_array3(*x.shape)
    else:
        x2 = np.atleast_2d(x) if x.ndim < 2 else x
        a = L.mxCreateDoubleMatrix(x2.shape[0], x2.shape[1], 0)
        x = x2
    n = x.size
    buf = (C.c_double * n).from_address(L.mxGetPr(a))
    buf[:] = np.asfortranarray(x).ravel(order="F")
    return a


def from_mx(a):
    L = lib()
    m, n = L.mxGetM(a), L.mxGetN(a)
    data = np.ctypeslib.as_array((C.c_double * (m * n)).from_address(L.mxGetPr(a))).copy()
    return data.reshape((m, n), order="F")


def call(name, nlhs, *args):
    L = lib()
    fn = getattr(L, f"mexFunction_{name}")
    prhs = (C.c_void_p * max(len(args), 1))(*[to_mx(a) for a in args])
    plhs = (C.c_void_p * max(nlhs, 1))()
    rc = L.stub_call(C.cast(fn, C.c_void_p), nlhs, plhs, len(args), prhs)
    for q in range(len(args)):
        L.mxDestroyArray(prhs[q])
    if rc:
        raise MexError(L.stub_err_id().decode(), L.stub_err_msg().decode())
    outs = []
    for q in range(nlhs):
        outs.append(from_mx(plhs[q]) if plhs[q] else None)
        if plhs[q]:
            L.mxDestroyArray(plhs[q])
    return outs
