"""ctypes binding of libaiyagari_hip.so (include/aiyagari_hip.h).

The product path has no CPU fallback: if the HIP library is missing or fails to load, every
entry point raises.  Status codes map to Python exceptions carrying aiy_last_error()."""
from __future__ import annotations

import ctypes as C
import os
import re
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
# AIY_HIP_LIB: another build of the same library (A/B timing of a kernel change on one box);
# the product default is the in-tree build
LIB_PATH = Path(os.environ.get("AIY_HIP_LIB") or (PKG_DIR / "libaiyagari_hip.so"))
HEADER = PKG_DIR.parent / "include" / "aiyagari_hip.h"

STATUS = {0: "AIY_OK", 1: "AIY_BAD_SHAPE", 2: "AIY_NON_FINITE", 3: "AIY_HIP_ERROR",
          4: "AIY_RCCL_ERROR", 5: "AIY_NO_DEVICE", 6: "AIY_BAD_ARG", 7: "AIY_FIND_EMPTY",
          8: "AIY_NO_MEMORY"}


class AiyError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{STATUS.get(code, code)}: {msg}")
        self.code = code
        self.status = STATUS.get(code, str(code))


_lib = None


def lib() -> C.CDLL:
    """Load the HIP library (fails loudly: there is no fallback path)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise RuntimeError(f"HIP library {LIB_PATH} not built: run __graft_entry__.build() "
                               f"or `make -C {PKG_DIR / 'csrc'}`")
        L = C.CDLL(str(LIB_PATH))
        L.aiy_last_error.restype = C.c_char_p
        _lib = L
    return _lib


def check(rc: int):
    if rc != 0:
        raise AiyError(rc, lib().aiy_last_error().decode(errors="replace"))


def declared_symbols(header: Path = HEADER):
    """Every function name the C ABI header declares."""
    text = re.sub(r"/\*.*?\*/", "", header.read_text(), flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**((?:aiy|ks)_\w+)\s*\(", text,
                                 flags=re.M)))


d = C.c_double
i64 = C.c_int64
vp = C.c_void_p
ip = C.c_int


def ptr(x):
    """Pointer to a numpy array's data or a torch tensor's device data (or None)."""
    if x is None:
        return None
    if hasattr(x, "data_ptr"):
        return C.c_void_p(x.data_ptr())
    return x.ctypes.data_as(C.c_void_p)


def stream_handle(stream=None):
    """hipStream_t of a torch stream (current stream when None)."""
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)
