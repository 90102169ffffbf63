"""ctypes wrapper for tools/synth.c (canonical synthetic libsvm / CSV rows)."""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

LIBSVM, CSV, LIBFM, LIBSVM_QID, LIBSVM_CMT, CSV_SP, LIBSVM_1B, CSV_NAN, LIBSVM_HDRS, LIBSVM_DIRTY, CSV_NANP = 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "_build", "libsynth.so")
        src = os.path.join(_HERE, "synth.c")
        if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
            build()
        L = ctypes.CDLL(path)
        L.synth_bound.restype = ctypes.c_size_t
        L.synth_bound.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int]
        L.synth_rows.restype = ctypes.c_size_t
        L.synth_rows.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                                 ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        _LIB = L
    return _LIB


def build():
    os.makedirs(os.path.join(_HERE, "_build"), exist_ok=True)
    import subprocess
    subprocess.check_call(["gcc", "-O2", "-fopenmp", "-fPIC", "-shared", "-o",
                           os.path.join(_HERE, "_build", "libsynth.so"),
                           os.path.join(_HERE, "synth.c")])


def rows(fmt, nrows, width, seed=1, row0=0, line_offsets=False, out=None):
    """Return (uint8 array of text, line offsets or None).

    If `out` (a writable uint8 buffer, e.g. pinned host memory) is given, the
    text is written there and a view of the written prefix is returned."""
    L = lib()
    cap = L.synth_bound(fmt, nrows, width)
    if out is None:
        buf = np.empty(cap, dtype=np.uint8)
    else:
        buf = out
        if buf.nbytes < cap:
            raise ValueError("output buffer too small: %d < %d" % (buf.nbytes, cap))
    offs = np.empty(nrows + 1, dtype=np.uint64) if line_offsets else None
    n = L.synth_rows(fmt, row0, nrows, width, seed, buf.ctypes.data, buf.nbytes,
                     offs.ctypes.data if offs is not None else None)
    if n == 0 and nrows:
        raise RuntimeError("synth buffer overflow")
    return buf[:n], offs
