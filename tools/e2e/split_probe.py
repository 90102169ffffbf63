"""Diagnostic: time the host text InputSplit alone (dmlc_amd_host_split over
a file in the page cache) next to the end-to-end driver, to see which side
bounds the end-to-end rate.  usage: python tools/e2e/split_probe.py"""
import ctypes
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT]
from tools import synth  # noqa: E402

L = ctypes.CDLL(os.path.join(ROOT, "dmlc-core_amd", "lib", "libdmlc_amd_host.so"))
L.dmlc_amd_host_split.argtypes = [ctypes.c_char_p, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint64,
                                  ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p),
                                  ctypes.POINTER(ctypes.c_uint64)]
L.dmlc_amd_host_free.argtypes = [ctypes.c_void_p]
text, _ = synth.rows(synth.LIBSVM, 1 << 20, 128, seed=1)
path = os.path.join(os.environ.get("TMPDIR", tempfile.gettempdir()), "probe.txt")
open(path, "wb").write(text.tobytes())
for _ in range(2):
    buf, off, n = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64()
    t0 = time.perf_counter()
    L.dmlc_amd_host_split(path.encode(), 0, 1, 8 << 20, ctypes.byref(buf), ctypes.byref(off), ctypes.byref(n))
    dt = time.perf_counter() - t0
    L.dmlc_amd_host_free(buf)
    L.dmlc_amd_host_free(off)
    print(json.dumps({"split_only_s": round(dt, 3), "GBps": round(text.size / dt / 1e9, 2)}))
exe = os.path.join(ROOT, "tools", "e2e", "_build", "e2e_bench")
print(subprocess.run([exe, path, "libsvm", "3"], capture_output=True, text=True, timeout=600).stdout)
os.remove(path)
