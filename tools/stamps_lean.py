"""Phase breakdown of the lean single-pass libsvm kernel (svm_lean.h; diagnostic
stamps build, make -C dmlc-core_amd stamps): mean shader cycles per tile per
phase, thread 0's view.  Stamp values never feed an output."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dmlc-core_amd", "python")]
os.environ["DMLC_AMD_LEAN"] = "1"
import dmlc_amd  # noqa: E402
from tools import synth  # noqa: E402

PHASES = ["loads+tables", "classify+roles", "scan+publish", "lists", "decode", "look-back", "stores"]
SLOTS = 20

dmlc_amd.LIB_PATH = os.path.join(ROOT, "dmlc-core_amd", "lib", "libdmlc_amd_stamps.so")
L = dmlc_amd.lib()
L.dmlc_amd_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
import torch  # noqa: E402
text, _ = synth.rows(synth.LIBSVM, 1 << 20, 128, seed=1)
starts = dmlc_amd.text_chunk_starts(text)
d_text = torch.from_numpy(text).cuda()
d_cs = torch.from_numpy(starts).cuda()
p = dmlc_amd.DeviceParser("libsvm")
res = torch.zeros(16, dtype=torch.int64, device="cuda")
out = p.alloc(p.count(d_text, d_cs, result=res))
out["_csr"] = p.csr_of(out)
tile, _ = dmlc_amd.fast_geometry()
n = min((text.size + tile - 1) // tile, 1 << 17)
for _ in range(3):
    p.parse_into(d_text, d_cs, out, res)
torch.cuda.synchronize()
st = np.zeros(n * SLOTS, dtype=np.uint64)
assert L.dmlc_amd_debug_stamps(st.ctypes.data, st.nbytes) == 0
st = st.reshape(n, SLOTS).astype(np.int64)
d = np.diff(st[:, 1:9], axis=1)
rt = st[:, 0]
print("lean: %d tiles, wall span of tile starts %.3f ms" % (n, (rt.max() - rt.min()) / 1e5))
for i in range(d.shape[1]):
    col = d[:, i]
    print("  %-16s mean %8.0f cyc  p50 %8.0f  p99 %8.0f" % (PHASES[i], col.mean(), np.median(col), np.percentile(col, 99)))
print("  total            mean %8.0f cyc" % d.sum(axis=1).mean())
