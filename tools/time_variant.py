"""Time dmlc_amd_parse (full call, HBM-resident) for ablation variants without
checking results: DMLC_AMD_LIB=<variant.so> python tools/time_variant.py [config].
Diagnostic only; bench.py is the measured number."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dmlc-core_amd", "python")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import dmlc_amd  # noqa: E402
from tools import synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "libsvm"
fmt, rows, width, kind = {"libsvm": ("libsvm", 1 << 20, 128, synth.LIBSVM), "csv": ("csv", 1 << 20, 256, synth.CSV),
                          "qid": ("libsvm", 1 << 20, 128, synth.LIBSVM_QID),
                          "cmt": ("libsvm", 1 << 20, 128, synth.LIBSVM_CMT),
                          "hdrs": ("libsvm", 1 << 20, 128, synth.LIBSVM_HDRS),
                          "dirty": ("libsvm", 1 << 20, 128, synth.LIBSVM_DIRTY),
                          "csv_dirty": ("csv", 1 << 20, 256, synth.CSV_NANP),
                          "libfm": ("libfm", 1 << 20, 64, synth.LIBFM),
                          "csv_nan": ("csv", 1 << 20, 256, synth.CSV_NAN),
                          "exact": ("libsvm", 1 << 20, 128, synth.LIBSVM),
                          "csv_exact": ("csv", 1 << 20, 256, synth.CSV),
                          "libfm_exact": ("libfm", 1 << 20, 64, synth.LIBFM)}[cfg]
text, _ = synth.rows(kind, rows, width, seed=1)
starts = dmlc_amd.text_chunk_starts(text)
dev = torch.device("cuda", 0)
d_text = torch.from_numpy(text).to(dev)
d_starts = torch.from_numpy(starts).to(dev)
p = dmlc_amd.DeviceParser(fmt, flags=dmlc_amd.FLAG_EXACT if cfg.endswith("exact") else 0,
                          tile_bytes=int(os.environ.get("TILE_BYTES", "0")))
res = torch.zeros(16, dtype=torch.int64, device=dev)
counts = p.count(d_text, d_starts, result=res)
out = p.alloc(counts)
out["_csr"] = p.csr_of(out)
for _ in range(3):
    p.parse_into(d_text, d_starts, out, res)
torch.cuda.synchronize()
dmlc_amd.profile_begin()
t0 = time.perf_counter()
for _ in range(10):
    p.parse_into(d_text, d_starts, out, res)
torch.cuda.synchronize()
call_ms = (time.perf_counter() - t0) * 100.0  # per call, whole pipeline
ms, n, name = dmlc_amd.profile_end()
r = res.cpu().numpy().view(np.uint64)
print("tile=%s %s %s %.4f ms call %.3f ms path=%d err=%#x res15=%d" % (os.environ.get("TILE_BYTES", "0"),
                                                          os.path.basename(os.environ.get("DMLC_AMD_LIB", "default")),
                                                  name, ms / max(n, 1), call_ms, int(r[9]), int(r[8]), int(r[15])))
