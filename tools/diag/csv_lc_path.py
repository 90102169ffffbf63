"""Diagnostic: which gate value sends synthetic CSV with a label column to the exact path."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dmlc-core_amd", "python")]
import numpy as np, torch
import dmlc_amd as dm
from tools import synth
text, _ = synth.rows(synth.CSV, 6000, 256, seed=17)
offs = dm.text_chunk_starts(text, 1 << 20)
d_text = torch.from_numpy(text).cuda()
d_cs = torch.from_numpy(offs).cuda()
for lc in (None, 0, 5):
    for rep in range(3):
        kw = {} if lc is None else {"label_column": lc}
        p = dm.DeviceParser("csv", **kw)
        res = torch.zeros(16, dtype=torch.int64, device="cuda")
        c = p.count(d_text, d_cs, result=res)
        r1 = res.cpu().numpy().view(np.uint64).copy()
        out = p.parse(d_text, d_cs)
        print("lc", lc, "count gate/path", int(r1[9]), "err", hex(int(r1[8])), "full path", out["path"], "err", hex(out["error"]), "counts", out["result_counts"][:3], flush=True)
