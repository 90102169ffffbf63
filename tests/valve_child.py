"""TEST INFRASTRUCTURE ONLY -- child process of test_gpu_parity.py's valve test.

Loads the test-only valve build (lib/variants/libdmlc_amd_valve.so: the
single-pass write kernels always hand tile 1 over to the exact path, as the
kSpinLimit valve would) and parses multi-tile inputs through COUNT_ONLY ->
FILL_ONLY (the host parser's sequence) and through one full call; every result
must equal the oracle.  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["DMLC_AMD_LIB"] = os.path.join(ROOT, "dmlc-core_amd", "lib", "variants", "libdmlc_amd_valve.so")
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "dmlc-core_amd", "python")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import dmlc_amd  # noqa: E402
from golden_util import diff  # noqa: E402
from oracle import pyoracle as po  # noqa: E402
from tools import synth  # noqa: E402


def main():
    out = []
    for fmt, name, kind in ((po.LIBSVM, "libsvm", synth.LIBSVM), (po.CSV, "csv", synth.CSV),
                            (po.LIBFM, "libfm", None)):
        if kind is None:
            import fuzz_text
            data = fuzz_text.libfm_rows(np.random.default_rng(3), 800, 20)
        else:
            text, _ = synth.rows(kind, 600, 40, seed=5)
            data = text.tobytes()
        offs = dmlc_amd.text_chunk_starts(np.frombuffer(data, dtype=np.uint8), 1 << 16)
        o = po.parse_chunks(data, offs, fmt=fmt)
        d_text = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
        d_cs = torch.tensor(offs, device="cuda")
        p = dmlc_amd.DeviceParser(name)
        # count (single-pass, no hand-over) -> fill (tile 1 hands over: recount)
        r = p.parse(d_text, d_cs)
        h = dmlc_amd.to_host(r)
        bad = diff(h, o)
        # one full call (count and write in the same call)
        res = torch.zeros(16, dtype=torch.int64, device="cuda")
        r2 = p.alloc(r["counts"])
        p.parse_into(d_text, d_cs, r2, res)
        torch.cuda.synchronize()
        rr = res.cpu().numpy().view(np.uint64)
        h2 = dmlc_amd.to_host(r2)
        bad2 = diff(h2, o)
        out.append({"fmt": name, "bytes": len(data), "split_path": int(r["path"]), "split_error": int(r["error"]),
                    "split_diff": bad, "full_path": int(rr[9]), "full_error": int(rr[8]), "full_diff": bad2})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
