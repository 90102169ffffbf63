"""Phase breakdown of the single-pass libsvm kernel (diagnostic build).

Loads dmlc-core_amd/lib/libdmlc_amd_stamps.so (make -C dmlc-core_amd stamps),
parses a synthetic shard, and prints the mean shader cycles each tile spends
per phase: 1->2 staging, 2->3 classify, 3->4 roles + block scan,
4->5 run lists, 5->6 first decode batch, 6->7 look-back, 7->8 stores.  Stamp values never feed an output.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dmlc-core_amd", "python")]

import dmlc_amd  # noqa: E402
from tools import synth  # noqa: E402

PHASES = ["stage", "classify", "roles+scan", "lists", "batch decode", "look-back", "stores"]
SLOTS = 20  # fast_common.h kStampSlots


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    width = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    kind = {"libsvm": synth.LIBSVM, "qid": synth.LIBSVM_QID, "cmt": synth.LIBSVM_CMT,
            "hdrs": synth.LIBSVM_HDRS}[
        sys.argv[3] if len(sys.argv) > 3 else "libsvm"]
    dmlc_amd.LIB_PATH = os.path.join(ROOT, "dmlc-core_amd", "lib", "libdmlc_amd_stamps.so")
    L = dmlc_amd.lib()
    L.dmlc_amd_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    import torch
    text, _ = synth.rows(kind, rows, width, seed=1)
    starts = dmlc_amd.text_chunk_starts(text)
    d_text = torch.from_numpy(text).cuda()
    d_cs = torch.from_numpy(starts).cuda()
    p = dmlc_amd.DeviceParser("libsvm")
    res = torch.zeros(16, dtype=torch.int64, device="cuda")
    counts = p.count(d_text, d_cs, result=res)
    out = p.alloc(counts)
    out["_csr"] = p.csr_of(out)
    tile, _ = dmlc_amd.fast_geometry()
    ntiles = (text.size + tile - 1) // tile
    n = min(ntiles, 1 << 17)
    for mode in ("count", "full"):
        for _ in range(3):
            if mode == "count":
                p.count_async(d_text, d_cs, res)
            else:
                p.parse_into(d_text, d_cs, out, res)
        torch.cuda.synchronize()
        st = np.zeros(n * SLOTS, dtype=np.uint64)
        assert L.dmlc_amd_debug_stamps(st.ctypes.data, st.nbytes) == 0
        st = st.reshape(n, SLOTS).astype(np.int64)
        last = 8 if mode == "full" else 4
        d = np.diff(st[:, 1:last + 1], axis=1)
        rt = st[:, 0]
        print("%s: %d tiles, wall span of tile starts %.3f ms (100 MHz clock)"
              % (mode, n, (rt.max() - rt.min()) / 1e5))
        for i in range(d.shape[1]):
            col = d[:, i]
            print("  %-14s mean %8.0f cyc  p50 %8.0f  p99 %8.0f" % (PHASES[i], col.mean(), np.median(col),
                                                                   np.percentile(col, 99)))
        print("  total          mean %8.0f cyc" % d.sum(axis=1).mean())
        if mode == "full":  # sub-phases (thread 0): stage issue / wait; classify compute / chunk list / barrier
            for name, a0, a1 in (("  stage issue", 1, 11), ("  stage wait+sync", 11, 2), ("  classify body", 2, 9),
                                 ("  chunk list end", 9, 10), ("  classify barrier", 10, 3)):
                col = st[:, a1] - st[:, a0]
                print("  %-18s mean %8.0f cyc  p50 %8.0f" % (name, col.mean(), np.median(col)))
        if mode == "full":  # the slowest tiles (e.g. the comment / dirty-line pass) and their successors' wait
            cls = st[:, 3] - st[:, 2]
            top = np.argsort(cls)[::-1][:6]
            print("  slowest classify (tile: cycles): %s" % ", ".join("%d: %d" % (k, cls[k]) for k in top))
            hz = st[:, 12] > st[:, 2]  # tiles that took the comment / dirty-line pass this run
            if hz.any():
                for name, a0, a1 in (("comment pass", 2, 12), ("  erase", 10, 16), ("    masks+prehalo", 10, 17),
                                     ("    scan 1", 17, 18), ("    scan 2", 18, 19), ("    blank+sync", 19, 16),
                                     ("  reclassify", 16, 12),
                                     ("dirty: walk", 12, 13), ("dirty: rest", 13, 14)):
                    sel = hz & (st[:, a1] > 0) & (st[:, a0] > 0)
                    if not sel.any():
                        continue
                    col = (st[:, a1] - st[:, a0])[sel]
                    print("  %-14s %d tiles mean %8.0f cyc  max %8.0f" % (name, sel.sum(), col.mean(), col.max()))
            lbk = d[:, 5]
            print("  look-back p99.9 %.0f max %.0f; tiles with look-back > 40k cycles: %d"
                  % (np.percentile(lbk, 99.9), lbk.max(), int((lbk > 40000).sum())))
        rounds = st[:, 15]
        print("  look-back rounds: mean %.2f p50 %.0f p99 %.0f max %d"
              % (rounds.mean(), np.median(rounds), np.percentile(rounds, 99), rounds.max()))


if __name__ == "__main__":
    main()
