"""Full-size fixtures (tests/golden/synth_full.json): the BASELINE configs
2-5 as the bench generates them (tools/synth.c, seed 1; config 5 as the 8
per-rank shards of bench.py), cut into 8 MiB InputSplit chunks
(dmlc_amd.text_chunk_starts), parsed chunk by chunk by the GENUINE reference
(oracle/_ref, TextParserBase::FillData + the format's ParseBlock, compiled
from /root/reference), and recorded as per-array SHA-256 of the concatenated
little-endian arrays -- offsets rebased across chunks as
RowBlockContainer::Push does (row_block.h:126-168).

The text is generated and parsed in a stream (the 37 GB of config 4 never
exist at once); chunks are parsed by 8 threads (ctypes releases the GIL) and
hashed in order.  Run in the build container (needs oracle/_ref):

    python tests/golden/make_fullsize.py [name ...]

tests/test_gpu_parity.py::test_gpu_fullsize_vs_reference_hashes parses the
same inputs on the GPU and compares the hashes.
"""
import concurrent.futures as cf
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dmlc-core_amd", "python")]
from oracle import pyoracle as po  # noqa: E402
from tools import synth  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "synth_full.json")
CHUNK = 8 << 20
ARRAYS = ("offset", "label", "weight", "qid", "field", "index", "value")

# name -> (synth format, oracle format, rows, width, row0)
CONFIGS = {
    "libsvm_1m_x128": (synth.LIBSVM, po.LIBSVM, 1 << 20, 128, 0),
    "csv_1m_x256": (synth.CSV, po.CSV, 1 << 20, 256, 0),
    "libsvm_1m_x2048": (synth.LIBSVM, po.LIBSVM, 1 << 20, 2048, 0),
    # the bench's grammar / parameter variants of configs 2 and 3 (bench.py CONFIGS)
    "libsvm_nt2_1m_x128": (synth.LIBSVM, po.LIBSVM, 1 << 20, 128, 0),
    "libsvm_exact_1m_x128": (synth.LIBSVM, po.LIBSVM, 1 << 20, 128, 0),
    "csv_exact_1m_x256": (synth.CSV, po.CSV, 1 << 20, 256, 0),
    "csv_nan_1m_x256": (synth.CSV_NAN, po.CSV, 1 << 20, 256, 0),
    "libsvm_qid_1m_x128": (synth.LIBSVM_QID, po.LIBSVM, 1 << 20, 128, 0),
    "libsvm_cmt_1m_x128": (synth.LIBSVM_CMT, po.LIBSVM, 1 << 20, 128, 0),
    "libsvm_hdrs_1m_x128": (synth.LIBSVM_HDRS, po.LIBSVM, 1 << 20, 128, 0),
    "libsvm_1b_im1_1m_x128": (synth.LIBSVM_1B, po.LIBSVM, 1 << 20, 128, 0),
    "libfm_1m_x64": (synth.LIBFM, po.LIBFM, 1 << 20, 64, 0),
    # round 5: the CSV label / weight-column single pass (csv_fast_tile_sp)
    # and libfm's exact kernels at full size
    "csv_label0_1m_x256": (synth.CSV, po.CSV, 1 << 20, 256, 0),
    "csv_lw_1m_x256": (synth.CSV, po.CSV, 1 << 20, 256, 0),
    "libfm_exact_1m_x64": (synth.LIBFM, po.LIBFM, 1 << 20, 64, 0),
    # round 6: integer DTypes (glibc strtoll, csv_parser.h:99-105) and 64-bit
    # indices (data.cc:214-221's Parser<uint64_t, .> registrations)
    "csv_i32_1m_x256": (synth.CSV, po.CSV, 1 << 20, 256, 0),
    "csv_sp_i64_1m_x256": (synth.CSV_SP, po.CSV, 1 << 20, 256, 0),
    "libsvm_w64_1m_x128": (synth.LIBSVM, po.LIBSVM, 1 << 20, 128, 0),
    # round 6: words and -inf values on every eighth row (svm_fast.h dirty_rewrite)
    "libsvm_dirty_1m_x128": (synth.LIBSVM_DIRTY, po.LIBSVM, 1 << 20, 128, 0),
    # round 6: a "NaN(x)" field on every 64th row (csv_fast.h: no longer the exact kernels)
    "csv_dirty_1m_x256": (synth.CSV_NANP, po.CSV, 1 << 20, 256, 0),
}
for _r in range(8):  # config 5: bench.py's rank r shard of 32M x 64 (4M rows from row r * 4M)
    CONFIGS["libsvm_32m_x64_part%d" % _r] = (synth.LIBSVM, po.LIBSVM, 4 << 20, 64, _r * (4 << 20))
# parser arguments (the reference's URI args) per config, for the reference
# and the GPU alike; FLAGS: GPU-only dmlc_amd_params.flags (the result must not
# depend on them) and the path the GPU must report (0 single pass, 1 exact)
PARAMS = {
    "libsvm_nt2_1m_x128": {"nthread": 2},
    "libsvm_1b_im1_1m_x128": {"indexing_mode": -1},
    "csv_label0_1m_x256": {"label_column": 0},
    "csv_lw_1m_x256": {"label_column": 3, "weight_column": 7},
}
# value DType and index width per config (the reference's Parser<IndexType,
# DType> instantiation; default uint32_t / float)
TYPES = {"csv_i32_1m_x256": ("i32", 32), "csv_sp_i64_1m_x256": ("i64", 32), "libsvm_w64_1m_x128": ("f32", 64)}


def ref_kw(name):
    """The reference-side arguments of a config (pyoracle.params)."""
    kw = dict(PARAMS.get(name, {}))
    if name in TYPES:
        vt, ib = TYPES[name]
        kw.update(value_kind={"f32": po.F32, "i32": po.I32, "i64": po.I64}[vt], index_bits=ib)
    return kw


def gpu_kw(name):
    """The GPU-side arguments of a config (dmlc_amd.make_params)."""
    kw = dict(PARAMS.get(name, {}))
    if name in TYPES:
        vt, ib = TYPES[name]
        kw.update(value_type=vt, index_bits=ib)
    return kw


FLAGS = {"libsvm_exact_1m_x128": ("exact", 1), "csv_exact_1m_x256": ("exact", 1), "libfm_exact_1m_x64": ("exact", 1)}


def stream_chunks(sfmt, rows, width, row0, block_rows):
    """InputSplit chunks of the generated text, in order, as bytes
    (dmlc_amd.text_chunk_starts: cut after the last newline inside each 8 MiB
    buffer; a record longer than the buffer grows it)."""
    buf = bytearray()
    r = 0
    while True:
        while len(buf) <= CHUNK and r < rows:
            n = min(block_rows, rows - r)
            t, _ = synth.rows(sfmt, n, width, seed=1, row0=row0 + r)
            buf += t.tobytes()
            r += n
        if r >= rows and len(buf) <= CHUNK:
            if buf:
                yield bytes(buf)
            return
        lim = CHUNK
        while True:
            q = max(buf.rfind(b"\n", 1, lim), buf.rfind(b"\r", 1, lim))
            if q > 0:
                e = q + 1
                break
            lim *= 2
            while len(buf) <= lim and r < rows:
                n = min(block_rows, rows - r)
                t, _ = synth.rows(sfmt, n, width, seed=1, row0=row0 + r)
                buf += t.tobytes()
                r += n
            if len(buf) <= lim:
                e = len(buf)
                break
        yield bytes(buf[:e])
        del buf[:e]


def parse_batch(chunks, ofmt, kw):
    offs = np.cumsum([0] + [len(c) for c in chunks]).tolist()
    return po.ref_parse_chunks(b"".join(chunks), offs, fmt=ofmt, **kw)


def run(name):
    sfmt, ofmt, rows, width, row0 = CONFIGS[name]
    kw = ref_kw(name)
    block_rows = max(1, (16 << 20) // (width * 16))
    hs = {k: hashlib.sha256() for k in ARRAYS}
    sizes = {k: 0 for k in ARRAYS}
    nbytes = nchunks = 0
    base = 0  # index entries before the batch (offset rebasing)
    first_chunk_sha = None
    t0 = time.time()

    def consume(out):
        nonlocal base
        if out["status"] != 0:  # the reference refused the input: no fixture
            raise SystemExit("%s: reference error %s" % (name, out["msg"]))
        off = np.asarray(out["offset"], dtype=np.uint64)
        if sizes["offset"]:
            off = off[1:]  # the batch's leading 0 is the previous batch's closing offset
        off = off + np.uint64(base)
        hs["offset"].update(off.tobytes())
        sizes["offset"] += off.size
        for k in ARRAYS[1:]:
            a = np.ascontiguousarray(out[k])
            hs[k].update(a.tobytes())
            sizes[k] += a.size
        base += len(out["index"])

    batch, pending = [], []
    with cf.ThreadPoolExecutor(8) as ex:
        for ch in stream_chunks(sfmt, rows, width, row0, block_rows):
            if first_chunk_sha is None:
                first_chunk_sha = hashlib.sha256(ch).hexdigest()
            nbytes += len(ch)
            nchunks += 1
            batch.append(ch)
            if len(batch) == 4:
                pending.append(ex.submit(parse_batch, batch, ofmt, kw))
                batch = []
            while len(pending) > 12 or (pending and pending[0].done()):
                consume(pending.pop(0).result())
        if batch:
            pending.append(ex.submit(parse_batch, batch, ofmt, kw))
        for f in pending:
            consume(f.result())
    if sizes["offset"] == 0:
        hs["offset"].update(np.zeros(1, np.uint64).tobytes())
        sizes["offset"] = 1
    res = {"format": {po.LIBSVM: "libsvm", po.CSV: "csv", po.LIBFM: "libfm"}[ofmt], "rows": rows,
           "width": width, "row0": row0, "seed": 1, "input_bytes": nbytes, "chunks": nchunks,
           "first_chunk_sha256": first_chunk_sha, "reference": "oracle/_ref (genuine ParseBlock, nthread %d)" % kw.get("nthread", 1),
           "params": PARAMS.get(name, {}), "types": TYPES.get(name, ("f32", 32)),
           "sha256": {k: hs[k].hexdigest() for k in ARRAYS}, "sizes": sizes}
    print("%s: %.2f GB, %d chunks, %d rows, %d entries in %.0f s" % (name, nbytes / 1e9, nchunks,
                                                                        sizes["offset"] - 1, sizes["index"],
                                                                        time.time() - t0), flush=True)
    return res


def main():
    if not po.ref_available():
        raise SystemExit("oracle/_ref not built (make -C oracle ref; needs /root/reference)")
    names = sys.argv[1:] or list(CONFIGS)
    old = json.load(open(OUT)) if os.path.exists(OUT) else {}
    for n in names:
        old[n] = run(n)
        with open(OUT, "w") as f:
            json.dump(old, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
