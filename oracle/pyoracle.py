"""TEST INFRASTRUCTURE ONLY -- ctypes access to the parity checkers.

* ``oracle/_build/libdmlc_oracle.so``: the C restatement (oracle/dmlc_oracle.c).
* ``oracle/_ref/libdmlc_ref.so``: the genuine reference compiled from
  /root/reference sources (oracle/ref_harness.cc).  Present in this container
  after ``make -C oracle ref``; travels to the GPU box as a built file.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this
module; the product path (dmlc-core_amd/) never imports it.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIBSVM, CSV, LIBFM = 0, 1, 2
F32, I32, I64 = 0, 1, 2
_VAL_DTYPE = {F32: np.float32, I32: np.int32, I64: np.int64}


class Params(ctypes.Structure):
    _fields_ = [("format", ctypes.c_int32), ("index_bits", ctypes.c_int32),
                ("value_kind", ctypes.c_int32), ("indexing_mode", ctypes.c_int32),
                ("label_column", ctypes.c_int32), ("weight_column", ctypes.c_int32),
                ("delimiter", ctypes.c_int32), ("nthread", ctypes.c_int32)]


class Csr(ctypes.Structure):
    _fields_ = [("n_rows", ctypes.c_uint64), ("n_index", ctypes.c_uint64),
                ("n_value", ctypes.c_uint64), ("n_weight", ctypes.c_uint64),
                ("n_qid", ctypes.c_uint64), ("n_field", ctypes.c_uint64),
                ("n_label", ctypes.c_uint64),
                ("offset", ctypes.c_void_p), ("label", ctypes.c_void_p),
                ("weight", ctypes.c_void_p), ("qid", ctypes.c_void_p),
                ("field", ctypes.c_void_p), ("index", ctypes.c_void_p),
                ("value", ctypes.c_void_p), ("n_blocks", ctypes.c_uint64),
                ("block_rows", ctypes.c_void_p), ("block_index", ctypes.c_void_p),
                ("block_value", ctypes.c_void_p), ("block_weight", ctypes.c_void_p),
                ("block_qid", ctypes.c_void_p), ("status", ctypes.c_int32),
                ("msg", ctypes.c_char * 256)]


class Chunks(ctypes.Structure):
    _fields_ = [("n_chunks", ctypes.c_uint64), ("off", ctypes.c_void_p), ("buf", ctypes.c_void_p)]


def params(fmt=LIBSVM, index_bits=32, value_kind=F32, indexing_mode=0, label_column=-1,
           weight_column=-1, delimiter=",", nthread=1):
    return Params(fmt, index_bits, value_kind, indexing_mode, label_column, weight_column,
                  ord(delimiter) if isinstance(delimiter, str) else int(delimiter), nthread)


def _arr(ptr, n, dtype):
    if n == 0 or not ptr:
        return np.zeros(0, dtype=dtype)
    itemsize = np.dtype(dtype).itemsize
    buf = (ctypes.c_char * (n * itemsize)).from_address(ptr)
    return np.frombuffer(bytes(buf), dtype=dtype).copy()


def _csr_to_dict(c, value_kind, index_bits):
    vt = _VAL_DTYPE[value_kind]
    it = np.uint32 if index_bits == 32 else np.uint64
    nb = c.n_blocks
    return {
        "status": c.status, "msg": c.msg.decode(errors="replace"),
        "offset": _arr(c.offset, c.n_rows + 1, np.uint64),
        "label": _arr(c.label, c.n_label, vt),
        "weight": _arr(c.weight, c.n_weight, np.float32),
        "qid": _arr(c.qid, c.n_qid, np.uint64),
        "field": _arr(c.field, c.n_field, np.uint64).astype(it),
        "index": _arr(c.index, c.n_index, np.uint64).astype(it),
        "value": _arr(c.value, c.n_value, vt),
        "blocks": {k: _arr(getattr(c, "block_" + k), nb, np.uint64)
                   for k in ("rows", "index", "value", "weight", "qid")},
    }


_ORACLE = None
_REF = None


def oracle_lib():
    global _ORACLE
    if _ORACLE is None:
        path = os.path.join(HERE, "_build", "libdmlc_oracle.so")
        if not os.path.exists(path):
            subprocess.check_call(["make", "-s", "-C", HERE])
        L = ctypes.CDLL(path)
        L.dmo_parse_float.restype = ctypes.c_float
        L.dmo_parse_float.argtypes = [ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.POINTER(ctypes.c_void_p)]
        for fn in ("dmo_parse_chunk", "dmo_parse_block"):
            getattr(L, fn).argtypes = [ctypes.c_void_p, ctypes.c_size_t,
                                       ctypes.POINTER(Params), ctypes.POINTER(Csr)]
        L.dmo_csr_init.argtypes = [ctypes.POINTER(Csr), ctypes.c_int]
        L.dmo_csr_free.argtypes = [ctypes.POINTER(Csr)]
        L.dmo_split_text.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_uint64),
                                     ctypes.c_int, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint64,
                                     ctypes.POINTER(Chunks)]
        L.dmo_chunks_free.argtypes = [ctypes.POINTER(Chunks)]
        L.dmo_bench_chunks.restype = ctypes.c_double
        L.dmo_bench_chunks.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                       ctypes.POINTER(Params), ctypes.POINTER(ctypes.c_uint64)]
        _ORACLE = L
    return _ORACLE


def ref_available():
    return os.path.exists(os.path.join(HERE, "_ref", "libdmlc_ref.so"))


def ref_lib():
    global _REF
    if _REF is None:
        path = os.path.join(HERE, "_ref", "libdmlc_ref.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle/_ref/libdmlc_ref.so not built (make -C oracle ref)")
        L = ctypes.CDLL(path)
        L.ref_parse_block.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(Params),
                                      ctypes.POINTER(Csr)]
        L.ref_parse_uri.argtypes = [ctypes.c_char_p, ctypes.c_uint, ctypes.c_uint, ctypes.c_char_p,
                                    ctypes.c_int, ctypes.c_int, ctypes.POINTER(Csr),
                                    ctypes.POINTER(ctypes.c_double)]
        L.ref_split_chunks.argtypes = [ctypes.c_char_p, ctypes.c_uint, ctypes.c_uint,
                                       ctypes.POINTER(Chunks)]
        L.ref_parse_chunks.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(Params),
                                       ctypes.POINTER(Csr)]
        L.ref_parse_float.restype = ctypes.c_float
        L.ref_parse_float.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_size_t)]
        L.ref_bench_blocks.restype = ctypes.c_double
        L.ref_bench_blocks.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]
        _REF = L
    return _REF


def _as_bytes(data):
    if isinstance(data, str):
        data = data.encode("latin-1")
    if isinstance(data, np.ndarray):
        data = data.tobytes()
    return bytes(data)


def _run(fn, data, prm):
    raw = _as_bytes(data)
    buf = ctypes.create_string_buffer(raw, len(raw) + 1)
    c = Csr()
    oracle_lib().dmo_csr_init(ctypes.byref(c), prm.value_kind)
    fn(ctypes.cast(buf, ctypes.c_void_p), len(raw), ctypes.byref(prm), ctypes.byref(c))
    out = _csr_to_dict(c, prm.value_kind, prm.index_bits)
    oracle_lib().dmo_csr_free(ctypes.byref(c))
    return out


def parse_block(data, **kw):
    """Oracle: one ParseBlock over the whole buffer (unittest_parser.cc seam)."""
    return _run(oracle_lib().dmo_parse_block, data, params(**kw))


def parse_chunk(data, **kw):
    """Oracle: one InputSplit chunk through TextParserBase::FillData."""
    return _run(oracle_lib().dmo_parse_chunk, data, params(**kw))


def parse_chunks(data, chunk_offsets, **kw):
    """Oracle: a sequence of chunks (contiguous in `data`), concatenated."""
    raw = _as_bytes(data)
    outs = [parse_chunk(raw[int(a):int(b)], **kw) for a, b in zip(chunk_offsets[:-1], chunk_offsets[1:])]
    return concat(outs)


def concat(outs):
    """RowBlockContainer::Push-style concatenation of several results."""
    res = {"status": 0, "msg": ""}
    for o in outs:
        if o["status"] and not res["status"]:
            res["status"], res["msg"] = o["status"], o["msg"]
    offs = [np.zeros(1, np.uint64)]
    shift = np.uint64(0)
    for o in outs:
        offs.append(o["offset"][1:] + shift)
        shift = shift + np.uint64(o["offset"][-1])
    res["offset"] = np.concatenate(offs)
    for k in ("label", "weight", "qid", "field", "index", "value"):
        res[k] = np.concatenate([o[k] for o in outs]) if outs else np.zeros(0)
    res["blocks"] = {k: np.concatenate([o["blocks"][k] for o in outs]) if outs else np.zeros(0, np.uint64)
                     for k in ("rows", "index", "value", "weight", "qid")}
    return res


def parse_float(s):
    """Oracle ParseFloat over a NUL-terminated string: (value, bytes consumed)."""
    raw = _as_bytes(s)
    buf = ctypes.create_string_buffer(raw, len(raw) + 1)
    base = ctypes.addressof(buf)
    end = ctypes.c_void_p()
    v = oracle_lib().dmo_parse_float(base, base + len(raw), ctypes.byref(end))
    return v, (end.value or base) - base


def split_text(files, rank=0, nsplit=1, buffer_bytes=8 << 20):
    """Oracle InputSplit restatement: list of chunk byte strings."""
    raws = [_as_bytes(f) for f in files]
    bufs = [ctypes.create_string_buffer(r, len(r) + 1) for r in raws]
    arr = (ctypes.c_char_p * len(raws))(*[ctypes.cast(b, ctypes.c_char_p) for b in bufs])
    sizes = (ctypes.c_uint64 * len(raws))(*[len(r) for r in raws])
    c = Chunks()
    oracle_lib().dmo_split_text(arr, sizes, len(raws), rank, nsplit, buffer_bytes, ctypes.byref(c))
    off = _arr(c.off, c.n_chunks + 1, np.uint64)
    data = _arr(c.buf, int(off[-1]), np.uint8).tobytes() if c.n_chunks else b""
    oracle_lib().dmo_chunks_free(ctypes.byref(c))
    return [data[int(a):int(b)] for a, b in zip(off[:-1], off[1:])]


def bench_chunks(buf, offs, fmt=LIBSVM, nthread=1, use_ref=None):
    """CPU-baseline timing (bench.py only): parse the chunks buf[offs[i]:offs[i+1]].

    Uses the genuine reference's ParseBlock (oracle/_ref, ``nthread`` threads
    each taking whole chunks) when it is built, else the C restatement on one
    thread.  Returns (seconds, nnz, kind, threads)."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    nch = len(offs) - 1
    nnz = ctypes.c_uint64(0)
    if use_ref is None:
        use_ref = ref_available()
    if use_ref:
        secs = ref_lib().ref_bench_blocks(buf.ctypes.data, offs.ctypes.data, nch, fmt, nthread,
                                          ctypes.byref(nnz))
        return secs, int(nnz.value), "reference", nthread
    prm = params(fmt=fmt)
    secs = oracle_lib().dmo_bench_chunks(buf.ctypes.data, offs.ctypes.data, nch, ctypes.byref(prm),
                                         ctypes.byref(nnz))
    return secs, int(nnz.value), "port", 1


# ------------------------------------------------------------------ reference

def ref_parse_block(data, **kw):
    prm = params(**kw)
    raw = _as_bytes(data)
    buf = ctypes.create_string_buffer(raw, len(raw) + 1)
    c = Csr()
    oracle_lib().dmo_csr_init(ctypes.byref(c), prm.value_kind)
    ref_lib().ref_parse_block(ctypes.cast(buf, ctypes.c_void_p), len(raw), ctypes.byref(prm),
                              ctypes.byref(c))
    out = _csr_to_dict(c, prm.value_kind, prm.index_bits)
    oracle_lib().dmo_csr_free(ctypes.byref(c))
    return out


def ref_parse_chunks(data, chunk_offsets, **kw):
    """Genuine reference: each chunk through TextParserBase::FillData with
    ``nthread`` ranges (the ParseNext seam of oracle/ref_harness.cc); one
    block per non-empty container.  DMLC_REF_NPROCS lifts the reference's
    omp_get_num_procs()-based thread cap for this call."""
    prm = params(**kw)
    raw = _as_bytes(data)
    buf = ctypes.create_string_buffer(raw, len(raw) + 1)
    offs = np.ascontiguousarray(chunk_offsets, dtype=np.uint64)
    c = Csr()
    oracle_lib().dmo_csr_init(ctypes.byref(c), prm.value_kind)
    old = os.environ.get("DMLC_REF_NPROCS")
    os.environ["DMLC_REF_NPROCS"] = str(2 * max(prm.nthread, 1) + 8)
    try:
        ref_lib().ref_parse_chunks(ctypes.cast(buf, ctypes.c_void_p), offs.ctypes.data, len(offs) - 1,
                                   ctypes.byref(prm), ctypes.byref(c))
    finally:
        if old is None:
            del os.environ["DMLC_REF_NPROCS"]
        else:
            os.environ["DMLC_REF_NPROCS"] = old
    out = _csr_to_dict(c, prm.value_kind, prm.index_bits)
    oracle_lib().dmo_csr_free(ctypes.byref(c))
    return out


def ref_parse_uri(uri, part=0, nparts=1, fmt="libsvm", index_bits=32, value_kind=F32):
    c = Csr()
    oracle_lib().dmo_csr_init(ctypes.byref(c), value_kind)
    secs = ctypes.c_double(0)
    ref_lib().ref_parse_uri(uri.encode(), part, nparts, fmt.encode(), index_bits, value_kind,
                            ctypes.byref(c), ctypes.byref(secs))
    out = _csr_to_dict(c, value_kind, index_bits)
    out["seconds"] = secs.value
    oracle_lib().dmo_csr_free(ctypes.byref(c))
    return out


def ref_split_chunks(uri, part=0, nparts=1):
    c = Chunks()
    ref_lib().ref_split_chunks(uri.encode(), part, nparts, ctypes.byref(c))
    off = _arr(c.off, c.n_chunks + 1, np.uint64)
    data = _arr(c.buf, int(off[-1]), np.uint8).tobytes() if c.n_chunks else b""
    oracle_lib().dmo_chunks_free(ctypes.byref(c))
    return [data[int(a):int(b)] for a, b in zip(off[:-1], off[1:])]


def ref_parse_float(s):
    raw = _as_bytes(s)
    n = ctypes.c_size_t(0)
    v = ref_lib().ref_parse_float(raw, ctypes.byref(n))
    return v, n.value
