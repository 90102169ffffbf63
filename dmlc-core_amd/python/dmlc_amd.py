"""Python binding of the MI355X parse path (ctypes over include/dmlc_amd.h).

PyTorch is used only as plumbing: device buffers (torch.cuda tensors) and the
current HIP stream.  All parsing runs in libdmlc_amd.so's HIP kernels; there is
no CPU fallback -- importing this module on a machine without the built
library, or calling parse() without a GPU, raises.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DMLC_AMD_LIB") or os.path.join(os.path.dirname(_HERE), "lib", "libdmlc_amd.so")

LIBSVM, CSV, LIBFM = 0, 1, 2
F32, I32, I64 = 0, 1, 2
ROWS, INDEX, VALUE, WEIGHT, QID, LABEL, FIELD = range(7)
FLAG_COUNT_ONLY = 1
FLAG_FILL_ONLY = 2
FLAG_EXACT = 4
FLAG_MAX_INDEX = 8  # result.max_index / max_field (RowBlockContainer::max_index, NumCol)
ERR_CAPACITY = 16
_FMT = {"libsvm": LIBSVM, "csv": CSV, "libfm": LIBFM}
_VT = {"f32": F32, "float32": F32, "i32": I32, "int32": I32, "i64": I64, "int64": I64}


class Params(ctypes.Structure):
    _fields_ = [("format", ctypes.c_int32), ("index_bits", ctypes.c_int32),
                ("value_type", ctypes.c_int32), ("indexing_mode", ctypes.c_int32),
                ("label_column", ctypes.c_int32), ("weight_column", ctypes.c_int32),
                ("delimiter", ctypes.c_int32), ("tile_bytes", ctypes.c_uint32),
                ("flags", ctypes.c_uint32), ("nthread", ctypes.c_int32), ("reserved", ctypes.c_uint32 * 2)]


class Csr(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_void_p), ("label", ctypes.c_void_p), ("weight", ctypes.c_void_p),
                ("qid", ctypes.c_void_p), ("field", ctypes.c_void_p), ("index", ctypes.c_void_p),
                ("value", ctypes.c_void_p), ("cap", ctypes.c_uint64 * 8)]


_LIB = None


def lib():
    """Load libdmlc_amd.so; raises if it was not built (no silent fallback)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("libdmlc_amd.so not built: run `make -C dmlc-core_amd` "
                               "(or __graft_entry__.build())")
        # One HIP runtime per process: PyTorch ships its own libamdhip64; load
        # it first so this library binds to the same runtime (loaded the other
        # way round, two runtimes coexist and the second sees no device).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        L.dmlc_amd_workspace_bytes.restype = ctypes.c_size_t
        L.dmlc_amd_workspace_bytes.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(Params)]
        L.dmlc_amd_parse.restype = ctypes.c_int
        L.dmlc_amd_parse.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int,
                                     ctypes.POINTER(Params), ctypes.POINTER(Csr), ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
        L.dmlc_amd_error_string.restype = ctypes.c_char_p
        L.dmlc_amd_error_string.argtypes = [ctypes.c_int]
        L.dmlc_amd_device_count.restype = ctypes.c_int
        L.dmlc_amd_abi_version.restype = ctypes.c_int
        if hasattr(L, "dmlc_amd_build_id"):  # (A/B variant libraries built from older sources lack it)
            L.dmlc_amd_build_id.restype = ctypes.c_char_p
        L.dmlc_amd_strtof_batch.restype = ctypes.c_int
        L.dmlc_amd_strtof_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p]
        L.dmlc_amd_last_hip_error.restype = ctypes.c_char_p
        L.dmlc_amd_copy.restype = ctypes.c_int
        L.dmlc_amd_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        if hasattr(L, "dmlc_amd_copy_n"):  # (absent from older diagnostic variant builds)
            L.dmlc_amd_copy_n.restype = ctypes.c_int
            L.dmlc_amd_copy_n.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p),
                                          ctypes.POINTER(ctypes.c_uint64), ctypes.c_int, ctypes.c_void_p]
        if hasattr(L, "dmlc_amd_fast_geometry"):  # (A/B builds of older sources lack it)
            L.dmlc_amd_fast_geometry.restype = ctypes.c_int
            L.dmlc_amd_fast_geometry.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]
        L.dmlc_amd_profile_begin.restype = ctypes.c_int
        L.dmlc_amd_profile_end.restype = ctypes.c_int
        L.dmlc_amd_profile_end.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int),
                                           ctypes.POINTER(ctypes.c_char_p)]
        _LIB = L
    return _LIB


def profile_begin():
    lib().dmlc_amd_profile_begin()


def profile_end():
    """-> (summed kernel ms, launches, kernel name) since profile_begin()."""
    t, n, k = ctypes.c_double(0), ctypes.c_int(0), ctypes.c_char_p()
    if lib().dmlc_amd_profile_end(ctypes.byref(t), ctypes.byref(n), ctypes.byref(k)) != 0:
        raise RuntimeError("dmlc_amd_profile_end failed")
    return t.value, n.value, (k.value or b"").decode()


EXPORTED_SYMBOLS = ("dmlc_amd_parse", "dmlc_amd_workspace_bytes", "dmlc_amd_error_string",
                    "dmlc_amd_device_count", "dmlc_amd_abi_version", "dmlc_amd_strtof_batch",
                    "dmlc_amd_profile_begin", "dmlc_amd_profile_end", "dmlc_amd_last_hip_error",
                    "dmlc_amd_copy", "dmlc_amd_copy_n", "dmlc_amd_copy_n_dev", "dmlc_amd_fast_geometry",
                    "dmlc_amd_build_id")


def fast_geometry():
    """(text bytes per single-pass tile, unit starts one tile takes) of the
    loaded library (dmlc_amd_fast_geometry)."""
    t, m = ctypes.c_uint32(0), ctypes.c_uint32(0)
    lib().dmlc_amd_fast_geometry(ctypes.byref(t), ctypes.byref(m))
    return int(t.value), int(m.value)


def make_params(fmt="libsvm", index_bits=32, value_type="f32", indexing_mode=0, label_column=-1,
                weight_column=-1, delimiter=",", tile_bytes=0, flags=0, nthread=1):
    p = Params()
    p.format = _FMT[fmt] if isinstance(fmt, str) else int(fmt)
    p.index_bits = index_bits
    p.value_type = _VT[value_type] if isinstance(value_type, str) else int(value_type)
    p.indexing_mode = indexing_mode
    p.label_column = label_column
    p.weight_column = weight_column
    p.delimiter = ord(delimiter) if isinstance(delimiter, str) else int(delimiter)
    p.tile_bytes = tile_bytes
    p.flags = flags
    p.nthread = nthread
    return p


def units_per_chunk(params):
    """ParseBlock units per chunk (FillData ranges, dmlc_amd_params.nthread)."""
    return max(int(params.nthread), 1)


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("dmlc_amd: no HIP device visible")
    return torch


def _vdt(torch, vt):
    return {F32: torch.float32, I32: torch.int32, I64: torch.int64}[vt]


class DeviceParser:
    """One parser configuration bound to the current HIP device.

    parse(text, chunk_starts) takes a device uint8 tensor and a device int64
    tensor of nchunks+1 chunk boundaries and returns device tensors."""

    def __init__(self, fmt="libsvm", **kw):
        self.params = make_params(fmt, **kw)
        self.torch = _torch()
        self._ws = None

    def _workspace(self, nbytes, nchunks):
        need = lib().dmlc_amd_workspace_bytes(nbytes, nchunks, ctypes.byref(self.params))
        if self._ws is None or self._ws.numel() < need:
            self._ws = self.torch.empty(need, dtype=self.torch.uint8, device="cuda")
        return self._ws, need

    def _call(self, text, chunk_starts, csr, chunk_table, result, params, stream):
        torch = self.torch
        nbytes = int(text.numel())
        nchunks = int(chunk_starts.numel()) - 1
        ws, need = self._workspace(nbytes, max(nchunks, 1))
        s = stream if stream is not None else torch.cuda.current_stream()
        rc = lib().dmlc_amd_parse(text.data_ptr() if nbytes else None, nbytes,
                                  chunk_starts.data_ptr() if nbytes else None, nchunks,
                                  ctypes.byref(params), ctypes.byref(csr),
                                  chunk_table.data_ptr() if chunk_table is not None else None,
                                  ws.data_ptr(), ws.numel(), result.data_ptr(), s.cuda_stream)
        if rc != 0:
            msg = lib().dmlc_amd_error_string(rc).decode()
            if rc == 33:
                msg += " (%s)" % lib().dmlc_amd_last_hip_error().decode()
            raise RuntimeError("dmlc_amd_parse: %s" % msg)

    def count(self, text, chunk_starts, stream=None, result=None):
        """Size query: exact per-slot totals (device work, then a host sync).
        The per-tile counts stay in this parser's workspace for fill()."""
        torch = self.torch
        res = result if result is not None else torch.zeros(16, dtype=torch.int64, device="cuda")
        self.count_async(text, chunk_starts, res, stream=stream)
        if stream is not None:
            stream.synchronize()
        return res.cpu().numpy().view(np.uint64)

    def count_async(self, text, chunk_starts, result, out=None, stream=None):
        """Launch the count phase (count -> scan) without a host sync."""
        p = Params.from_buffer_copy(self.params)
        p.flags |= FLAG_COUNT_ONLY
        csr = Csr() if out is None else out.get("_csr") or self.csr_of(out)
        self._call(text, chunk_starts, csr, None, result, p, stream)

    def fill_async(self, text, chunk_starts, out, result, chunk_table=None, stream=None):
        """Launch the write pass over the counts of the preceding count phase."""
        p = Params.from_buffer_copy(self.params)
        p.flags |= FLAG_FILL_ONLY
        self._call(text, chunk_starts, out.get("_csr") or self.csr_of(out), chunk_table, result, p,
                   stream)

    def alloc(self, counts):
        """Allocate exact-size outputs for the given totals."""
        torch = self.torch
        wide = self.params.index_bits == 64
        it = torch.int64 if wide else torch.int32
        vt = _vdt(torch, self.params.value_type if self.params.format == CSV else F32)
        c = [int(x) for x in counts]
        out = {
            "offset": torch.empty(c[ROWS] + 1, dtype=torch.int64, device="cuda"),
            "label": torch.empty(max(c[LABEL], 1), dtype=vt, device="cuda"),
            "weight": torch.empty(max(c[WEIGHT], 1), dtype=torch.float32, device="cuda"),
            "qid": torch.empty(max(c[QID], 1), dtype=torch.int64, device="cuda"),
            "field": torch.empty(max(c[FIELD], 1), dtype=it, device="cuda"),
            "index": torch.empty(max(c[INDEX], 1), dtype=it, device="cuda"),
            "value": torch.empty(max(c[VALUE], 1), dtype=vt, device="cuda"),
            "counts": c,
        }
        return out

    def csr_of(self, out):
        csr = Csr()
        for k in ("offset", "label", "weight", "qid", "field", "index", "value"):
            setattr(csr, k, out[k].data_ptr())
        c = out["counts"]
        caps = [c[ROWS], c[INDEX], c[VALUE], c[WEIGHT], c[QID], c[LABEL], c[FIELD], 0]
        for i, v in enumerate(caps):
            csr.cap[i] = v
        return csr

    def parse_into(self, text, chunk_starts, out, result, chunk_table=None, stream=None):
        """Launch the full pipeline into preallocated outputs (no host sync)."""
        self._call(text, chunk_starts, out["_csr"] if "_csr" in out else self.csr_of(out),
                   chunk_table, result, self.params, stream)

    def parse(self, text, chunk_starts, stream=None):
        """Count, allocate, fill; returns dict of device tensors + counts/error."""
        torch = self.torch
        res = torch.zeros(16, dtype=torch.int64, device="cuda")
        counts = self.count(text, chunk_starts, stream, result=res)
        out = self.alloc(counts)
        nchunks = int(chunk_starts.numel()) - 1
        nunits = nchunks * units_per_chunk(self.params)
        out["chunk_table"] = torch.zeros(max(nunits, 1) * 8, dtype=torch.int64, device="cuda")
        self.fill_async(text, chunk_starts, out, res,
                        chunk_table=out["chunk_table"] if nchunks > 0 else None, stream=stream)
        r = res.cpu().numpy().view(np.uint64)
        out["error"] = int(r[8])
        out["path"] = int(r[9])
        out["result_counts"] = [int(x) for x in r[:8]]
        out["max_index"], out["max_field"] = int(r[10]), int(r[11])
        return out


def build_id():
    """SHA-256 prefix of the sources the loaded library was built from."""
    L = lib()
    return L.dmlc_amd_build_id().decode() if hasattr(L, "dmlc_amd_build_id") else "unknown"


def error_code(err):
    return int(err) & 0xFFFF


def error_pos(err):
    return int(err) >> 16


def to_host(out, index_bits=32, value_type=F32):
    """Copy parse outputs to numpy with the reference's dtypes."""
    c = out["counts"]
    it = np.uint32 if index_bits == 32 else np.uint64
    vt = {F32: np.float32, I32: np.int32, I64: np.int64}[value_type]
    h = {
        "offset": out["offset"][: c[ROWS] + 1].cpu().numpy().view(np.uint64),
        "label": out["label"][: c[LABEL]].cpu().numpy().view(vt),
        "weight": out["weight"][: c[WEIGHT]].cpu().numpy().view(np.float32),
        "qid": out["qid"][: c[QID]].cpu().numpy().view(np.uint64),
        "field": out["field"][: c[FIELD]].cpu().numpy().view(it),
        "index": out["index"][: c[INDEX]].cpu().numpy().view(it),
        "value": out["value"][: c[VALUE]].cpu().numpy().view(vt),
    }
    if "chunk_table" in out:
        h["chunk_table"] = out["chunk_table"].cpu().numpy().view(np.uint64).reshape(-1, 8)
    return h


def parse_bytes(data, chunk_offsets=None, fmt="libsvm", exact=False, **kw):
    """Convenience: host bytes -> device -> parse -> host numpy dict."""
    torch = _torch()
    raw = data.encode("latin-1") if isinstance(data, str) else bytes(data)
    if chunk_offsets is None:
        chunk_offsets = [0, len(raw)] if raw else [0]
    text = torch.frombuffer(bytearray(raw), dtype=torch.uint8).cuda() if raw else \
        torch.empty(0, dtype=torch.uint8, device="cuda")
    cs = torch.tensor(np.asarray(chunk_offsets, dtype=np.int64), device="cuda")
    if exact:
        kw["flags"] = kw.get("flags", 0) | FLAG_EXACT
    p = DeviceParser(fmt, **kw)
    out = p.parse(text, cs)
    h = to_host(out, p.params.index_bits,
                p.params.value_type if p.params.format == CSV else F32)
    h["error"] = out["error"]
    h["path"] = "exact" if out["path"] else "fast"
    h["counts"] = out["counts"]
    h["units_per_chunk"] = units_per_chunk(p.params)
    return h


def strtof_batch(strings):
    """Device dmlc::strtof over a list of byte strings -> (f32 values, consumed, nan_err)."""
    torch = _torch()
    raws = [s.encode("latin-1") if isinstance(s, str) else bytes(s) for s in strings]
    offs = np.zeros(len(raws) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(r) for r in raws])
    blob = b"".join(raws) or b"\0"
    text = torch.frombuffer(bytearray(blob), dtype=torch.uint8).cuda()
    d_off = torch.tensor(offs, device="cuda")
    n = len(raws)
    out = torch.empty(max(n, 1), dtype=torch.float32, device="cuda")
    used = torch.empty(max(n, 1), dtype=torch.int32, device="cuda")
    bad = torch.empty(max(n, 1), dtype=torch.int32, device="cuda")
    rc = lib().dmlc_amd_strtof_batch(text.data_ptr(), d_off.data_ptr(), n, out.data_ptr(),
                                     used.data_ptr(), bad.data_ptr(),
                                     torch.cuda.current_stream().cuda_stream)
    if rc != 0:
        raise RuntimeError("dmlc_amd_strtof_batch failed")
    torch.cuda.synchronize()
    return out[:n].cpu().numpy(), used[:n].cpu().numpy(), bad[:n].cpu().numpy()


def chunk_check(h, fmt, nchunks, total_counts):
    """Per-unit consistency CHECKs of the reference, applied to GPU output
    (nchunks: table rows, i.e. chunks x units per chunk).

    The reference raises these from RowBlockContainer::GetBlock (row_block.h:
    174-178) and, for CSV, from ParseBlock itself (csv_parser.h:147-148); libfm
    adds field == index (libfm_parser.h:127).  Returns the first failing chunk
    index or -1."""
    f = _FMT[fmt] if isinstance(fmt, str) else fmt
    tab = h["chunk_table"][:nchunks].astype(np.int64)
    ends = np.vstack([tab[1:], np.asarray(total_counts[:8], dtype=np.int64)[None, :]])
    per = ends - tab
    for c in range(nchunks):
        rows, idx, val, w, lab, fld = (per[c, ROWS], per[c, INDEX], per[c, VALUE], per[c, WEIGHT],
                                       per[c, LABEL], per[c, FIELD])
        if f == CSV:
            if lab != 0 and lab != rows:
                return c
            if w != 0 and w != rows:
                return c
        if f == LIBFM and fld != idx:
            return c
        if rows and not (val == 0 or val == idx):
            return c
    return -1


def text_chunk_starts(text, chunk_bytes=8 << 20):
    """Chunk boundaries an InputSplit ("text", one part) would hand over for
    this buffer: each chunk ends just after the last '\\n' / '\\r' inside its
    `chunk_bytes` read buffer (LineSplitter::FindLastRecordBegin,
    src/io/line_split.cc:37-45; kBufferSize, src/io/input_split_base.h:39); a
    record longer than the buffer grows it until one fits
    (input_split_base.cc:272-291).  Returns int64 [nchunks + 1] offsets."""
    a = np.frombuffer(text, dtype=np.uint8) if not isinstance(text, np.ndarray) else text
    n = int(a.size)
    if n == 0:
        return np.zeros(1, dtype=np.int64)
    nl = np.flatnonzero((a == 10) | (a == 13)) + 1  # candidate chunk ends (record begins)
    starts = [0]
    s = 0
    while s < n:
        lim = s + chunk_bytes
        if lim >= n:
            starts.append(n)
            break
        while True:
            # last newline at p with s < p < lim; the record begins at p + 1
            j = int(np.searchsorted(nl, lim, side="right")) - 1
            if j >= 0 and int(nl[j]) - 1 > s:
                e = int(nl[j])
                break
            lim = s + (lim - s) * 2  # record longer than the buffer: grow
            if lim >= n:
                e = n
                break
        starts.append(e)
        s = e
    return np.asarray(starts, dtype=np.int64)
