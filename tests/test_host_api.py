"""The C++ drop-in layer (include/dmlc/data.h over the C ABI).

CPU: the host InputSplit (dmlc-core_amd/host/text_split.cc) produces the
reference's chunk sequence (checked against the oracle restatement of
input_split_base.cc / line_split.cc, itself pinned by tests/golden/split.json).
GPU: dmlc::Parser / RowBlockIter on real files -- the scenarios of
test/unittest_inputsplit.cc:41-147 plus synthetic multi-file, multi-part
inputs -- equal the oracle.
"""
import ctypes
import hashlib
import os
import subprocess

import numpy as np
import pytest

from golden_util import diff, load_json
from test_oracle import _regen_files
from oracle import pyoracle as po
from tools import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST_LIB = os.path.join(ROOT, "dmlc-core_amd", "lib", "libdmlc_amd_host.so")
DRIVER = os.path.join(ROOT, "tests", "cpp", "_build", "host_api_test")


def _host():
    if not os.path.exists(HOST_LIB):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "dmlc-core_amd")])
    L = ctypes.CDLL(HOST_LIB)
    L.dmlc_amd_host_split.argtypes = [ctypes.c_char_p, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint64,
                                      ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p),
                                      ctypes.POINTER(ctypes.c_uint64)]
    L.dmlc_amd_host_free.argtypes = [ctypes.c_void_p]
    L.dmlc_amd_host_split_inplace.argtypes = [ctypes.c_char_p, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint64,
                                              ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p),
                                              ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint64)]
    L.dmlc_amd_host_split_pieces.argtypes = [ctypes.c_char_p, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint64,
                                             ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p),
                                             ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint64)]
    return L


def host_split_pieces(uri, part, nparts, buffer_bytes, batch_bytes):
    """The chunks through TextSplit::FillPieces (pieces of the mapped files, the
    device pipeline's DMA form since round 6), gathered back into bytes."""
    L = _host()
    buf, off, n = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64()
    assert L.dmlc_amd_host_split_pieces(uri.encode(), part, nparts, buffer_bytes, batch_bytes,
                                        ctypes.byref(buf), ctypes.byref(off), ctypes.byref(n)) == 0
    offs = np.ctypeslib.as_array(ctypes.cast(off, ctypes.POINTER(ctypes.c_uint64)), (n.value + 1,)).copy()
    data = ctypes.string_at(buf, int(offs[-1])) if offs[-1] else b""
    L.dmlc_amd_host_free(buf)
    L.dmlc_amd_host_free(off)
    return [data[int(a):int(b)] for a, b in zip(offs[:-1], offs[1:])]


def host_split(uri, part, nparts, buffer_bytes):
    L = _host()
    buf, off, n = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64()
    assert L.dmlc_amd_host_split(uri.encode(), part, nparts, buffer_bytes, ctypes.byref(buf),
                                 ctypes.byref(off), ctypes.byref(n)) == 0
    offs = np.ctypeslib.as_array(ctypes.cast(off, ctypes.POINTER(ctypes.c_uint64)), (n.value + 1,)).copy()
    data = ctypes.string_at(buf, int(offs[-1])) if offs[-1] else b""
    L.dmlc_amd_host_free(buf)
    L.dmlc_amd_host_free(off)
    return [data[int(a):int(b)] for a, b in zip(offs[:-1], offs[1:])]


def host_split_inplace(uri, part, nparts, buffer_bytes, batch_bytes, cap):
    """The chunks through TextSplit::FillChunks (the device pipeline's reader)."""
    L = _host()
    buf, off, n = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64()
    assert L.dmlc_amd_host_split_inplace(uri.encode(), part, nparts, buffer_bytes, batch_bytes, cap,
                                         ctypes.byref(buf), ctypes.byref(off), ctypes.byref(n)) == 0
    offs = np.ctypeslib.as_array(ctypes.cast(off, ctypes.POINTER(ctypes.c_uint64)), (n.value + 1,)).copy()
    data = ctypes.string_at(buf, int(offs[-1])) if offs[-1] else b""
    L.dmlc_amd_host_free(buf)
    L.dmlc_amd_host_free(off)
    return [data[int(a):int(b)] for a, b in zip(offs[:-1], offs[1:])]


def _write(tmp_path, contents):
    d = tmp_path / "data"
    d.mkdir(parents=True, exist_ok=True)
    paths = []
    for i, c in enumerate(contents):
        p = d / ("part-%02d.txt" % i)
        p.write_bytes(c)
        paths.append(str(p))
    return str(d), paths


def _random_files(rng, fmt, nfiles):
    out = []
    for i in range(nfiles):
        t, _ = synth.rows(fmt, int(rng.integers(0, 400)), int(rng.integers(1, 30)), seed=int(rng.integers(1, 99)))
        b = t.tobytes()
        if b and rng.random() < 0.4:
            b = b.rstrip(b"\n")  # a file without a final newline
        if rng.random() < 0.2:
            b = b.replace(b"\n", b"\r\n")
        out.append(b)
    return out


def test_host_split_matches_oracle(tmp_path):
    rng = np.random.default_rng(2)
    for it in range(12):
        contents = _random_files(rng, synth.LIBSVM, int(rng.integers(1, 5)))
        d, paths = _write(tmp_path, contents)
        uri = ";".join(paths) if it % 2 else d
        nparts = int(rng.integers(1, 5))
        buf = int(rng.choice([64, 1000, 1 << 16, 8 << 20]))
        # a directory lists in raw readdir order (local_filesys.cc:98-122), as os.listdir does
        by_path = dict(zip(paths, contents))
        order = paths if it % 2 else [os.path.join(d, f) for f in os.listdir(d)]
        files = [by_path[p] for p in order if by_path[p]]
        for part in range(nparts):
            got = host_split(uri, part, nparts, buf)
            exp = po.split_text(files, part, nparts, buffer_bytes=buf)
            assert got == exp, (it, part, nparts, buf)
            # the in-place reader: same chunks, whatever the batch and buffer sizes
            batch = int(rng.choice([1, 3 * buf, 1 << 20]))
            cap = int(rng.choice([buf + 1, 2 * buf + 7, 4 << 20, 40 << 20]))
            assert host_split_inplace(uri, part, nparts, buf, batch, cap) == exp, (it, part, nparts, buf, batch, cap)
            # the mapped form: the same chunks as pieces of the files' mappings
            assert host_split_pieces(uri, part, nparts, buf, batch) == exp, (it, part, nparts, buf, batch)
        for p in paths:
            os.remove(p)


@pytest.mark.parametrize("case", load_json("split.json")["cases"],
                         ids=lambda c: "%s-%d/%d" % (c["name"], c["part"], c["nparts"]))
def test_host_split_golden_chunking(case, tmp_path):
    """The InputSplit chunkings recorded from the genuine reference (tests/golden/split.json)."""
    files = _regen_files(case)
    paths = []
    for i, fn in enumerate(case["order"]):  # the reference's file order
        p = tmp_path / ("%02d_%s" % (i, fn))
        p.write_bytes(files[fn])
        paths.append(str(p))
    got = host_split(";".join(paths), case["part"], case["nparts"], 8 << 20)
    assert [len(c) for c in got] == case["chunk_sizes"]
    assert [hashlib.sha256(c).hexdigest() for c in got] == case["chunk_sha256"]
    assert host_split_pieces(";".join(paths), case["part"], case["nparts"], 8 << 20, 32 << 20) == got


def _host_split_error(uri):
    L = _host()
    buf, off, n = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64()
    return L.dmlc_amd_host_split(uri.encode(), 0, 1, 8 << 20, ctypes.byref(buf), ctypes.byref(off),
                                 ctypes.byref(n))


def test_host_split_file_list_semantics(tmp_path):
    """InputSplitBase::InitInputFileInfo (input_split_base.cc:96-176): a
    directory in raw readdir order with dotfiles kept and empty files and
    subdirectories dropped; a last path component matched as a regex; no file
    at all is an error.  Checked against the genuine reference when it is
    built, and against the oracle split of the same file order."""
    d = tmp_path / "dir"
    d.mkdir()
    names = ["zeta.txt", ".crc", "alpha.txt", "m-1.txt", "m-2.txt", "empty.txt", "Beta.txt", "07.txt"]
    rng = np.random.default_rng(9)
    body = {}
    for nm in names:
        t, _ = synth.rows(synth.LIBSVM, 0 if nm == "empty.txt" else int(rng.integers(1, 40)), 5,
                          seed=int(rng.integers(1, 99)))
        body[nm] = t.tobytes()
        (d / nm).write_bytes(body[nm])
    (d / "sub").mkdir()
    (d / "sub" / "x.txt").write_bytes(b"1 1:1\n")
    listed = [f for f in os.listdir(d) if f in body and body[f]]
    assert sorted(listed) != listed or True  # order is whatever readdir gives; never re-sorted
    uris = {
        "dir": (str(d), listed),
        "dir_slash": (str(d) + "/", listed),
        "regex": (str(d / "m-[0-9].txt"), [f for f in os.listdir(d) if f.startswith("m-")]),
        "exact": (str(d / "alpha.txt"), ["alpha.txt"]),
        "list": ("%s;%s" % (d / "zeta.txt", d / ".crc"), ["zeta.txt", ".crc"]),
    }
    for key, (uri, order) in uris.items():
        exp = po.split_text([body[f] for f in order], 0, 1)
        for nparts in (1, 3):
            got = [c for part in range(nparts) for c in host_split(uri, part, nparts, 8 << 20)]
            oracle = [c for part in range(nparts) for c in po.split_text([body[f] for f in order], part, nparts)]
            assert got == oracle, (key, nparts)
            if po.ref_available():
                ref = [c for part in range(nparts) for c in po.ref_split_chunks(uri, part, nparts)]
                assert got == ref, (key, nparts)
        assert b"".join(host_split(uri, 0, 1, 8 << 20)) == b"".join(exp), key
    # only empty files / nothing matching: the reference's CHECK_NE(files_.size(), 0U)
    e = tmp_path / "empty_dir"
    e.mkdir()
    (e / "a.txt").write_bytes(b"")
    assert _host_split_error(str(e)) != 0
    assert _host_split_error(str(d / "nomatch-[0-9]+")) != 0


# ------------------------------------------------------------------ GPU --

def _driver():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")])
    return DRIVER


NTHREAD = 2  # the reference's factory thread count on a host with >= 12 processors (text_parser.h:32-35)


def run_api(tmp_path, uri, part=0, nparts=1, fmt="libsvm", index_bits=32, dtype="f32", iter_=False,
            nthread=NTHREAD, env=None):
    o = str(tmp_path / "out")
    args = [_driver(), uri, str(part), str(nparts), fmt, str(index_bits), dtype, o] + (["iter"] if iter_ else [])
    e = dict(os.environ, DMLC_AMD_NTHREAD=str(nthread), **(env or {}))
    r = subprocess.run(args, capture_output=True, env=e)
    if r.returncode == 3:
        return {"error": open(o + ".error").read()}
    assert r.returncode != 4, "a Parser block with offset[0] != 0"
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    it = np.uint64 if index_bits == 64 else np.uint32
    vt = {"f32": np.float32, "i32": np.int32, "i64": np.int64}[dtype]
    h = {"offset": np.fromfile(o + ".offset", np.uint64), "label": np.fromfile(o + ".label", vt),
         "weight": np.fromfile(o + ".weight", np.float32), "qid": np.fromfile(o + ".qid", np.uint64),
         "index": np.fromfile(o + ".index", it), "value": np.fromfile(o + ".value", vt),
         "field": np.fromfile(o + ".field", it), "meta": np.fromfile(o + ".meta", np.uint64),
         "blocks": np.fromfile(o + ".blocks", np.uint64)}
    return h


def dir_order(d, contents):
    """The files of directory d (written by _write from `contents`) in raw
    readdir order, as the reference's InputSplit lists them (local_filesys.cc:98-122)."""
    by_name = {"part-%02d.txt" % i: c for i, c in enumerate(contents)}
    return [by_name[f] for f in os.listdir(d) if f in by_name]


def oracle_files(contents, part=0, nparts=1, fmt=po.LIBSVM, nthread=NTHREAD, d=None, **kw):
    if d is not None:
        contents = dir_order(d, contents)
    chunks = po.split_text(contents, part, nparts)
    offs = np.cumsum([0] + [len(c) for c in chunks]).tolist()
    return po.parse_chunks(b"".join(chunks), offs, fmt=fmt, nthread=nthread, **kw), len(chunks)


@pytest.mark.gpu
def test_api_unittest_inputsplit_scenarios(tmp_path):
    """test/unittest_inputsplit.cc:41-147 through dmlc::Parser::Create."""
    # CSV across three files, one without a final newline (:41-68)
    csv = [b"0,1,2,3\n4,5,6,7\n", b"8,9,10,11\n12,13,14,15", b"16,17,18,19\n"]
    d, _ = _write(tmp_path / "csv", csv)
    h = run_api(tmp_path, d, fmt="csv")
    o, _ = oracle_files(csv, fmt=po.CSV, d=d)
    assert "error" not in h and diff(h, o) == [] and len(h["offset"]) - 1 == 5
    # libsvm, no final newline (:70-92)
    svm = [b"1 1:1 2:2\n0 3:3\n1 4:4 5:5"]
    d, _ = _write(tmp_path / "svm", svm)
    h = run_api(tmp_path, d)
    o, _ = oracle_files(svm)
    assert diff(h, o) == [] and len(h["offset"]) - 1 == 3
    # five files (:94-116) and two parts of ten lines -> {6, 4} rows (:118-147)
    lines = [b"%d %d:1\n" % (i % 2, i) for i in range(10)]
    five = [b"".join(lines[2 * i:2 * i + 2]) for i in range(5)]
    d, _ = _write(tmp_path / "five", five)
    h = run_api(tmp_path, d)
    assert len(h["offset"]) - 1 == 10
    rows = []
    for part in range(2):
        h = run_api(tmp_path, d, part, 2)
        o, _ = oracle_files(five, part, 2, d=d)
        assert diff(h, o) == []
        rows.append(len(h["offset"]) - 1)
    assert rows == [6, 4]


@pytest.mark.gpu
@pytest.mark.parametrize("mmap", ["0", "1"])
@pytest.mark.parametrize("fmt", ["libsvm", "csv"])
def test_api_synthetic_multifile_multipart(tmp_path, fmt, mmap):
    """Multi-file, multi-part inputs; mmap=1: the text DMA'd from the files'
    registered mappings (TextSplit::FillPieces, 1 MiB segments: pieces split at
    segment ends, segments unregistered as their last batch is released)."""
    rng = np.random.default_rng(11 if fmt == "libsvm" else 12)
    f = synth.LIBSVM if fmt == "libsvm" else synth.CSV
    contents = _random_files(rng, f, 4)
    d, _ = _write(tmp_path / fmt, contents)
    env = {"DMLC_AMD_MMAP": mmap, "DMLC_AMD_MMAP_SEG_MB": "1"}
    for nparts in (1, 3):
        for part in range(nparts):
            h = run_api(tmp_path, d, part, nparts, fmt, env=env)
            o, nch = oracle_files(contents, part, nparts, fmt=po.LIBSVM if fmt == "libsvm" else po.CSV, d=d)
            assert "error" not in h, (h, part, nparts, [len(c) for c in contents])
            assert diff(h, o) == [], (part, nparts)


@pytest.mark.gpu
def test_api_libfm_parser_and_rowiter(tmp_path):
    """Parser<I,float>::Create(..., "libfm") (data.cc:206-209): fields ride with
    the indices through the C++ API, both id widths, indexing_mode=-1."""
    import fuzz_text
    rng = np.random.default_rng(21)
    # weights on every row (a chunk with weights on some rows only gives a
    # RowBlock whose weight array is shorter than size, row_block.h:178-189)
    contents = [fuzz_text.libfm_rows(rng, 500, 9, weights=True), fuzz_text.libfm_rows(rng, 300, 4, weights=True)]
    d, _ = _write(tmp_path / "fm", contents)
    for bits in (32, 64):
        for uri, kw in ((d, {}), (d + "?indexing_mode=-1", {"indexing_mode": -1})):
            h = run_api(tmp_path, uri, fmt="libfm", index_bits=bits)
            o, _ = oracle_files(contents, fmt=po.LIBFM, index_bits=bits, d=d, **kw)
            assert "error" not in h, h
            assert len(h["field"]) == len(h["index"]) > 0 and diff(h, o) == [], (bits, uri)
    hi = run_api(tmp_path, d, fmt="libfm", iter_=True)
    o, _ = oracle_files(contents, fmt=po.LIBFM, d=d)
    assert diff(hi, o) == []


@pytest.mark.gpu
@pytest.mark.parametrize("mmap", ["0", "1"])
def test_api_large_multibatch_and_rowiter(tmp_path, monkeypatch, mmap):
    """Several 8 MiB chunks and several device batches; RowBlockIter concat + NumCol
    (mmap=1: the text from the registered mappings in 1 MiB segments, each
    unregistered when its last batch is released; the multi-file test keeps
    them for the parser's life)."""
    text, _ = synth.rows(synth.LIBSVM, 60000, 128, seed=4)
    d, _ = _write(tmp_path / "big", [text.tobytes()])
    monkeypatch.setenv("DMLC_AMD_BATCH_BYTES", str(24 << 20))
    monkeypatch.setenv("DMLC_AMD_MMAP", mmap)
    monkeypatch.setenv("DMLC_AMD_MMAP_SEG_MB", "1")
    monkeypatch.setenv("DMLC_AMD_MMAP_KEEP_MB", "0")  # segments unregistered as their last batch is released
    h = run_api(tmp_path, d)
    o, nch = oracle_files([text.tobytes()])
    assert diff(h, o) == []
    # one block per non-empty FillData range, as ParserImpl::Next hands them out
    assert h["blocks"].tolist() == o["blocks"]["rows"].tolist() and len(h["blocks"]) == 2 * nch
    assert int(h["meta"][1]) == len(text)
    hi = run_api(tmp_path, d, iter_=True)
    assert diff(hi, o) == [] and int(hi["meta"][2]) == int(o["index"].max()) + 1


@pytest.mark.gpu
def test_api_errors_and_args(tmp_path):
    d, _ = _write(tmp_path / "neg", [b"1 -3:1\n"])
    assert "sign == true" in run_api(tmp_path, d)["error"]
    d2, _ = _write(tmp_path / "ok", [b"1 3:1\n"])
    assert "Cannot find argument" in run_api(tmp_path, d2 + "?bogus=1")["error"]
    h = run_api(tmp_path, d2 + "?indexing_mode=1")
    assert h["index"].tolist() == [2]
    d3, _ = _write(tmp_path / "lab", [b"1,2,3\n4,5,6\n"])
    h = run_api(tmp_path, d3 + "?format=csv&label_column=0", fmt="auto")
    o, _ = oracle_files([b"1,2,3\n4,5,6\n"], fmt=po.CSV, label_column=0)
    assert diff(h, o) == []


@pytest.mark.gpu
def test_api_blocks_nthread_indexing_auto(tmp_path):
    """FillData ranges through Parser::Create: nthread 1..3 (DMLC_AMD_NTHREAD),
    indexing_mode=-1 decided per range, one block per non-empty range with
    offset[0] == 0 -- equal to the oracle's blocks."""
    lines = [b"1 0:1 2:3\n", b"0 5:1\n", b"1 1:2 7:1\n", b"0 3:4\n"] * 300
    d, _ = _write(tmp_path / "idx", [b"".join(lines)])
    for nt in (1, 2, 3):
        for uri, kw in ((d, {}), (d + "?indexing_mode=-1", {"indexing_mode": -1})):
            h = run_api(tmp_path, uri, nthread=nt)
            o, _ = oracle_files([b"".join(lines)], nthread=nt, **kw)
            assert "error" not in h and diff(h, o) == [], (nt, uri)
            assert h["blocks"].tolist() == o["blocks"]["rows"].tolist(), (nt, uri)


@pytest.mark.gpu
def test_api_checks_registry_and_multi_worker(tmp_path):
    """RowBlock / Row CHECKs and MemCostBytes with the reference's semantics,
    a parser type registered by the calling program (DMLC_REGISTER_DATA_PARSER)
    found by Parser::Create, and the pipeline with 1..4 workers per device
    and small batches (parse-ahead, in-order delivery)."""
    text, _ = synth.rows(synth.LIBSVM, 3000, 40, seed=6)
    d, paths = _write(tmp_path / "api", [text.tobytes()])
    r = subprocess.run([_driver(), "--api", paths[0]], capture_output=True)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    big, _ = synth.rows(synth.LIBSVM, 30000, 64, seed=8)
    d2, _ = _write(tmp_path / "mw", [big.tobytes()])
    o, _ = oracle_files([big.tobytes()])
    for workers in ("1", "3"):
        h = run_api(tmp_path, d2, env={"DMLC_AMD_WORKERS": workers, "DMLC_AMD_BATCH_BYTES": str(1 << 20)})
        assert "error" not in h and diff(h, o) == [], workers
        assert h["blocks"].tolist() == o["blocks"]["rows"].tolist()


@pytest.mark.gpu
def test_api_errors_raise_at_the_failing_block(tmp_path):
    """A parse error in a later chunk surfaces after the blocks before it, as
    the reference's ThreadedParser rethrows it at that chunk's Next()."""
    good, _ = synth.rows(synth.LIBSVM, 20000, 32, seed=2)
    d, _ = _write(tmp_path / "late", [good.tobytes() + b"1 -3:1\n"])
    h = run_api(tmp_path, d, env={"DMLC_AMD_BATCH_BYTES": str(64 << 20)})
    assert "sign == true" in h["error"]
    # invalid batch-size settings fall back to the default instead of looping
    d2, _ = _write(tmp_path / "ok2", [b"1 3:1\n"])
    for bad in ("0", "abc"):
        h = run_api(tmp_path, d2, env={"DMLC_AMD_BATCH_BYTES": bad})
        assert h["index"].tolist() == [3], bad


@pytest.mark.gpu
def test_api_multi_device_dispatch(tmp_path):
    """DMLC_AMD_DEVICES: the batches of one parser dispatched over a device
    list ("all", or a list naming devices, here the box's device several
    times: every slot gets its own workers and streams) come back in input
    order -- Parser blocks and RowBlockIter (NumCol) equal to the oracle's
    whole parse; a device that does not exist raises."""
    text, _ = synth.rows(synth.LIBSVM, 40000, 64, seed=14)
    d, _ = _write(tmp_path / "md", [text.tobytes()])
    o, _ = oracle_files([text.tobytes()])
    for devs in ("all", "0", "0,0,0"):
        env = {"DMLC_AMD_DEVICES": devs, "DMLC_AMD_BATCH_BYTES": str(1 << 20)}
        h = run_api(tmp_path, d, env=env)
        assert "error" not in h and diff(h, o) == [], devs
        assert h["blocks"].tolist() == o["blocks"]["rows"].tolist(), devs
        hi = run_api(tmp_path, d, iter_=True, env=env)
        assert diff(hi, o) == [] and int(hi["meta"][2]) == int(o["index"].max()) + 1, devs
    bad = run_api(tmp_path, d, env={"DMLC_AMD_DEVICES": "99"})
    assert "no HIP device" in bad["error"]


@pytest.mark.gpu
@pytest.mark.parametrize("mode,precopy", [("d2h_kernel", 1), ("d2h_kernel", 0), ("kernel", 1), ("h2d_kernel", 1),
                                          ("dma", 1)])
def test_api_copy_modes(tmp_path, mode, precopy):
    """DMLC_AMD_COPY: the text in and the batch's CSR arrays out by copy
    kernels (kernel), by DMA (dma), or one direction each (d2h_kernel, the
    default: the copy-out by one kernel queued behind the parse with sizes
    read on the device; h2d_kernel); DMLC_AMD_PRECOPY=0 waits for the parse's
    counts before copying out.  Every mode's blocks equal the oracle's parse,
    over many batches, with weights and qids, a CSV / libfm file, and a file
    whose later batches hold far more entries per byte than the first (the
    queued copy-out's size estimate is exceeded and the batch copies again,
    hip_engine.h `again`)."""
    text, _ = synth.rows(synth.LIBSVM, 30000, 48, seed=21)
    lines = text.tobytes().split(b"\n")
    for i in range(0, len(lines) - 1):  # label:weight and qid on every row (a RowBlock reader takes `size`)
        head, _, rest = lines[i].partition(b" ")
        lines[i] = head + b":0.%d qid:%d " % (1 + i % 9, i // 3) + rest
    svm = b"\n".join(lines)
    env = {"DMLC_AMD_COPY": mode, "DMLC_AMD_BATCH_BYTES": str(1 << 20), "DMLC_AMD_PRECOPY": str(precopy)}
    d, _ = _write(tmp_path / "svm", [svm])
    o, _ = oracle_files([svm])
    h = run_api(tmp_path, d, env=env)
    assert "error" not in h and diff(h, o) == [], mode
    assert h["blocks"].tolist() == o["blocks"]["rows"].tolist(), mode
    for fmt, pfmt in ((synth.CSV, po.CSV), (synth.LIBFM, po.LIBFM)):
        t, _ = synth.rows(fmt, 20000, 24, seed=22)
        name = {po.CSV: "csv", po.LIBFM: "libfm"}[pfmt]
        dd, _ = _write(tmp_path / name, [t.tobytes()])
        oo, _ = oracle_files([t.tobytes()], fmt=pfmt)
        hh = run_api(tmp_path, dd, fmt=name, env=env)
        assert "error" not in hh and diff(hh, oo) == [], (mode, name)
    # long-valued rows first (~20 bytes per entry), then dense short ones (~4)
    rng = np.random.default_rng(23)
    grow = b"".join(b"1 " + b" ".join(b"%d:%.12f" % (j, rng.random()) for j in range(40)) + b"\n"
                    for _ in range(4000))
    grow += b"".join(b"0 " + b" ".join(b"%d:1" % j for j in range(1, 60)) + b"\n" for _ in range(12000))
    dg, _ = _write(tmp_path / "grow", [grow])
    og, _ = oracle_files([grow])
    hg = run_api(tmp_path, dg, env=env)
    assert "error" not in hg and diff(hg, og) == [], (mode, "grow")
    assert hg["blocks"].tolist() == og["blocks"]["rows"].tolist(), mode


@pytest.mark.gpu
def test_api_disk_row_cache_partial_weights_and_qids(tmp_path):
    """uri#cachefile over libsvm blocks where only some rows carry label:weight
    or qid: (fewer weights / qids than rows in a block): the cache pages hold
    each block's own weights and qids followed by zeros up to its row count
    -- RowBlockContainer::Push appends `size` of them per block
    (row_block.h:131-135), so later blocks stay row-aligned; the reference
    reads past the block's values there -- and iterate back equal to the
    oracle's parse."""
    lines = []
    for i in range(30000):
        lab = b"%d:0.%d" % (i % 2, 1 + i % 9) if i % 3 == 0 else b"%d" % (i % 2)
        q = b" qid:%d" % (i // 7) if i % 5 == 0 else b""
        lines.append(lab + q + b" %d:1.5 %d:2.25\n" % (i % 11, 20 + i % 13))
    contents = [b"".join(lines)]
    d, _ = _write(tmp_path / "pw", contents)
    cache = str(tmp_path / "pw.cache")
    h = run_api(tmp_path, d + "#" + cache, iter_=True)
    o, _ = oracle_files(contents)
    assert "error" not in h, h
    assert len(o["weight"]) == 10000 and len(o["qid"]) == 6000
    # the page file itself (RowBlockContainer::Save, row_block.h:190-216): each
    # vector as a u64 count + its elements, then max_field / max_index
    pages = _cache_pages(cache)
    assert len(pages) == 1
    pg = pages[0]
    blk = o["blocks"]
    assert len(blk["rows"]) > 1  # several blocks: the padding is per block
    assert pg["weight"].tobytes() == _pad_per_block(o["weight"], blk["weight"], blk["rows"], np.float32).tobytes()
    assert pg["qid"].tolist() == _pad_per_block(o["qid"], blk["qid"], blk["rows"], np.uint64).tolist()
    assert pg["offset"].tolist() == np.asarray(o["offset"]).tolist()
    assert pg["index"].tolist() == np.asarray(o["index"]).tolist()
    # iterated back: a RowBlock carries no weight / qid count, so a reader
    # takes `size` of them (as from the reference's own pages); the rest equal
    keep = {k: v for k, v in o.items() if k not in ("weight", "qid")}
    assert diff(h, keep) == []
    assert h["weight"].tobytes() == pg["weight"].tobytes() and h["qid"].tolist() == pg["qid"].tolist()
    again = run_api(tmp_path, d + "#" + cache, iter_=True)  # the cache reused
    assert diff(again, keep) == [] and _cache_pages(cache)[0]["weight"].size == 30000


def _pad_per_block(vals, own, rows, dtype):
    """Each block's own values, then zeros up to its row count (blocks with
    none contribute nothing: RowBlock.weight / qid is NULL there)."""
    out, pos = [], 0
    for k, r in zip(own.tolist(), rows.tolist()):
        if k:
            out.append(np.asarray(vals[pos:pos + k], dtype))
            out.append(np.zeros(r - k, dtype))
        pos += k
    return np.concatenate(out) if out else np.zeros(0, dtype)


def _cache_pages(path, index_dtype=np.uint32, value_dtype=np.float32):
    """Pages of a uri#cachefile (RowBlockContainer<uint32_t, real_t>::Save)."""
    raw = open(path, "rb").read()
    pos, pages = 0, []
    spec = (("offset", np.uint64), ("label", value_dtype), ("weight", np.float32), ("qid", np.uint64),
            ("field", index_dtype), ("index", index_dtype), ("value", value_dtype))
    while pos < len(raw):
        pg = {}
        for name, dt in spec:
            n = int(np.frombuffer(raw, np.uint64, 1, pos)[0])
            pos += 8
            pg[name] = np.frombuffer(raw, dt, n, pos)
            pos += n * np.dtype(dt).itemsize
        pos += 2 * np.dtype(index_dtype).itemsize  # max_field, max_index
        pages.append(pg)
    return pages
