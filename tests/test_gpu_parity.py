"""GPU parity: the HIP parse path against the reference goldens and the oracle.

All tests run through the C-ABI (libdmlc_amd.so via dmlc_amd.py).  Integer and
index arrays must be bit-identical; float values bit-identical as well (the
north star allows 1 ulp, the design targets 0 and the tests demand 0).
"""
import hashlib

import numpy as np
import pytest

from golden_util import FIELDS, blocks_of, dec, diff, load_cases, load_floats, load_json, same
from oracle import pyoracle as po
from tools import synth

pytestmark = pytest.mark.gpu

FMT_NAME = {po.LIBSVM: "libsvm", po.CSV: "csv", po.LIBFM: "libfm"}


@pytest.fixture(scope="module")
def dm():
    import dmlc_amd
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    dmlc_amd.lib()
    return dmlc_amd


def gpu_kwargs(params):
    kw = {}
    for k, v in params.items():
        if k == "fmt":
            continue
        if k == "value_kind":
            kw["value_type"] = int(v)
        else:
            kw[k] = v
    return kw


def gpu_parse(dm, data, chunk_offsets=None, fmt=po.LIBSVM, **kw):
    name = FMT_NAME[fmt]
    h = dm.parse_bytes(data, chunk_offsets, fmt=name, **kw)
    nch = (len(chunk_offsets) - 1) if chunk_offsets is not None else (1 if len(data) else 0)
    nch *= h["units_per_chunk"]
    failed = nch > 0 and dm.chunk_check(h, name, nch, h["counts"]) >= 0
    h["failed"] = bool(h["error"]) or failed
    return h


CASES = load_cases()


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_gpu_matches_reference_goldens(dm, case):
    prm = case["params"]
    h = gpu_parse(dm, case["data_latin1"], None, prm["fmt"], **gpu_kwargs(prm))
    if case["status"]:
        assert h["failed"], "reference raised (%s) but GPU did not" % case["msg"]
        return
    assert not h["failed"], (h["error"], h["counts"])
    exp = {k: dec(v) for k, v in case["expect"].items()}
    bad = diff(h, exp)
    assert bad == [], {k: (h[k][:20], exp[k][:20]) for k in bad}


def test_gpu_strtof_goldens(dm):
    strs, bits, used = load_floats()
    v, n, bad = dm.strtof_batch(strs)
    got = v.view(np.uint32)
    mism = np.nonzero((got != bits) | (n != used))[0]
    assert len(mism) == 0, [(strs[i], hex(bits[i]), hex(got[i]), used[i], n[i]) for i in mism[:10]]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("name", ["libsvm_10k_x128", "csv_10k_x256"])
def test_gpu_synthetic_config1(dm, name):
    g = load_json("synth_cfg1.json")[name]
    fmt = po.LIBSVM if g["format"] == "libsvm" else po.CSV
    text, _ = synth.rows(synth.LIBSVM if fmt == po.LIBSVM else synth.CSV, g["rows"], g["width"],
                         seed=g["seed"])
    assert sha(text) == g["input_sha256"]
    # chunked exactly as the reference's InputSplit would (oracle restatement)
    chunks = po.split_text([text.tobytes()])
    offs = np.cumsum([0] + [len(c) for c in chunks])
    h = gpu_parse(dm, b"".join(chunks), offs, fmt)
    assert not h["failed"]
    for k, hv in g["sha256"].items():
        assert sha(h[k]) == hv, k


def _oracle_vs_gpu(dm, data, offs, fmt, **kw):
    okw = {("value_kind" if k == "value_type" else k): v for k, v in kw.items() if k not in ("tile_bytes", "exact")}
    o = po.parse_chunks(data, offs, fmt=fmt, **okw)
    h = gpu_parse(dm, data, offs, fmt, **kw)
    assert (o["status"] != 0) == h["failed"], (o["msg"], h["error"])
    if o["status"] == 0:
        bad = diff(h, o)
        assert bad == [], bad
    return h


def _random_chunks(rng, data, nmax=8):
    """Split at random line boundaries like an InputSplit would (after a '\\n' or '\\r')."""
    nl = [i + 1 for i, b in enumerate(data) if b in (10, 13) and i + 1 < len(data)]
    k = int(rng.integers(0, min(nmax, len(nl)) + 1)) if nl else 0
    cuts = sorted(set(rng.choice(nl, size=k, replace=False).tolist())) if k else []
    return [0] + cuts + [len(data)]


@pytest.mark.parametrize("fmt", [po.LIBSVM, po.CSV])
def test_gpu_multichunk_synthetic_vs_oracle(dm, fmt):
    rng = np.random.default_rng(7)
    text, _ = synth.rows(synth.LIBSVM if fmt == po.LIBSVM else synth.CSV, 3000, 37, seed=3)
    data = text.tobytes()
    for _ in range(4):
        _oracle_vs_gpu(dm, data, _random_chunks(rng, data, 12), fmt)


@pytest.mark.parametrize("tile", [64, 1000, 4096, 20000])
def test_gpu_tile_sizes_vs_oracle(dm, tile):
    """Small tiles put many tile/window boundaries inside lines and heads."""
    text, _ = synth.rows(synth.LIBSVM, 2000, 50, seed=11)
    data = text.tobytes()
    offs = [0, len(data) // 3 + data[len(data) // 3:].index(b"\n") + 1, len(data)]
    _oracle_vs_gpu(dm, data, offs, po.LIBSVM, tile_bytes=tile)
    ctext, _ = synth.rows(synth.CSV, 800, 40, seed=12)
    _oracle_vs_gpu(dm, ctext.tobytes(), [0, len(ctext)], po.CSV, tile_bytes=tile)


def test_gpu_long_lines_vs_oracle(dm):
    """Lines far longer than a window (8 KiB) and than a tile."""
    rng = np.random.default_rng(5)
    lines = []
    for r in range(12):
        k = int(rng.integers(1, 6000))
        feats = " ".join("%d:%.9g" % (i * 3, rng.random()) for i in range(k))
        head = "%d" % (r % 2) + (":0.5" if r % 3 == 0 else "") + (" qid:%d" % r if r % 4 == 0 else "")
        lines.append(head + " " + feats + (" # tail" if r % 5 == 0 else ""))
    data = ("\n".join(lines) + "\n").encode()
    for tile in (0, 4096, 100000):
        _oracle_vs_gpu(dm, data, [0, len(data)], po.LIBSVM, tile_bytes=tile)
    csvl = "\n".join(",".join("%.6g" % x for x in rng.random(int(rng.integers(1, 5000))))
                     for _ in range(8)) + "\n"
    _oracle_vs_gpu(dm, csvl.encode(), [0, len(csvl)], po.CSV, tile_bytes=4096)


@pytest.mark.parametrize("form", ["valued", "mid_pair", "dangling", "long_head", "index_only"])
def test_gpu_exact_rows_past_the_records(dm, form):
    """Rows over 32 KiB crossing exact tile ends at tile_bytes=4096: the write
    pass runs past the count pass's three recorded windows per tile and
    restores the role state and pending token from rec_meta
    (libsvm_core.h:406); rows ending mid-pair / with "idx:" / long heads."""
    rng = np.random.default_rng(500 + ["valued", "mid_pair", "dangling", "long_head", "index_only"].index(form))
    for it in range(6):
        data = fuzz_text.long_row_libsvm(rng, form)
        h = _oracle_vs_gpu(dm, data, fuzz_text.random_cuts(rng, data, 2), po.LIBSVM, exact=True, tile_bytes=4096)
        assert h["path"] == "exact"


def test_gpu_csv_exact_wide_rows_past_the_records(dm):
    """The CSV write pass recounts windows past its records (csv_core.h:451)."""
    rng = np.random.default_rng(577)
    for it in range(8):
        data = fuzz_text.wide_row_csv(rng)
        h = _oracle_vs_gpu(dm, data, fuzz_text.random_cuts(rng, data, 2), po.CSV, exact=True, tile_bytes=4096)
        assert h["path"] == "exact"


def _fuzz_text(rng, fmt):
    alpha = {po.LIBSVM: list("0123456789") * 6 + list("  ::.-+eE#\tq") + ["qid:", "nan", "inf", "\r"],
             po.CSV: list("0123456789") * 6 + list(",,,,.-+eE \t") + ["nan", "inf", "0x", "\xef\xbb\xbf"],
             po.LIBFM: list("0123456789") * 6 + list("  :::.-+eE#\t") + ["\r", "nan", "x"]}[fmt]
    lines = []
    for _ in range(int(rng.integers(1, 12))):
        n = int(rng.integers(0, 60))
        lines.append("".join(alpha[int(i)] for i in rng.integers(0, len(alpha), n)))
    t = "\n".join(lines)
    if rng.random() < 0.5:
        t += "\n"
    return t.encode("latin-1")


@pytest.mark.parametrize("fmt", [po.LIBSVM, po.CSV, po.LIBFM])
def test_gpu_fuzz_vs_oracle(dm, fmt):
    rng = np.random.default_rng(4242 + fmt)
    for it in range(300):
        data = _fuzz_text(rng, fmt)
        offs = _random_chunks(rng, data, 4) if data else [0]
        kw = {}
        if fmt == po.CSV:
            if rng.random() < 0.3:
                kw["label_column"] = int(rng.integers(0, 3))
            if rng.random() < 0.2:
                kw["value_type"] = int(rng.integers(1, 3))
            if rng.random() < 0.2:
                kw["delimiter"] = " "
        else:
            if rng.random() < 0.3:
                kw["indexing_mode"] = int(rng.integers(-1, 2))
            if rng.random() < 0.2:
                kw["index_bits"] = 64
        if rng.random() < 0.3:
            kw["tile_bytes"] = int(rng.integers(16, 200))
        try:
            _oracle_vs_gpu(dm, data, offs, fmt, **kw)
        except AssertionError as e:
            raise AssertionError("case %d kw=%s data=%r offs=%s: %s" % (it, kw, data, offs, e))


def test_gpu_empty_and_tiny(dm):
    for fmt in (po.LIBSVM, po.CSV, po.LIBFM):
        for d in (b"", b"\n", b"\r\n\r\n", b"1", b"1\n", b"   \n"):
            offs = [0, len(d)] if d else [0]
            _oracle_vs_gpu(dm, d, offs, fmt)


# ------------------------------------------------- single-pass fast path --
import fuzz_text  # noqa: E402


def _gpu_vs_oracle_paths(dm, data, offs, fmt=po.LIBSVM, **kw):
    """Default path and forced exact path both equal the oracle."""
    o = po.parse_chunks(data, offs, fmt=fmt, **kw)
    res = {}
    name = FMT_NAME[fmt]
    for exact in (False, True):
        h = dm.parse_bytes(data, offs, fmt=name, exact=exact, **kw)
        nch = len(offs) - 1
        failed = bool(h["error"]) or (nch > 0 and dm.chunk_check(h, name, nch, h["counts"]) >= 0)
        assert (o["status"] != 0) == failed, (exact, o["msg"], h["error"], data[:200], offs, kw)
        if not failed:
            bad = diff(h, o)
            assert bad == [], (exact, bad, offs, kw)
        res[exact] = h
    if o["status"] == 0:
        assert res[False]["chunk_table"].tolist() == res[True]["chunk_table"].tolist()
    return res[False]


def test_gpu_fast_fuzz_vs_oracle(dm):
    rng = np.random.default_rng(31337)
    paths = {"fast": 0, "exact": 0}
    for it in range(400):
        data = fuzz_text.uniform_libsvm(rng, int(rng.integers(1, 40)), int(rng.integers(0, 40)),
                                        violate=rng.random() < 0.25)
        offs = fuzz_text.random_cuts(rng, data, 6, anywhere=rng.random() < 0.3)
        kw = {}
        if rng.random() < 0.2:
            kw["index_bits"] = 64
        if rng.random() < 0.2:
            kw["indexing_mode"] = int(rng.integers(0, 2))
        try:
            paths[_gpu_vs_oracle_paths(dm, data, offs, **kw)["path"]] += 1
        except AssertionError as e:
            raise AssertionError("case %d: %s" % (it, e))
    assert paths["fast"] > 200, paths


def test_gpu_fast_multi_tile_vs_oracle(dm):
    rng = np.random.default_rng(4711)
    for it in range(24):
        data = fuzz_text.uniform_libsvm(rng, int(rng.integers(200, 3000)), int(rng.integers(1, 120)),
                                        violate=it % 6 == 5)
        offs = fuzz_text.random_cuts(rng, data, int(rng.integers(0, 40)), anywhere=it % 3 == 1)
        h = _gpu_vs_oracle_paths(dm, data, offs)
        if it % 6 != 5 and it % 3 != 1:
            assert h["path"] == "fast", it


def test_gpu_fast_dense_runs_vs_oracle(dm):
    """Thousands of one-byte runs per 16 KiB tile: the libsvm write pass
    decodes its run lists in several passes (svm_fast.h kPassRuns)."""
    rng = np.random.default_rng(1212)
    for it, style in enumerate(("pairs", "weights", "labels", "mixed", "pairs", "mixed")):
        data = fuzz_text.dense_libsvm(rng, int(rng.integers(3, 40)) * 16384 + int(rng.integers(0, 999)), style)
        offs = fuzz_text.random_cuts(rng, data, int(rng.integers(0, 12)), anywhere=False)
        kw = {"index_bits": 64} if it % 2 else {}
        h = _gpu_vs_oracle_paths(dm, data, offs, **kw)
        assert h["path"] == "fast", (it, style)


def test_gpu_libfm_dense_runs_vs_oracle(dm):
    """libfm tiles of one-byte runs: the index, field and value lists in passes."""
    rng = np.random.default_rng(1313)
    for it in range(4):
        data = fuzz_text.dense_libfm(rng, int(rng.integers(3, 30)) * 16384 + int(rng.integers(0, 999)))
        offs = fuzz_text.random_cuts(rng, data, int(rng.integers(0, 8)), anywhere=False)
        h = _gpu_vs_oracle_paths(dm, data, offs, fmt=po.LIBFM, **({"index_bits": 64} if it % 2 else {}))
        assert h["path"] == "fast", it


def test_gpu_csv_dense_tokens_vs_oracle(dm):
    """CSV tiles of one-digit fields: the token lists in passes (csv_fast.h
    kPassTokens), rows carried across tiles, a row past 2^17 columns."""
    rng = np.random.default_rng(1414)
    for it in range(5):
        delim = ",;"[it % 2]
        wide = it == 4
        data = fuzz_text.dense_csv(rng, 300000 if wide else int(rng.integers(3, 40)) * 16384 + 77, delim, wide=wide)
        offs = fuzz_text.random_cuts(rng, data, int(rng.integers(0, 8)), anywhere=False)
        h = _gpu_vs_oracle_paths(dm, data, offs, fmt=po.CSV, delimiter=delim)
        assert h["path"] == "fast", it


def test_gpu_fast_qid_vs_oracle(dm):
    """"qid:" rows through the single-pass kernel (svm_fast.h qid_clean /
    qid_ok, qid_fix_kernel): fast and exact paths both equal the oracle;
    the reference's odd readings and rows without a qid take the exact path."""
    rng = np.random.default_rng(8128)
    paths = {"fast": 0, "exact": 0}
    for it in range(120):
        big = it % 10 == 0
        data = fuzz_text.qid_libsvm(rng, 3000 if big else int(rng.integers(1, 40)), 60 if big else 16,
                                    violate=it % 4 == 3, mixed=it % 10 == 9)
        offs = fuzz_text.random_cuts(rng, data, int(rng.integers(0, 8)), anywhere=it % 5 == 4)
        kw = {"index_bits": 64} if it % 3 == 1 else {}
        h = _gpu_vs_oracle_paths(dm, data, offs, **kw)
        paths[h["path"]] += 1
        if it % 4 != 3 and it % 10 != 9 and it % 5 != 4:
            assert h["path"] == "fast", it
    assert paths["fast"] >= 60 and paths["exact"] >= 20, paths


def test_gpu_fast_comments_vs_oracle(dm):
    """'#' comments through the single-pass kernel (svm_fast.h comment_erase):
    headers, trailing comments with any text, comments longer than the
    pre-halo, qid rows; '#' lines after the first and the forms the reference
    reads otherwise take the exact path -- both equal the oracle."""
    rng = np.random.default_rng(6161)
    paths = {"fast": 0, "exact": 0}
    for it in range(120):
        big = it % 10 == 0
        data = fuzz_text.comment_libsvm(rng, 3000 if big else int(rng.integers(1, 40)), 60 if big else 16,
                                        long_frac=0.0 if it % 2 == 0 else 0.2, violate=it % 4 == 3,
                                        qid=it % 5 == 2, line_comments=it % 8 == 5)
        offs = fuzz_text.random_cuts(rng, data, int(rng.integers(0, 8)), anywhere=it % 3 == 1)
        kw = {"index_bits": 64} if it % 7 == 1 else {}
        h = _gpu_vs_oracle_paths(dm, data, offs, **kw)
        paths[h["path"]] += 1
        if it % 2 == 0 and it % 4 != 3 and it % 3 != 1 and not big:
            assert h["path"] == "fast", it
    assert paths["fast"] >= 30 and paths["exact"] >= 10, paths


@pytest.mark.parametrize("body", ["x", " 1 2:3 4", "q:i#d"])
def test_gpu_comments_across_tile_ends(dm, body):
    """A comment d bytes before a 16 KiB tile end, L bytes long: the next tile
    blanks it from its pre-halo when the '#' and the pair before it lie there,
    else the gate hands over."""
    rng = np.random.default_rng(17)
    base = fuzz_text.uniform_libsvm(rng, 400, 20).replace(b"\r", b"\n")
    for d in (1, 2, 40, 63, 64, 65, 300):
        for L in (0, 3, 80, 600, 20000):
            cut = base.index(b"\n", 16384 - d - 200) + 1
            pre = base[:cut] + b"7" + b" " * max(0, 16384 - d - cut - 6) + b" 1:2 "  # '#' right after a pair
            com = (b"#" + (body.encode() * (L // len(body) + 1))[:L]).replace(b"\n", b" ")
            data = pre + com + b"\n" + base[cut:]
            for offs in ([0, len(data)], [0, cut, len(data)]):
                h = _gpu_vs_oracle_paths(dm, data, offs)
                if d <= 60 and L <= 600 and len(offs) == 2:  # the pair before the '#' in the pre-halo
                    assert h["path"] == "fast", (d, L)


def test_gpu_dirty_lines_vs_oracle(dm):
    """Per-line fallback (svm_fast.h dirty_lines): lines holding bytes outside
    the grammar -- file headers mid-chunk, words, symbols, inf / nan values --
    at several rates, across and near tile ends, with odd chunkings, 64-bit
    ids and indexing_mode -1, and long dirty lines (the exact kernels' case):
    the default path and the forced exact path both equal the oracle, and
    inputs whose dirty lines are all short stay on the single pass."""
    rng = np.random.default_rng(4242)
    paths = {"fast": 0, "exact": 0}
    for it in range(60):
        data = fuzz_text.dirty_libsvm(rng, 120000 if it % 3 else 5000, rate=(0.002, 0.01, 0.05)[it % 3],
                                      long_frac=0.3 if it % 5 == 4 else 0.0, near_tile_end=it % 3 == 1,
                                      eol=(b"\n", b"\r\n", b"\n", b"\r")[it % 4])
        offs = fuzz_text.random_cuts(rng, data, 6, anywhere=it % 4 == 3)
        kw = {"index_bits": 64} if it % 7 == 1 else ({"indexing_mode": -1} if it % 7 == 2 else {})
        h = _gpu_vs_oracle_paths(dm, data, offs, **kw)
        paths[h["path"]] += 1
    assert paths["fast"] >= 15 and paths["exact"] >= 5, paths


def test_gpu_dirty_rows_stay_single_pass(dm):
    """Rows carrying words, symbols, bytes >= 0x80, a ':' behind a non-blank
    byte, inf / nan values and labels (fuzz_text.dirty_rows_libsvm) at 1/8,
    1/2 and every row, rows of up to 2 KB across tile ends, CRLF / lone-CR
    line ends, odd chunkings, 64-bit ids and indexing_mode -1 / 1: the single
    pass keeps every input (svm_fast.h dirty_rewrite) and both paths equal the
    oracle (a third of the inputs also hold words with digitchar runs, whose
    index-only ids fail the reference's RowBlock CHECK: the failure is
    compared)."""
    rng = np.random.default_rng(6062)
    for it in range(48):
        width = int(rng.integers(4, 130))
        data = fuzz_text.dirty_rows_libsvm(rng, max(4, 120000 // (width * 16 + 4)), width,
                                           rate=(0.125, 0.5, 1.0)[it % 3], eol=(b"\n", b"\r\n", b"\r", b"\n")[it % 4],
                                           near_tile_end=it % 2 == 1, runs=it % 3 == 2)
        offs = fuzz_text.random_cuts(rng, data, 6, anywhere=False)
        kw = {"index_bits": 64} if it % 4 == 1 else ({"indexing_mode": -1} if it % 4 == 2 else
                                                      ({"indexing_mode": 1} if it % 4 == 3 else {}))
        h = _gpu_vs_oracle_paths(dm, data, offs, **kw)
        assert h["path"] == "fast", (it, kw)


def test_gpu_file_headers_stay_on_single_pass(dm):
    """Files with a "# ..." first line read as a directory by the text
    InputSplit ('\\n' between files, input_split_base.cc:204-210): every
    header after the first sits mid-chunk, a line the reference reads (an
    empty one: no digitchar); headers placed across 16 KiB tile ends at every
    offset of the last 80 bytes stay on the single pass."""
    rng = np.random.default_rng(808)
    for it in range(24):
        files = []
        for f in range(5):
            body = fuzz_text.uniform_libsvm(rng, int(rng.integers(100, 500)), 20).replace(b"\r", b"\n")
            files.append(b"# synth libsvm shard\n" + body.rstrip(b"\n") + b"\n")
        data = b"\n".join(files) + b"\n"
        k = data.find(b"# synth", 16384 - 3000)
        if 0 < k < 16384:  # this header from 70 bytes before the tile end to 10 after
            pad = 16384 - 70 + 3 * it - k
            if pad > 0:
                data = data[:k - 1] + b" " * pad + data[k - 1:]
        offs = fuzz_text.random_cuts(rng, data, 4, anywhere=False)
        h = _gpu_vs_oracle_paths(dm, data, offs, nthread=1 + it % 2)
        assert h["path"] == "fast", it


def test_gpu_comment_bench_size_fast_equals_exact(dm):
    """Config 2 rows, each with a trailing '# row <r>' comment, and a header
    line: single-pass == exact bit for bit (the comment path in every tile)."""
    import torch
    text, _ = synth.rows(synth.LIBSVM, 1 << 18, 128, seed=3)
    body = bytes(text).replace(b"\n", b" # c:1 qid:2 #x\n")
    data = b"# header: label idx:val ...\n" + body
    arr = np.frombuffer(data, dtype=np.uint8)
    starts = dm.text_chunk_starts(arr)
    d_text, d_cs = torch.from_numpy(arr.copy()).cuda(), torch.from_numpy(starts).cuda()
    outs = {}
    for exact in (False, True):
        p = dm.DeviceParser("libsvm", flags=dm.FLAG_EXACT if exact else 0)
        out = p.parse(d_text, d_cs)
        assert out["error"] == 0 and out["path"] == (1 if exact else 0), (exact, out["path"])
        outs[exact] = out
    assert outs[False]["counts"][:7] == outs[True]["counts"][:7]
    for k in ("offset", "label", "index", "value"):
        a, b = outs[False][k], outs[True][k]
        assert torch.equal(a.view(torch.int32) if a.dtype == torch.float32 else a,
                           b.view(torch.int32) if b.dtype == torch.float32 else b), k


def test_gpu_csv_fast_weight_column_vs_oracle(dm):
    """weight_column on the single-pass CSV kernel (csv_fast_tile_sp), alone
    and with a label column; the forms it leaves to the exact kernels (weight
    column 0, {label, weight} = {0, 1}, empty weights, short rows) -- both
    paths equal the oracle."""
    rng = np.random.default_rng(9191)
    paths = {"fast": 0, "exact": 0}
    combos = [(-1, 1), (-1, 3), (0, 2), (3, 1), (1, 4), (2, 0), (0, 1), (-1, 0)]
    for it in range(96):
        lc, wc = combos[it % len(combos)]
        nl = 3000 if it % 16 == 7 else int(rng.integers(1, 60))
        data = fuzz_text.labeled_csv(rng, nl, int(rng.integers(max(lc, wc) + 2, max(lc, wc) + 40)), lc,
                                     defects=0.0 if it % 16 < 8 else 0.1, weight_col=wc)
        offs = fuzz_text.random_cuts(rng, data, int(rng.integers(0, 6)))
        h = _gpu_vs_oracle_paths(dm, data, offs, fmt=po.CSV, label_column=lc, weight_column=wc,
                                 **({"index_bits": 64} if it % 5 == 1 else {}))
        paths[h["path"]] += 1
        if it % 16 < 8 and it % 8 < 5:
            assert h["path"] == "fast", (it, lc, wc)
    assert paths["fast"] >= 30 and paths["exact"] >= 20, paths


def test_gpu_qid_bench_size_fast_equals_exact(dm):
    """The qid bench config (1M rows x 128 nnz, qid:<row/16> on every row):
    single-pass == exact bit for bit, qid[r] = r / 16."""
    import torch
    text, _ = synth.rows(synth.LIBSVM_QID, 1 << 20, 128, seed=1)
    starts = dm.text_chunk_starts(text)
    d_text, d_cs = torch.from_numpy(text).cuda(), torch.from_numpy(starts).cuda()
    outs = {}
    for exact in (False, True):
        p = dm.DeviceParser("libsvm", flags=dm.FLAG_EXACT if exact else 0)
        out = p.parse(d_text, d_cs)
        assert out["error"] == 0 and out["path"] == (1 if exact else 0)
        outs[exact] = out
    c = outs[False]["counts"]
    assert c[:7] == outs[True]["counts"][:7] and c[dm.QID] == 1 << 20
    for k in ("offset", "label", "qid", "index", "value"):
        a, b = outs[False][k], outs[True][k]
        assert torch.equal(a.view(torch.int32) if a.dtype == torch.float32 else a,
                           b.view(torch.int32) if b.dtype == torch.float32 else b), k
    q = outs[False]["qid"][: 1 << 20].to(torch.int64)
    assert bool((q == torch.arange(1 << 20, device=q.device) // 16).all())


def test_gpu_fast_synthetic_vs_oracle(dm):
    """~100 MB of canonical synthetic text (many tiles, 8 MiB InputSplit chunks)."""
    text, _ = synth.rows(synth.LIBSVM, 50000, 128, seed=21)
    offs = dm.text_chunk_starts(text, 8 << 20).tolist()
    o = po.parse_chunks(text.tobytes(), offs, fmt=po.LIBSVM)
    h = dm.parse_bytes(text.tobytes(), offs, fmt="libsvm")
    assert h["path"] == "fast" and h["error"] == 0
    assert diff(h, o) == []


# ------------------------------------------------- single-pass CSV path --


def test_gpu_csv_fast_fuzz_vs_oracle(dm):
    rng = np.random.default_rng(8086)
    paths = {"fast": 0, "exact": 0}
    for it in range(300):
        delim = ",;|"[it % 3]
        data = fuzz_text.uniform_csv(rng, int(rng.integers(1, 40)), int(rng.integers(1, 40)), delim,
                                     violate=rng.random() < 0.2)
        offs = fuzz_text.random_cuts(rng, data, 6, anywhere=rng.random() < 0.3)
        kw = {"delimiter": delim}
        if rng.random() < 0.2:
            kw["index_bits"] = 64
        try:
            paths[_gpu_vs_oracle_paths(dm, data, offs, fmt=po.CSV, **kw)["path"]] += 1
        except AssertionError as e:
            raise AssertionError("case %d: %s" % (it, e))
    assert paths["fast"] > 150, paths


def test_gpu_csv_fast_text_fields_vs_oracle(dm):
    """Text in CSV float columns on the single-pass kernel (csv_fast.h
    csv_junk_byte): header rows, text columns, numbers followed by text,
    "nan" / "inf" / "f" fields (after signs and blanks too), bytes >= 0x80 and
    BOMs at row starts stay on it, and so (round 6) do "NaN(...)" fields --
    closed, or not (the reference's "Invalid NAN literal").  Either path gives
    the reference's result."""
    rng = np.random.default_rng(4711)
    paths = {"fast": 0, "exact": 0}
    for it in range(160):
        delim = ",;| "[it % 4]
        big = it % 16 == 15
        violate = it % 5 == 4
        data = fuzz_text.junk_csv(rng, 1500 if big else int(rng.integers(1, 40)), 40 if big else 16, delim,
                                  header=it % 2 == 0, violate=violate)
        offs = fuzz_text.random_cuts(rng, data, 6, anywhere=rng.random() < 0.3)
        try:
            h = _gpu_vs_oracle_paths(dm, data, offs, fmt=po.CSV, delimiter=delim)
        except AssertionError as e:
            raise AssertionError("case %d: %s" % (it, e))
        paths[h["path"]] += 1
        if delim == ",":
            assert h["path"] == "fast", (it, data[:200])
    assert paths["fast"] > 80, paths


def test_gpu_csv_header_row_bench_shape(dm):
    """Config 3's shape behind a header row of column names: the single-pass
    kernel stays on.  Names ParseFloat reads nothing from ("c7") make an empty
    row; names starting with 'f' ("feature_7") are its suffix, the value 0 in
    every column (strtonum.h ParseFloat) -- the headerless parse with that row
    in front."""
    text, _ = synth.rows(synth.CSV, 60000, 256, seed=5)
    h0 = gpu_parse(dm, text.tobytes(), dm.text_chunk_starts(text).tolist(), po.CSV)
    assert not h0["failed"]
    off0 = np.asarray(h0["offset"]).astype(np.int64)
    for name, row in (("c%d", 0), ("feature_%d", 256)):
        header = (",".join(name % j for j in range(256)) + "\n").encode()
        data = header + text.tobytes()
        h1 = gpu_parse(dm, data, dm.text_chunk_starts(np.frombuffer(data, np.uint8)).tolist(), po.CSV)
        assert h1["path"] == "fast" and not h1["failed"], name
        off1 = np.asarray(h1["offset"]).astype(np.int64)
        assert off1[:2].tolist() == [0, row], name
        assert (off1[1:] - row).tolist() == off0.tolist(), name
        idx1, val1 = np.asarray(h1["index"]), np.asarray(h1["value"])
        assert idx1[:row].tolist() == list(range(row)) and not np.asarray(val1[:row]).any(), name
        assert idx1[row:].tobytes() == np.asarray(h0["index"]).tobytes(), name
        assert val1[row:].tobytes() == np.asarray(h0["value"]).tobytes(), name


def test_gpu_csv_fast_multi_tile_vs_oracle(dm):
    """Rows and fields crossing 16 KiB tiles: the segmented column carry
    through the look-back, long rows spanning several tiles."""
    rng = np.random.default_rng(4242)
    for it in range(16):
        maxcols = [8, 60, 400, 3000][it % 4]
        data = fuzz_text.uniform_csv(rng, int(rng.integers(100, 2000)) if maxcols < 3000 else 40, maxcols)
        offs = fuzz_text.random_cuts(rng, data, int(rng.integers(0, 30)), anywhere=it % 3 == 1)
        h = _gpu_vs_oracle_paths(dm, data, offs, fmt=po.CSV)
        assert h["path"] == "fast", it


def test_gpu_sharded_parts_concat(dm):
    """Each rank's byte range (dmlc_amd_dist.part_range: the reference's
    ResetPartition split) parsed on the GPU and concatenated on the host with
    offset rebasing equals one parse of the whole input (BASELINE config 5's
    sharding, here sequentially on one device)."""
    import dmlc_amd_dist as dd
    for fmt, name in ((po.LIBSVM, "libsvm"), (po.CSV, "csv")):
        text, _ = synth.rows(synth.LIBSVM if fmt == po.LIBSVM else synth.CSV, 40000, 64, seed=5)
        data = text.tobytes()
        whole = dm.parse_bytes(data, dm.text_chunk_starts(text).tolist(), fmt=name)
        for world in (2, 8):
            parts = [dd.parse_part(data, r, world, fmt=name, chunk_bytes=1 << 20) for r in range(world)]
            assert all(p["error"] == 0 and p["path"] == "fast" for p in parts)
            cat = dd.concat_csr(parts)
            for k in ("offset", "index", "value"):
                assert np.asarray(cat[k]).tobytes() == np.asarray(whole[k]).tobytes(), (name, world, k)


def test_gpu_config4_wide_rows_vs_oracle(dm):
    """BASELINE config 4's rows (2048 nnz each, ~35 KiB: every row crosses
    two or three 16 KiB tiles) at an oracle-checkable size: 6000 rows in 8 MiB
    InputSplit chunks, nthread 1 and 2, both index widths."""
    text, _ = synth.rows(synth.LIBSVM, 6000, 2048, seed=4)
    data = text.tobytes()
    offs = dm.text_chunk_starts(text, 8 << 20).tolist()
    assert len(offs) > 20
    for kw in ({}, {"nthread": 2}, {"index_bits": 64}):
        o = po.parse_chunks(data, offs, fmt=po.LIBSVM, **kw)
        h = dm.parse_bytes(data, offs, fmt="libsvm", **kw)
        assert o["status"] == 0 and h["error"] == 0 and h["path"] == "fast", kw
        assert diff(h, o) == [], kw
        assert h["counts"][dm.INDEX] == 6000 * 2048


def test_gpu_max_index_flag(dm):
    """FLAG_MAX_INDEX: result.max_index / max_field are the largest index and
    field written (RowBlockContainer::max_index, BasicRowIter::NumCol - 1),
    on the fast and the exact path, libsvm and libfm."""
    import torch
    for fmt, kind in (("libsvm", synth.LIBSVM), ("libfm", synth.LIBFM)):
        text, _ = synth.rows(kind, 30000, 40, seed=12)
        starts = dm.text_chunk_starts(text, 1 << 20)
        d_text, d_cs = torch.from_numpy(text).cuda(), torch.from_numpy(starts).cuda()
        for flags in (dm.FLAG_MAX_INDEX, dm.FLAG_MAX_INDEX | dm.FLAG_EXACT):
            p = dm.DeviceParser(fmt, flags=flags)
            out = p.parse(d_text, d_cs)
            assert out["error"] == 0
            n = out["counts"][dm.INDEX]
            assert out["max_index"] == int(out["index"][:n].max())
            if fmt == "libfm":
                assert out["max_field"] == int(out["field"][:n].max())


def test_gpu_config5_shards_vs_oracle(dm):
    """BASELINE config 5's sharding (64-nnz rows, 8 parts): each part's byte
    range (dmlc_amd_dist.part_range) is the oracle InputSplit's part k, each
    part's GPU parse equals the oracle's parse of that part's chunks, and the
    Push-style concatenation equals the oracle's parse of the whole file."""
    import dmlc_amd_dist as dd
    text, _ = synth.rows(synth.LIBSVM, 200000, 64, seed=5)
    data = text.tobytes()
    world = 8
    whole = po.parse_chunks(data, dm.text_chunk_starts(text, 8 << 20).tolist(), fmt=po.LIBSVM)
    assert whole["status"] == 0
    parts = []
    for r in range(world):
        chunks = po.split_text([data], r, world, 8 << 20)
        b, e = dd.part_range(data, r, world)
        assert b"".join(chunks) == data[b:e], r
        offs = np.concatenate([[0], np.cumsum([len(c) for c in chunks])]).tolist()
        o = po.parse_chunks(b"".join(chunks), offs, fmt=po.LIBSVM)
        h = dd.parse_part(data, r, world, fmt="libsvm", chunk_bytes=8 << 20)
        assert o["status"] == 0 and h["error"] == 0 and h["path"] == "fast", r
        assert diff(h, o) == [], r
        parts.append(h)
    cat = dd.concat_csr(parts)
    for k in ("offset", "label", "index", "value"):
        assert np.asarray(cat[k]).tobytes() == np.asarray(whole[k]).tobytes(), k


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [po.LIBSVM, po.CSV])
def test_gpu_fast_many_chunks_vs_oracle(dm, fmt):
    """Hundreds to thousands of chunks: the 64-ary chunk search of every tile
    (fast_common.h chunk_list, 1-3 load rounds) and a cluster of more starts
    than one tile takes (kMaxCs) that sends the input to the exact kernels."""
    rng = np.random.default_rng(5150)
    if fmt == po.LIBSVM:
        text, _ = synth.rows(synth.LIBSVM, 20000, 24, seed=8)
    else:
        text, _ = synth.rows(synth.CSV, 12000, 24, seed=8)
    data = text.tobytes()
    a = np.frombuffer(data, dtype=np.uint8)
    nl = np.flatnonzero(a == 10) + 1
    nl = nl[nl < len(data)]
    name = FMT_NAME[fmt]
    tile, max_cs = dm.fast_geometry()
    for n_cuts, cluster in ((65, False), (600, False), (5000, False), (600, True)):
        cuts = set(rng.choice(nl, size=min(n_cuts, len(nl)), replace=False).tolist())
        if cluster:
            cuts |= set(nl[(nl > 2 * tile + 100) & (nl < 3 * tile - 100)].tolist())  # one tile
        offs = [0] + sorted(cuts) + [len(data)]
        st = np.asarray(offs[:-1])  # chunk starts a tile lists: tlo <= s <= thi (fast_common.h)
        tl = np.arange(0, len(data), tile)
        per_tile = int((np.searchsorted(st, np.minimum(tl + tile, len(data)), "right")
                        - np.searchsorted(st, tl, "left")).max())
        h = _oracle_vs_gpu(dm, data, offs, fmt)
        assert h["path"] == ("exact" if per_tile > max_cs else "fast"), (name, n_cuts, per_tile, h["path"])


@pytest.mark.gpu
def test_gpu_libfm_synthetic_vs_oracle(dm):
    """libfm over many tiles and InputSplit-style chunks, 1-based ids with the
    three indexing modes, 32- and 64-bit ids, weights on some rows."""
    rng = np.random.default_rng(31337)
    data = fuzz_text.libfm_rows(rng, 3000, 40) + fuzz_text.libfm_rows(rng, 200, 7, weights=True)
    assert len(data) > 1 << 20
    for kw in ({}, {"indexing_mode": 1}, {"indexing_mode": -1}, {"index_bits": 64, "tile_bytes": 4096}):
        h = _oracle_vs_gpu(dm, data, _random_chunks(rng, data, 12), po.LIBFM, **kw)
        # the single-pass kernel in every mode (indexing_mode < 0: per-unit fix-up, svm_fast.h umin_fix)
        assert h["path"] == "fast", kw
        assert len(h["field"]) == len(h["index"]) > 100000
        he = _oracle_vs_gpu(dm, data, [0, len(data)], po.LIBFM, exact=True, **kw)
        assert he["path"] == "exact"


@pytest.mark.gpu
def test_gpu_csv_fast_label_column_vs_oracle(dm):
    """label_column on the single-pass CSV kernel (clean inputs of 2+ fields stay fast;
    empty labels, short rows and one-field rows go exact with the reference's
    result or error), plus canonical synthetic CSV with label_column 0 and 5."""
    rng = np.random.default_rng(9090)
    fast = 0
    for it in range(60):
        lc = int(rng.choice([0, 0, 1, 3]))
        nl = 3000 if it % 10 == 9 else int(rng.integers(1, 60))
        data = fuzz_text.labeled_csv(rng, nl, int(rng.integers(lc + 2, lc + 20)), lc,
                                     defects=0.0 if it % 2 == 0 else 0.08)
        offs = fuzz_text.random_cuts(rng, data, 6)
        h = _oracle_vs_gpu(dm, data, offs, po.CSV, label_column=lc)
        if it % 2 == 0:
            assert h["path"] == "fast", it
        fast += h["path"] == "fast"
    assert fast >= 30
    text, _ = synth.rows(synth.CSV, 6000, 256, seed=17)
    offs = dm.text_chunk_starts(text, 1 << 20).tolist()
    for lc in (0, 5):
        h = _oracle_vs_gpu(dm, text.tobytes(), offs, po.CSV, label_column=lc)
        assert h["path"] == "fast" and len(h["label"]) == 6000 and len(h["index"]) == 6000 * 255


@pytest.mark.gpu
def test_gpu_libfm_fast_fuzz_vs_oracle(dm):
    """Uniform-grammar libfm (pairs without values, dropped lone fields,
    weights, CR/LF, chunk cuts anywhere) through the single-pass kernel and
    violations through the exact kernels: the reference's result or error."""
    rng = np.random.default_rng(717)
    paths = {"fast": 0, "exact": 0}
    for it in range(200):
        big = it % 10 == 9
        data = fuzz_text.uniform_libfm(rng, 2000 if big else int(rng.integers(1, 60)), 24 if big else 10,
                                       violate=it % 3 == 2)
        offs = fuzz_text.random_cuts(rng, data, 8, anywhere=it % 5 == 4)
        kw = {}
        if it % 4 == 1:
            kw["indexing_mode"] = 1
        if it % 7 == 3:
            kw["index_bits"] = 64
        h = _oracle_vs_gpu(dm, data, offs, po.LIBFM, **kw)
        paths[h["path"]] += 1
        if it % 3 != 2 and it % 5 != 4:
            assert h["path"] == "fast", it
    assert paths["fast"] >= 90 and paths["exact"] >= 30, paths


# ------------------------------------------ FillData nthread range split --
FILLDATA = load_json("filldata.json")


def test_gpu_filldata_goldens(dm):
    """TextParserBase::FillData with nthread = 1..4 ranges per chunk
    (range_kernel + per-unit parsing): the genuine reference's arrays, errors
    and per-block counts (indexing_mode < 0 detection is per range)."""
    for case in FILLDATA:
        prm = case["params"]
        h = gpu_parse(dm, case["data_latin1"], case["offs"], prm["fmt"], **gpu_kwargs(prm))
        assert h["failed"] == bool(case["status"]), (case["name"], h["error"], case["msg"])
        if case["status"]:
            continue
        exp = {k: dec(v) for k, v in case["expect"].items()}
        assert diff(h, exp) == [], case["name"]
        assert blocks_of(h) == case["blocks"], case["name"]


@pytest.mark.parametrize("fmt", [po.LIBSVM, po.CSV, po.LIBFM])
def test_gpu_filldata_fuzz_vs_oracle(dm, fmt):
    """nthread in {1, 2, 3} x indexing_mode in {-1, 0, 1} on the fast and the
    exact path, many chunks and long lines: equal to the oracle's FillData."""
    rng = np.random.default_rng(606 + fmt)
    for it in range(90):
        nthread = 1 + it % 3
        if fmt == po.CSV:
            data = fuzz_text.uniform_csv(rng, int(rng.integers(1, 300)), int(rng.integers(1, 30)), ",",
                                         violate=it % 5 == 4)
            kw = {}
        elif fmt == po.LIBSVM:
            data = fuzz_text.uniform_libsvm(rng, int(rng.integers(1, 300)), int(rng.integers(0, 30)),
                                            violate=it % 5 == 4)
            kw = {"indexing_mode": (it // 3) % 3 - 1}
        else:
            data = fuzz_text.uniform_libfm(rng, int(rng.integers(1, 300)), 10, violate=it % 5 == 4)
            kw = {"indexing_mode": (it // 3) % 3 - 1}
        offs = fuzz_text.random_cuts(rng, data, 6)
        o = po.parse_chunks(data, offs, fmt=fmt, nthread=nthread, **kw)
        for exact in (False, True):
            h = gpu_parse(dm, data, offs, fmt, nthread=nthread, exact=exact, **kw)
            assert (o["status"] != 0) == h["failed"], (it, exact, o["msg"], h["error"])
            if o["status"] == 0:
                assert diff(h, o) == [], (it, exact, kw, nthread)
                assert blocks_of(h)["rows"] == o["blocks"]["rows"].tolist(), (it, exact)


def test_gpu_valve_hand_over_vs_oracle(dm):
    """a COUNT_ONLY that stood on the single-pass kernel followed by
    a FILL_ONLY whose single-pass write hands over (the kSpinLimit valve) must
    count on the exact path before writing.  The valve build makes tile 1 of
    every write pass hand over; results must equal the oracle (child process:
    the valve library replaces the product library)."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "dmlc-core_amd", "lib", "variants", "libdmlc_amd_valve.so")
    assert os.path.exists(lib), "build it: make -C dmlc-core_amd valve"
    r = subprocess.run([sys.executable, os.path.join(root, "tests", "valve_child.py")], capture_output=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    res = json.loads(r.stdout.decode().strip().splitlines()[-1])
    for e in res:
        assert e["split_path"] & 2 and e["full_path"] & 2, e  # the valve fired in the write pass
        assert e["split_error"] == 0 and e["full_error"] == 0, e
        assert e["split_diff"] == [] and e["full_diff"] == [], e


@pytest.mark.parametrize("nbytes,shift", [(10_000_007, 0), (4096, 0), (15, 0), (1 << 20, 3)])
def test_gpu_kernel_copy_host_device(dm, nbytes, shift):
    """dmlc_amd_copy (the engine's H2D / D2H): page-locked host <-> HBM byte for
    byte, odd sizes through the tail kernel, unaligned pointers through the
    hipMemcpyAsync fallback."""
    import torch
    L = dm.lib()
    rng = np.random.default_rng(nbytes)
    src = torch.from_numpy(rng.integers(0, 256, nbytes + shift, dtype=np.uint8)).pin_memory()
    dev = torch.zeros(nbytes + 16, dtype=torch.uint8, device="cuda")
    back = torch.zeros(nbytes + shift, dtype=torch.uint8).pin_memory()
    s = torch.cuda.current_stream().cuda_stream
    assert L.dmlc_amd_copy(dev.data_ptr(), src.data_ptr() + shift, nbytes, s) == 0
    assert L.dmlc_amd_copy(back.data_ptr() + shift, dev.data_ptr(), nbytes, s) == 0
    torch.cuda.synchronize()
    assert torch.equal(dev[:nbytes].cpu(), src[shift:])
    assert int(dev[nbytes:].sum()) == 0  # nothing past the end
    assert torch.equal(back[shift:], src[shift:])


def test_gpu_kernel_copy_n(dm):
    """dmlc_amd_copy_n (the engine's D2H of a batch's CSR arrays in one
    launch): every pair byte for byte, odd sizes (tails), empty entries
    skipped, an unaligned pair on its own, nothing written past an end."""
    import ctypes
    import torch
    L = dm.lib()
    rng = np.random.default_rng(5)
    sizes = [8 * 300001, 0, 13, 4 * 2_000_003, 4096, 1 << 20, 7, 64 * 1001]
    srcs = [torch.from_numpy(rng.integers(0, 256, n + 32, dtype=np.uint8)).cuda() for n in sizes]
    dsts = [torch.zeros(n + 32, dtype=torch.uint8).pin_memory() for n in sizes]
    shift = [0] * len(sizes)
    shift[6] = 3  # unaligned host side
    dp = (ctypes.c_void_p * len(sizes))(*[d.data_ptr() + h for d, h in zip(dsts, shift)])
    sp = (ctypes.c_void_p * len(sizes))(*[x.data_ptr() for x in srcs])
    nb = (ctypes.c_uint64 * len(sizes))(*sizes)
    s = torch.cuda.current_stream().cuda_stream
    assert L.dmlc_amd_copy_n(dp, sp, nb, len(sizes), s) == 0
    torch.cuda.synchronize()
    for n, h, x, d in zip(sizes, shift, srcs, dsts):
        assert torch.equal(d[h:h + n], x[:n].cpu()), n
        assert int(d[h + n:].sum()) == 0 and int(d[:h].sum()) == 0, n
    assert L.dmlc_amd_copy_n(dp, sp, nb, 17, s) != 0  # more than DMLC_AMD_COPY_MAX


def test_gpu_kernel_copy_n_dev(dm):
    """dmlc_amd_copy_n_dev (the engine's copy-out queued behind the parse):
    sizes count * scale + add read on the device, clamped at max_bytes,
    constant sizes for slot < 0, nothing written past a size."""
    import ctypes
    import torch
    L = dm.lib()
    L.dmlc_amd_copy_n_dev.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                      ctypes.c_void_p]
    rng = np.random.default_rng(6)
    counts = torch.tensor([300001, 0, 7, 2_000_003, 5, 9, 11, 1], dtype=torch.int64, device="cuda")
    slot = [0, 1, 2, 3, 4, -1, 6, 7]
    scale = [8, 4, 1, 4, 16, 0, 4, 4]
    add = [8, 0, 6, 0, 0, 4096, 0, 0]
    maxb = [8 * 300002 + 64, 64, 64, 4 * 2_000_003 + 64, 48, 5000, 40, 64]  # entries 4 and 6 clamp
    c = counts.cpu().numpy()
    want = [min(maxb[i], (int(c[slot[i]]) * scale[i] + add[i]) if slot[i] >= 0 else add[i]) for i in range(8)]
    srcs = [torch.from_numpy(rng.integers(0, 256, m + 32, dtype=np.uint8)).cuda() for m in maxb]
    dsts = [torch.zeros(m + 32, dtype=torch.uint8).pin_memory() for m in maxb]
    arr = lambda t, v: (t * len(v))(*v)  # noqa: E731
    rc = L.dmlc_amd_copy_n_dev(arr(ctypes.c_void_p, [d.data_ptr() for d in dsts]),
                               arr(ctypes.c_void_p, [x.data_ptr() for x in srcs]), counts.data_ptr(),
                               arr(ctypes.c_int, slot), arr(ctypes.c_uint64, scale), arr(ctypes.c_uint64, add),
                               arr(ctypes.c_uint64, maxb), 8, torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    for n, x, d in zip(want, srcs, dsts):
        assert torch.equal(d[:n], x[:n].cpu()), n
        assert int(d[n:].sum()) == 0, n


@pytest.mark.parametrize("fmt", [po.LIBSVM, po.LIBFM])
def test_gpu_qid_letter_forms_vs_oracle(dm, fmt):
    """Letters of "qid" that spell no "qid:" token leave the single-pass
    grammar (svm_fast.h qid_clean's verdict is kept): the reference's result
    or its error, in a one-line input and in the middle of a multi-tile file."""
    lines = ["1 dqi:5 3:4\n", "1 iq:5 3:4\n", "1 qi 3:4\n", "1 d 2:3\n", "1 qid:7 3:4\n",
             "1 qidd:7 3:4\n", "1 q 2:3:4\n", "1 2:3:4 d\n", "1 qqid:3 2:1\n", "1:2 idq:4 5:6\n"]
    for line in lines:
        for data in (line, "0 1:1\n" * 7000 + line + "0 1:1\n" * 3000):
            _gpu_vs_oracle_paths(dm, data, [0, len(data)], fmt=fmt)


def _gpu_vs_oracle_vt(dm, data, offs, vt, **kw):
    """_gpu_vs_oracle_paths with a CSV value type (the oracle calls it value_kind)."""
    o = po.parse_chunks(data, offs, fmt=po.CSV, value_kind=vt, **kw)
    res = {}
    for exact in (False, True):
        h = dm.parse_bytes(data, offs, fmt="csv", exact=exact, value_type=vt, **kw)
        nch = len(offs) - 1
        failed = bool(h["error"]) or (nch > 0 and dm.chunk_check(h, "csv", nch, h["counts"]) >= 0)
        assert (o["status"] != 0) == failed, (exact, o["msg"], h["error"], data[:200], offs, kw)
        if not failed:
            assert diff(h, o) == [], (exact, diff(h, o), offs, kw)
        res[exact] = h
    if o["status"] == 0:
        assert res[False]["chunk_table"].tolist() == res[True]["chunk_table"].tolist()
    return res[False]


@pytest.mark.parametrize("vt", [0, 1, 2])
def test_gpu_csv_fast_blanks_and_ints_vs_oracle(dm, vt):
    """Blanks around values (", " separators, padded and blank-only fields)
    and integer DTypes (strtoll base 0) on the single-pass CSV kernels
    (csv_fast.h): bit-exact against the oracle on both paths, most inputs on
    the single pass; a blank field that runs into the next line goes exact."""
    rng = np.random.default_rng(900 + vt)
    paths = {"fast": 0, "exact": 0}
    for it in range(120):
        big = it % 10 == 9
        delim = ",;|"[it % 3]
        data = fuzz_text.blank_csv(rng, 2500 if big else int(rng.integers(1, 40)), 50 if big else 25, delim,
                                   ints=vt != 0 or rng.random() < 0.2, violate=(not big) and rng.random() < 0.2)
        offs = fuzz_text.random_cuts(rng, data, 8 if big else 5, anywhere=rng.random() < 0.2)
        kw = {"delimiter": delim}
        if rng.random() < 0.2:
            kw["index_bits"] = 64
        if vt and rng.random() < 0.3:
            kw["weight_column"] = int(rng.integers(0, 3))
        try:
            paths[_gpu_vs_oracle_vt(dm, data, offs, vt, **kw)["path"]] += 1
        except AssertionError as e:
            raise AssertionError("case %d: %s" % (it, e))
    assert paths["fast"] > 70, paths


def test_gpu_csv_variant_bench_configs_fast(dm):
    """The bench's CSV grammar variants (", " separators; int32 / int64
    DTypes: glibc strtoll base 0, csv_parser.h:99-105) at 100k rows x 256
    columns: the single-pass kernels and the exact kernels each equal the
    oracle bit for bit (at full size: the reference hashes csv_i32_1m_x256 /
    csv_sp_i64_1m_x256 in test_gpu_fullsize_vs_reference_hashes)."""
    import torch
    for fmt, vt in ((synth.CSV_SP, 0), (synth.CSV, 1), (synth.CSV_SP, 2)):
        text, _ = synth.rows(fmt, 100000, 256, seed=3)
        starts = dm.text_chunk_starts(text)
        d_text = torch.from_numpy(text).cuda()
        d_cs = torch.from_numpy(starts).cuda()
        o = po.parse_chunks(text.tobytes(), starts.tolist(), fmt=po.CSV, value_kind=vt)
        assert o["status"] == 0
        for exact in (False, True):
            p = dm.DeviceParser("csv", value_type=vt, flags=dm.FLAG_EXACT if exact else 0)
            out = p.parse(d_text, d_cs)
            assert out["error"] == 0 and out["path"] == (1 if exact else 0), (fmt, vt, exact, out["path"])
            for k in ("offset", "index", "value"):  # (no label column: no labels)
                a, b = out[k].cpu().numpy(), np.asarray(o[k])
                assert a.shape == b.shape and a.tobytes() == b.astype(a.dtype).tobytes(), (fmt, vt, exact, k)


def test_gpu_indexing_mode_auto_one_based_bench_shape(dm):
    """indexing_mode=-1 at bench shape (bench.py libsvm_1b_im1_1m_x128): the
    1-based rows (tools/synth.c fmt 6, every id of config 2 one higher) hold
    no 0 id in any unit, so every id drops by one -- the result equals the
    0-based rows parsed as they are (nthread 1 and 2, 8 MiB chunks)."""
    text1, _ = synth.rows(synth.LIBSVM_1B, 120000, 128, seed=3)
    text0, _ = synth.rows(synth.LIBSVM, 120000, 128, seed=3)
    for nthread in (1, 2):
        offs1 = dm.text_chunk_starts(text1).tolist()
        offs0 = dm.text_chunk_starts(text0).tolist()
        h1 = gpu_parse(dm, text1.tobytes(), offs1, indexing_mode=-1, nthread=nthread)
        h0 = gpu_parse(dm, text0.tobytes(), offs0, nthread=nthread)
        assert h1["path"] == "fast" and not h1["failed"] and not h0["failed"]
        for k in ("offset", "label", "index", "value"):
            assert np.asarray(h1[k]).tobytes() == np.asarray(h0[k]).tobytes(), (nthread, k)


@pytest.mark.parametrize("nthread", [1, 2])
def test_gpu_fast_indexing_mode_auto_vs_oracle(dm, nthread):
    """indexing_mode=-1 on the single-pass libsvm / libfm kernels: each
    ParseBlock unit's ids drop by one when all of them are > 0
    (libsvm_parser.h:165-171, libfm_parser.h:133-143); 1-based and 0-based
    units side by side, tile-crossing unit starts, both id widths."""
    rng = np.random.default_rng(64 + nthread)
    for it in range(12):
        rows = []
        n = int(rng.integers(50, 3000))
        zeros = set(rng.integers(0, n, size=int(rng.integers(0, 3))).tolist())
        for r in range(n):
            ids = sorted(set(int(x) for x in rng.integers(1, 100000, size=int(rng.integers(1, 40)))))
            if r in zeros:
                ids = [0] + ids
            rows.append("%d %s" % (r % 2, " ".join("%d:%.7g" % (i, rng.random()) for i in ids)))
        data = ("\n".join(rows) + "\n").encode()
        offs = fuzz_text.random_cuts(rng, data, 8)
        kw = {"indexing_mode": -1, "nthread": nthread, "index_bits": 64 if it % 3 == 2 else 32}
        h = _gpu_vs_oracle_paths(dm, data, offs, **kw)
        assert h["path"] == "fast", it
    # libfm
    rng = np.random.default_rng(99)
    for it in range(6):
        rows = []
        for r in range(1500):
            lo = 0 if (it % 2 and r == 700) else 1
            rows.append("%d %s" % (r % 2, " ".join("%d:%d:%.6g" % (int(rng.integers(lo, 9)), int(rng.integers(lo, 900)),
                                                                     rng.random()) for _ in range(int(rng.integers(1, 12))))))
        data = ("\n".join(rows) + "\n").encode()
        offs = fuzz_text.random_cuts(rng, data, 5)
        h = _gpu_vs_oracle_paths(dm, data, offs, fmt=po.LIBFM, indexing_mode=-1, nthread=nthread)
        assert h["path"] == "fast", it


FULL = load_json("synth_full.json") if __import__("os").path.exists(
    __import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "synth_full.json")) else {}


@pytest.mark.parametrize("name", sorted(FULL))
def test_gpu_fullsize_vs_reference_hashes(dm, name):
    """BASELINE configs 2-5 at full size (config 5: each of bench.py's 8
    per-rank shards) and the bench's variants of configs 2 / 3 (nthread 2,
    the exact kernels, nan fields + BOM, qid, comments, 1-based ids with
    indexing_mode -1, libfm), generated and chunked exactly as the bench does,
    parsed on the GPU with the bench's parameters, every output array hashed and compared with the
    SHA-256 the GENUINE reference's ParseBlock produced for the same chunks
    (tests/golden/make_fullsize.py, oracle/_ref).  The text streams to the
    device chunk by chunk and the arrays stream back in slices, so host memory
    stays bounded (config 4 is 37 GB of text)."""
    import hashlib
    import sys
    import torch
    sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__file__), "golden"))
    import make_fullsize as mf
    fx = FULL[name]
    sfmt, _, rows, width, row0 = mf.CONFIGS[name]
    d_text = torch.empty(fx["input_bytes"], dtype=torch.uint8, device="cuda")
    starts, pos = [0], 0
    for i, ch in enumerate(mf.stream_chunks(sfmt, rows, width, row0, max(1, (16 << 20) // (width * 16)))):
        if i == 0:
            assert hashlib.sha256(ch).hexdigest() == fx["first_chunk_sha256"]
        d_text[pos:pos + len(ch)].copy_(torch.frombuffer(bytearray(ch), dtype=torch.uint8))
        pos += len(ch)
        starts.append(pos)
    assert pos == fx["input_bytes"] and len(starts) - 1 == fx["chunks"]
    d_cs = torch.tensor(starts, dtype=torch.int64, device="cuda")
    flags, want_path = mf.FLAGS.get(name, (None, 0))
    p = dm.DeviceParser(fx["format"], flags=dm.FLAG_EXACT if flags == "exact" else 0, **mf.gpu_kw(name))
    out = p.parse(d_text, d_cs)
    del d_text
    assert out["error"] == 0 and out["path"] == want_path, (out["error"], out["path"])
    c = out["counts"]
    for k, slot in (("offset", dm.ROWS), ("label", dm.LABEL), ("weight", dm.WEIGHT), ("qid", dm.QID),
                    ("field", dm.FIELD), ("index", dm.INDEX), ("value", dm.VALUE)):
        n = c[slot] + (1 if k == "offset" else 0)
        assert n == fx["sizes"][k], (k, n, fx["sizes"][k])
        h = hashlib.sha256()
        t = out[k]
        for a in range(0, n, 1 << 26):
            h.update(t[a:min(n, a + (1 << 26))].cpu().numpy().tobytes())
        assert h.hexdigest() == fx["sha256"][k], k


@pytest.mark.parametrize("fmt", ["libsvm", "libfm"])
def test_gpu_umin_fix_stays_inside_capacity(dm, fmt):
    """indexing_mode=-1 on the single pass with outputs smaller than the
    counts: the write pass raises the capacity error, and the 1-based shift
    afterwards (umin_fix_kernel) touches no entry past cap[INDEX] / cap[FIELD]
    -- guard words after the arrays stay as they were."""
    import torch
    rng = np.random.default_rng(11)
    lines = []
    for i in range(20000):
        ids = np.sort(rng.choice(np.arange(1, 5000), 8, replace=False))
        if fmt == "libsvm":
            lines.append("%d %s\n" % (i % 2, " ".join("%d:%.3f" % (j, rng.random()) for j in ids)))
        else:
            lines.append("%d %s\n" % (i % 2, " ".join("%d:%d:%.3f" % (1 + j % 7, j, rng.random()) for j in ids)))
    text = "".join(lines).encode()
    starts = dm.text_chunk_starts(text, 1 << 16)
    d_text = torch.frombuffer(bytearray(text), dtype=torch.uint8).cuda()
    d_cs = torch.tensor(starts, device="cuda")
    p = dm.DeviceParser(fmt, indexing_mode=-1)
    res = torch.zeros(16, dtype=torch.int64, device="cuda")
    counts = [int(x) for x in p.count(d_text, d_cs, result=res)]
    n = counts[dm.INDEX]
    assert n == 8 * 20000
    guard = 4096
    sent = 0x5A5A5A5A
    out = p.alloc(counts)
    out["index"] = torch.full((n + guard,), sent, dtype=torch.int32, device="cuda")
    out["field"] = torch.full((n + guard,), sent, dtype=torch.int32, device="cuda")
    small = list(counts)
    small[dm.INDEX] = n // 2
    if fmt == "libfm":
        small[dm.FIELD] = n // 3
    out["counts"] = small
    p.parse_into(d_text, d_cs, out, res)
    r = res.cpu().numpy().view(np.uint64)
    assert dm.error_code(r[8]) == dm.ERR_CAPACITY
    idx = out["index"].cpu().numpy()
    assert (idx[small[dm.INDEX]:] == sent).all()
    assert (idx[:small[dm.INDEX]] != sent).all()
    if fmt == "libfm":
        fld = out["field"].cpu().numpy()
        assert (fld[small[dm.FIELD]:] == sent).all()


def test_gpu_csv_nan_bom_bench_shape(dm):
    """The csv_nan_1m_x256 bench shape -- config 3's rows with 0.1 % of the
    fields "nan" and a UTF-8 BOM at the file head (tools/synth.c fmt 7) -- on
    the single-pass kernel, equal to the oracle (NaN bit patterns included)."""
    text, _ = synth.rows(synth.CSV_NAN, 40000, 256, seed=3)
    data = text.tobytes()
    assert data[:3] == b"\xef\xbb\xbf" and data.count(b"nan") > 5000
    offs = dm.text_chunk_starts(text, 1 << 20).tolist()
    h = gpu_parse(dm, data, offs, po.CSV)
    assert h["path"] == "fast" and not h["failed"]
    o = po.parse_chunks(data, offs, fmt=po.CSV)
    assert o["status"] == 0 and diff(h, o) == []
    assert np.isnan(np.asarray(h["value"])).sum() == data.count(b"nan")
