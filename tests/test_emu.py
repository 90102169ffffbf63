"""CPU runs of the kernel tile bodies (test-only emulator, ASan) vs goldens/oracle.

The emulator executes the same per-thread code as the HIP kernels
(dmlc-core_amd/csrc/*_core.h) with 256 host threads per workgroup; these tests
catch logic and memory-safety bugs in the kernel bodies without a GPU."""
import os

import numpy as np
import pytest

import fuzz_text
from golden_util import blocks_of, dec, diff, load_cases, load_json
from oracle import pyoracle as po
from tests.emu import pyemu
from tools import synth

FMT = {po.LIBSVM: "libsvm", po.CSV: "csv", po.LIBFM: "libfm"}


def check_fail(h, fmt, offs):
    import dmlc_amd
    nch = len(offs) - 1
    return bool(h["error"]) or (nch > 0 and dmlc_amd.chunk_check(h, fmt, nch, h["counts"]) >= 0)


def kw_of(params):
    kw = {}
    for k, v in params.items():
        if k in ("fmt", "nthread"):
            continue
        kw["value_type" if k == "value_kind" else k] = v
    return kw


CASES = [c for c in load_cases() if c["params"]["fmt"] in FMT]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_emu_goldens(case):
    prm = case["params"]
    data = case["data_latin1"].encode("latin-1")
    offs = [0, len(data)] if data else [0]
    h = pyemu.parse(data, offs, FMT[prm["fmt"]], **kw_of(prm))
    failed = check_fail(h, FMT[prm["fmt"]], offs)
    if case["status"]:
        assert failed
        return
    assert not failed, h["error"]
    exp = {k: dec(v) for k, v in case["expect"].items()}
    assert diff(h, exp) == []


def _fuzz(rng, fmt):
    alpha = {po.LIBSVM: list("0123456789") * 6 + list("  ::.-+eE#\tq") + ["qid:", "nan", "inf", "\r"],
             po.CSV: list("0123456789") * 6 + list(",,,,.-+eE \t") + ["nan", "inf", "0x", "\xef\xbb\xbf"],
             po.LIBFM: list("0123456789") * 6 + list("  :::.-+eE#\t") + ["\r", "nan", "x"]}[fmt]
    lines = ["".join(alpha[int(i)] for i in rng.integers(0, len(alpha), int(rng.integers(0, 60))))
             for _ in range(int(rng.integers(1, 10)))]
    t = "\n".join(lines) + ("\n" if rng.random() < 0.5 else "")
    return t.encode("latin-1")


@pytest.mark.parametrize("fmt", [po.LIBSVM, po.CSV, po.LIBFM])
def test_emu_fuzz_vs_oracle(fmt):
    rng = np.random.default_rng(99 + fmt)
    for it in range(60):
        data = _fuzz(rng, fmt)
        nl = [i + 1 for i, b in enumerate(data) if b in (10, 13) and i + 1 < len(data)]
        cuts = sorted(set(rng.choice(nl, size=min(len(nl), int(rng.integers(0, 3))), replace=False).tolist())) if nl else []
        offs = [0] + cuts + [len(data)]
        kw = {}
        if rng.random() < 0.4:
            kw["tile_bytes"] = int(rng.integers(8, 64))
        if fmt == po.CSV and rng.random() < 0.3:
            kw["label_column"] = int(rng.integers(0, 3))
        if fmt in (po.LIBSVM, po.LIBFM) and rng.random() < 0.3:
            kw["indexing_mode"] = int(rng.integers(-1, 2))
        if fmt == po.LIBFM and rng.random() < 0.2:
            kw["index_bits"] = 64
        okw = {k: v for k, v in kw.items() if k != "tile_bytes"}
        o = po.parse_chunks(data, offs, fmt=fmt, **okw)
        h = pyemu.parse(data, offs, FMT[fmt], **kw)
        failed = check_fail(h, FMT[fmt], offs)
        assert (o["status"] != 0) == failed, (it, data, offs, kw, o["msg"], h["error"])
        if not failed:
            assert diff(h, o) == [], (it, data, offs, kw, diff(h, o))


def test_emu_long_lines_small_tiles():
    rng = np.random.default_rng(3)
    lines = []
    for r in range(5):
        k = int(rng.integers(200, 1500))
        lines.append("%d%s %s" % (r % 2, " qid:%d" % r if r % 2 else "",
                                  " ".join("%d:%.6g" % (i, rng.random()) for i in range(k))))
    data = ("\n".join(lines) + "\n").encode()
    for tile in (0, 5000, 20000):
        o = po.parse_chunks(data, [0, len(data)], fmt=po.LIBSVM)
        h = pyemu.parse(data, [0, len(data)], "libsvm", tile_bytes=tile)
        assert h["error"] == 0 and diff(h, o) == []


# ---------------------------------------------------------------- fast path --


def _emu_vs_oracle(data, offs, exact=False, **kw):
    o = po.parse_chunks(data, offs, fmt=po.LIBSVM, **kw)
    h = pyemu.parse(data, offs, "libsvm", exact=exact, **kw)
    failed = check_fail(h, "libsvm", offs)
    assert (o["status"] != 0) == failed, (data[:200], offs, kw, o["msg"], h["error"])
    if not failed:
        assert diff(h, o) == [], (diff(h, o), offs, kw)
    return h


def test_emu_fast_fuzz_vs_oracle():
    """Uniform-grammar inputs (single tile) with violations and odd chunkings:
    whichever path runs, the result is the reference's."""
    rng = np.random.default_rng(2024)
    paths = {"fast": 0, "exact": 0}
    for it in range(50):
        data = fuzz_text.uniform_libsvm(rng, int(rng.integers(1, 30)), int(rng.integers(0, 30)),
                                        violate=rng.random() < 0.3)
        offs = fuzz_text.random_cuts(rng, data, 5, anywhere=rng.random() < 0.3)
        kw = {}
        if rng.random() < 0.2:
            kw["index_bits"] = 64
        if rng.random() < 0.2:
            kw["indexing_mode"] = 1
        paths[_emu_vs_oracle(data, offs, **kw)["path"]] += 1
    assert paths["fast"] > 20 and paths["exact"] > 5, paths


def test_emu_fast_multi_tile():
    """Inputs spanning several 16 KiB tiles: look-back across tiles, runs and
    lines crossing tile ends, long gaps, chunk starts at arbitrary bytes."""
    rng = np.random.default_rng(77)
    for it in range(4):
        data = fuzz_text.uniform_libsvm(rng, 300, 60)
        offs = fuzz_text.random_cuts(rng, data, 8, anywhere=it % 2 == 1)
        h = _emu_vs_oracle(data, offs)
        assert len(data) > 3 * 16384
        if it % 2 == 0:
            assert h["path"] == "fast"


def test_window_decoders_vs_byte_decoders():
    """The 16-byte window decoders (fast_common.h wfloat32m / wuint32m, the
    fast kernels' number conversion) against the exact byte decoders on 2M
    generated number strings: every string the window form accepts decodes
    bit-identically (tests/emu/dec_check.cpp)."""
    import os
    import subprocess
    pyemu.build()
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "emu", "_build", "dec_check")
    r = subprocess.run([exe, "2000000", "7"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:]
    fast_f = int(r.stdout.split("float fast ")[1].split(",")[0])
    assert fast_f > 1000000, r.stdout


def test_emu_fast_dense_runs():
    """Tiles with thousands of one-byte runs: the run lists of the libsvm
    write pass overflow the planes' LDS and are decoded in passes
    (svm_fast.h kPassRuns); labels, weights and values across the pass seams."""
    rng = np.random.default_rng(91)
    for it, style in enumerate(("pairs", "weights", "labels", "mixed")):
        data = fuzz_text.dense_libsvm(rng, 3 * 16384 + 777, style)
        offs = fuzz_text.random_cuts(rng, data, 4, anywhere=False)
        h = _emu_vs_oracle(data, offs, **({"index_bits": 64} if it == 1 else {}))
        assert h["path"] == "fast", style


def test_emu_fast_qid_vs_oracle():
    """"qid:" in the single-pass grammar (svm_fast.h qid_clean / qid_ok /
    qid_decide): ranking rows, one and several tiles, odd chunkings; the
    forms the reference reads differently and rows without a qid go to the
    exact kernels -- whichever path runs, the reference's result."""
    rng = np.random.default_rng(4242)
    paths = {"fast": 0, "exact": 0}
    for it in range(40):
        big = it % 8 == 0
        data = fuzz_text.qid_libsvm(rng, 400 if big else int(rng.integers(1, 30)), 40 if big else 12,
                                    violate=it % 4 == 3, mixed=it % 10 == 9)
        offs = fuzz_text.random_cuts(rng, data, 6, anywhere=it % 5 == 4)
        kw = {"index_bits": 64} if it % 3 == 1 else {}
        h = _emu_vs_oracle(data, offs, **kw)
        paths[h["path"]] += 1
        if it % 4 != 3 and it % 10 != 9 and it % 5 != 4:
            assert h["path"] == "fast", (it, data[:300])
    assert paths["fast"] >= 20 and paths["exact"] >= 5, paths


def test_emu_fast_qid_long_heads_vs_oracle():
    """qid runs whose line head (label, weight, blanks before the token) is
    longer than the tile's 64-byte pre-halo or crosses a tile start
    (svm_fast.h Tile::qid_ok reads the staged text only), tabs among long
    blanks."""
    rng = np.random.default_rng(4343)
    fast = 0
    for it in range(24):
        data = fuzz_text.qid_libsvm(rng, int(rng.integers(5, 60)), 10, violate=it % 6 == 5, long_head=True)
        offs = fuzz_text.random_cuts(rng, data, 4, anywhere=it % 4 == 3)
        h = _emu_vs_oracle(data, offs, **({"index_bits": 64} if it % 3 == 1 else {}))
        fast += h["path"] == "fast"
    assert fast >= 8, fast


def test_emu_libfm_dense_runs():
    """libfm tiles of one-byte runs: index, field and value lists in passes."""
    rng = np.random.default_rng(93)
    for it in range(3):
        data = fuzz_text.dense_libfm(rng, 2 * 16384 + 555)
        offs = fuzz_text.random_cuts(rng, data, 3, anywhere=False)
        o = po.parse_chunks(data, offs, fmt=po.LIBFM)
        h = pyemu.parse(data, offs, "libfm")
        assert o["status"] == 0 and not check_fail(h, "libfm", offs), o["msg"]
        assert h["path"] == "fast" and diff(h, o) == []


def test_emu_fast_equals_exact_synthetic():
    text, _ = synth.rows(synth.LIBSVM, 800, 40, seed=5)
    data = text.tobytes()
    offs = [0, len(data) // 2 + data[len(data) // 2:].index(b"\n") + 1, len(data)]
    hf = _emu_vs_oracle(data, offs)
    he = _emu_vs_oracle(data, offs, exact=True)
    assert hf["path"] == "fast" and he["path"] == "exact"
    assert hf["chunk_table"].tolist() == he["chunk_table"].tolist()


def test_emu_csv_fast_fuzz_vs_oracle():
    """Uniform-CSV inputs through the single-pass CSV tile body, one and
    several tiles, odd chunkings: whichever path runs, the reference's result."""
    rng = np.random.default_rng(606)
    fast = 0
    for it in range(40):
        delim = ",;"[it % 2]
        big = it % 8 == 7
        data = fuzz_text.uniform_csv(rng, 900 if big else int(rng.integers(1, 30)),
                                     120 if big else int(rng.integers(1, 30)), delim,
                                     violate=(not big) and rng.random() < 0.25)
        offs = fuzz_text.random_cuts(rng, data, 5, anywhere=rng.random() < 0.3)
        o = po.parse_chunks(data, offs, fmt=po.CSV, delimiter=delim)
        h = pyemu.parse(data, offs, "csv", delimiter=delim)
        failed = check_fail(h, "csv", offs)
        assert (o["status"] != 0) == failed, (it, data[:200], offs, o["msg"], h["error"])
        if not failed:
            assert diff(h, o) == [], (it, diff(h, o), offs)
        fast += h["path"] == "fast"
    assert fast > 20, fast


def test_emu_csv_dense_tokens():
    """CSV tiles of one-digit fields: the token lists (csv_fast.h) in several
    passes, rows carried across tiles, a row past 2^17 columns (its tokens'
    list columns count from the tile start, the look-back adds the rest)."""
    rng = np.random.default_rng(717)
    for it in range(4):
        delim = ",;"[it % 2]
        data = fuzz_text.dense_csv(rng, 3 * 16384 + 321 if it < 3 else 300000, delim, wide=it == 3)
        offs = fuzz_text.random_cuts(rng, data, 3, anywhere=False)
        o = po.parse_chunks(data, offs, fmt=po.CSV, delimiter=delim)
        h = pyemu.parse(data, offs, "csv", delimiter=delim)
        assert o["status"] == 0 and not check_fail(h, "csv", offs), o["msg"]
        assert diff(h, o) == [], (it, diff(h, o)[:3])
        assert h["path"] == "fast", it


def _many_chunks(rng, data, n_cuts, cluster):
    """Chunk starts after newlines, n_cuts of them; plus a dense cluster (more
    starts inside one single-pass tile than it takes, kMaxCs) so both the
    64-ary chunk search (nchunk > 64, fast_common.h chunk_list) and the
    too-many-chunks fallback are exercised."""
    import dmlc_amd
    tile, max_cs = dmlc_amd.fast_geometry()
    a = np.frombuffer(data, dtype=np.uint8)
    nl = (np.flatnonzero(a == 10) + 1)
    nl = nl[nl < len(data)]
    cuts = set(rng.choice(nl, size=min(n_cuts, len(nl)), replace=False).tolist())
    mid = nl[(nl > 2 * tile) & (nl < 3 * tile)]  # a cluster in tile 2
    assert len(mid) > max_cs
    if cluster:
        cuts |= set(mid.tolist())
    return [0] + sorted(cuts) + [len(data)]


def test_emu_fast_many_chunks():
    rng = np.random.default_rng(91)
    for fmt in ("libsvm", "csv"):
        if fmt == "libsvm":
            text, _ = synth.rows(synth.LIBSVM, 2500, 12, seed=3)
        else:
            text, _ = synth.rows(synth.CSV, 2000, 16, seed=3)
        data = text.tobytes()
        assert len(data) > 3 * 16384
        for n_cuts, cluster in ((70, False), (300, False), (300, True)):
            offs = _many_chunks(rng, data, n_cuts, cluster)
            f = po.LIBSVM if fmt == "libsvm" else po.CSV
            o = po.parse_chunks(data, offs, fmt=f)
            # libsvm: the lean kernel (svm_lean.h) takes up to 63 unit starts
            # per wave, so the cluster stays on the single pass; the full
            # kernel alone (DMLC_AMD_LEAN=0) hands it to the exact kernels
            for lean in (("1", "0") if fmt == "libsvm" else ("1",)):
                os.environ["DMLC_AMD_LEAN"] = lean
                try:
                    h = pyemu.parse(data, offs, fmt)
                finally:
                    os.environ.pop("DMLC_AMD_LEAN", None)
                assert o["status"] == 0 and not check_fail(h, fmt, offs)
                assert diff(h, o) == [], (fmt, n_cuts, lean, diff(h, o))
                want = "exact" if cluster and (fmt == "csv" or lean == "0") else "fast"
                assert h["path"] == want, (fmt, n_cuts, lean, h["path"])


def test_emu_csv_fast_label_column():
    """label_column on the single-pass CSV kernel: clean inputs stay on it;
    empty labels, short rows, one-field rows (label 0: the reference's fatal
    'Delimiter not found') go to the exact kernels -- the reference's result
    (or error) either way."""
    rng = np.random.default_rng(8080)
    fast = 0
    for it in range(24):
        lc = int(rng.choice([0, 0, 1, 3]))
        nl = 400 if it % 6 == 5 else int(rng.integers(1, 40))
        data = fuzz_text.labeled_csv(rng, nl, int(rng.integers(lc + 2, lc + 12)), lc,
                                     defects=0.0 if it % 2 == 0 else 0.1)
        offs = fuzz_text.random_cuts(rng, data, 4)
        o = po.parse_chunks(data, offs, fmt=po.CSV, label_column=lc)
        h = pyemu.parse(data, offs, "csv", label_column=lc)
        failed = check_fail(h, "csv", offs)
        assert (o["status"] != 0) == failed, (it, lc, o["msg"], h["error"])
        if not failed:
            assert diff(h, o) == [], (it, lc, diff(h, o))
        if it % 2 == 0:
            assert h["path"] == "fast", it
        fast += h["path"] == "fast"
    assert fast >= 12


def test_emu_libfm_fast_vs_oracle():
    """libfm through the single-pass kernel (svm_fast.h with the libfm roles):
    clean uniform inputs stay on it; violations go exact; the reference's
    result or error either way, chunk tables included."""
    rng = np.random.default_rng(515)
    paths = {"fast": 0, "exact": 0}
    for it in range(40):
        big = it % 8 == 7
        data = fuzz_text.uniform_libfm(rng, 600 if big else int(rng.integers(1, 30)), 20 if big else 8,
                                       violate=it % 3 == 2)
        offs = fuzz_text.random_cuts(rng, data, 5, anywhere=it % 5 == 4)
        kw = {"indexing_mode": 1} if it % 4 == 1 else {}
        o = po.parse_chunks(data, offs, fmt=po.LIBFM, **kw)
        h = pyemu.parse(data, offs, "libfm", **kw)
        failed = check_fail(h, "libfm", offs)
        assert (o["status"] != 0) == failed, (it, data[:300], offs, o["msg"], h["error"])
        if not failed:
            assert diff(h, o) == [], (it, diff(h, o), offs)
        paths[h["path"]] += 1
        if it % 3 != 2 and it % 5 != 4:
            assert h["path"] == "fast", (it, data[:300])
    assert paths["fast"] >= 15 and paths["exact"] >= 3, paths


FILLDATA = load_json("filldata.json")


@pytest.mark.parametrize("case", FILLDATA[::3], ids=[c["name"] for c in FILLDATA[::3]])
def test_emu_filldata_goldens(case):
    """FillData ranges as ParseBlock units (host-computed in the emulator,
    range_kernel on the GPU): the reference's arrays, errors and blocks."""
    prm = case["params"]
    data = case["data_latin1"].encode("latin-1")
    offs = case["offs"]
    h = pyemu.parse(data, offs, FMT[prm["fmt"]], nthread=prm.get("nthread", 1), **kw_of(prm))
    nunits = (len(offs) - 1) * max(prm.get("nthread", 1), 1)
    failed = check_fail(h, FMT[prm["fmt"]], [0] * (nunits + 1))
    assert failed == bool(case["status"]), (h["error"], case["msg"])
    if case["status"]:
        return
    exp = {k: dec(v) for k, v in case["expect"].items()}
    assert diff(h, exp) == []
    assert blocks_of(h) == case["blocks"]


QID_LETTER_FORMS = ["1 dqi:5 3:4\n", "1 iq:5 3:4\n", "1 qi 3:4\n", "1 d 2:3\n", "1 qid:7 3:4\n",
                    "1 qidd:7 3:4\n", "1 q 2:3:4\n", "1 2:3:4 d\n", "1 qqid:3 2:1\n", "1:2 idq:4 5:6\n"]


@pytest.mark.parametrize("fmt", ["libsvm", "libfm"])
def test_emu_qid_letter_forms(fmt):
    """Letters of "qid" that do not spell a "qid:" token (svm_fast.h qid_clean
    reports them) leave the single-pass grammar: the reference's result or its
    error, never a role read off blanked letters."""
    f = {"libsvm": po.LIBSVM, "libfm": po.LIBFM}[fmt]
    for line in QID_LETTER_FORMS:
        for data in (line, "0 1:1\n" * 700 + line + "0 1:1\n" * 300):  # one tile / mid-file
            offs = [0, len(data)]
            o = po.parse_chunks(data, offs, fmt=f)
            h = pyemu.parse(data, offs, fmt)
            failed = check_fail(h, fmt, offs)
            assert (o["status"] != 0) == failed, (fmt, line, o["msg"], h["error"])
            if not failed:
                assert diff(h, o) == [], (fmt, line, diff(h, o))


def test_emu_fast_comments_vs_oracle():
    """'#' comments in the single-pass grammar (svm_fast.h comment_erase):
    comment lines, a header, trailing comments with any text, comments longer
    than the pre-halo across tile ends, odd chunkings, qid rows; forms the
    reference reads otherwise go to the exact kernels -- whichever path runs,
    the reference's result."""
    rng = np.random.default_rng(5151)
    paths = {"fast": 0, "exact": 0}
    for it in range(36):
        big = it % 3 == 0
        data = fuzz_text.comment_libsvm(rng, 500 if big else int(rng.integers(1, 30)), 30 if big else 12,
                                        long_frac=0.0 if it % 2 == 0 else 0.2, violate=it % 4 == 3,
                                        qid=it % 5 == 2, line_comments=it % 8 == 5)
        offs = fuzz_text.random_cuts(rng, data, 6, anywhere=it % 3 == 1)
        kw = {"index_bits": 64} if it % 7 == 1 else {}
        h = _emu_vs_oracle(data, offs, **kw)
        paths[h["path"]] += 1
        if it % 2 == 0 and it % 4 != 3 and it % 3 != 1:  # short comments, no violations, line-aligned cuts
            assert h["path"] == "fast", (it, data[:300])
    assert paths["fast"] >= 12 and paths["exact"] >= 3, paths


@pytest.mark.parametrize("body", ["x", " 1 2:3 4", "q:i#d"])
def test_emu_comments_across_tile_ends(body):
    """A comment whose '#' sits d bytes before a 16 KiB tile end and runs L
    bytes: inside the next tile's pre-halo (d <= 64) the next tile blanks it
    itself; further back the tile holding the '#' raises the gate.  Comment
    text of letters, of digits and ':' (which would parse as features), and
    of qid letters."""
    rng = np.random.default_rng(17)
    base = fuzz_text.uniform_libsvm(rng, 400, 20).replace(b"\r", b"\n")
    for d in (2, 64, 65, 300):
        for L in (3, 80, 20000):
            cut = base.index(b"\n", 16384 - d - 200) + 1  # a line start before the tile end
            pre = base[:cut] + b"7" + b" " * max(0, 16384 - d - cut - 6) + b" 1:2 "  # '#' right after a pair
            assert len(pre) == 16384 - d
            com = (b"#" + (body.encode() * (L // len(body) + 1))[:L]).replace(b"\n", b" ")
            data = pre + com + b"\n" + base[cut:]
            _emu_vs_oracle(data, [0, len(data)] if (d + L) % 2 else [0, cut, len(data)])


def test_emu_csv_fast_weight_column():
    """weight_column (csv_parser.h:113-114) on the single-pass CSV kernel,
    alone and with a label column: clean inputs stay on it; empty weights,
    short rows and the column forms where a row of special fields is fatal
    (weight column 0, {label, weight} = {0, 1}) go to the exact kernels --
    the reference's result (or error) either way."""
    rng = np.random.default_rng(9090)
    fast = 0
    combos = [(-1, 1), (-1, 3), (0, 2), (3, 1), (1, 4), (2, 0), (0, 1), (-1, 0)]
    for it in range(32):
        lc, wc = combos[it % len(combos)]
        nl = 400 if it % 8 == 7 else int(rng.integers(1, 40))
        data = fuzz_text.labeled_csv(rng, nl, int(rng.integers(max(lc, wc) + 2, max(lc, wc) + 12)), lc,
                                     defects=0.0 if it % 16 < 8 else 0.1, weight_col=wc)
        offs = fuzz_text.random_cuts(rng, data, 4)
        kw = dict(label_column=lc, weight_column=wc)
        o = po.parse_chunks(data, offs, fmt=po.CSV, **kw)
        h = pyemu.parse(data, offs, "csv", **kw)
        failed = check_fail(h, "csv", offs)
        assert (o["status"] != 0) == failed, (it, lc, wc, o["msg"], h["error"])
        if not failed:
            assert diff(h, o) == [], (it, lc, wc, diff(h, o))
        if it % 16 < 8 and it % 8 < 5:
            assert h["path"] == "fast", (it, lc, wc)
        fast += h["path"] == "fast"
    assert fast >= 10


def _one_based(rng, nlines, width, shift_rows=()):
    """libsvm rows with ids starting at 1 except for the rows in shift_rows,
    which hold a 0 id (a 0-based unit wherever they land)."""
    out = []
    for r in range(nlines):
        ids = sorted(set(int(x) for x in rng.integers(1, 4000, size=int(rng.integers(1, width)))))
        if r in shift_rows:
            ids = [0] + ids
        out.append("%d %s" % (r % 2, " ".join("%d:%.7g" % (i, rng.random()) for i in ids)))
    return ("\n".join(out) + "\n").encode()


@pytest.mark.parametrize("nthread", [1, 3])
def test_emu_fast_indexing_mode_auto(nthread):
    """indexing_mode=-1 on the single-pass path (libsvm_parser.h:165-171):
    per ParseBlock unit (chunk x FillData range) the ids drop by one when the
    unit holds ids, all > 0; units with a 0 id keep theirs.  1-based and
    0-based units side by side, multi-tile, both id widths."""
    rng = np.random.default_rng(5150 + nthread)
    for it in range(4):
        n = 400 if it < 2 else 40
        data = _one_based(rng, n, 50 if it < 2 else 8, shift_rows=set(rng.integers(0, n, size=it).tolist()))
        offs = fuzz_text.random_cuts(rng, data, 6)
        kw = {"indexing_mode": -1, "nthread": nthread, "index_bits": 64 if it % 2 else 32}
        h = _emu_vs_oracle(data, offs, **kw)
        assert h["path"] == "fast", it


def test_emu_fast_libfm_indexing_mode_auto():
    rng = np.random.default_rng(616)
    for it in range(3):
        rows = []
        for r in range(200):
            k = int(rng.integers(1, 12))
            lo = 0 if (it == 1 and r == 77) else 1
            rows.append("%d %s" % (r % 2, " ".join("%d:%d:%.6g" % (int(rng.integers(lo, 9)), int(rng.integers(lo, 500)),
                                                                     rng.random()) for _ in range(k))))
        data = ("\n".join(rows) + "\n").encode()
        offs = fuzz_text.random_cuts(rng, data, 4)
        o = po.parse_chunks(data, offs, fmt=po.LIBFM, indexing_mode=-1)
        h = pyemu.parse(data, offs, "libfm", indexing_mode=-1)
        assert h["error"] == 0 and o["status"] == 0 and h["path"] == "fast"
        assert diff(h, o) == [], diff(h, o)


@pytest.mark.parametrize("vt", ["f32", "i32", "i64"])
def test_emu_csv_fast_blanks_and_ints(vt):
    """Blanks around CSV values and integer DTypes on the single-pass CSV
    kernel (csv_fast.h): the token of a field is its first non-blank byte; a
    blank-only field is ParseFloat's 0 but strtoll's missing value; integer
    tokens need a digit after the sign (strtoll base 0: octal, saturation by
    the byte decoder).  Multi-tile and odd chunkings; violations (a blank
    field running into the next line) go to the exact kernels."""
    rng = np.random.default_rng({"f32": 31, "i32": 32, "i64": 33}[vt])
    paths = {"fast": 0, "exact": 0}
    vmap = {"f32": 0, "i32": 1, "i64": 2}
    for it in range(36):
        big = it % 6 == 5
        violate = (not big) and rng.random() < 0.3
        data = fuzz_text.blank_csv(rng, 1500 if big else int(rng.integers(1, 40)), 40 if big else 20,
                                   ints=vt != "f32" or rng.random() < 0.2, violate=violate)
        offs = fuzz_text.random_cuts(rng, data, 5, anywhere=it % 3 == 1)  # cuts inside blank runs too
        kw = {"value_type": vmap[vt]}
        if vt != "f32" and rng.random() < 0.3:
            kw["weight_column"] = int(rng.integers(0, 3))  # an ordinary column for integer DTypes
        okw = {("value_kind" if k == "value_type" else k): v for k, v in kw.items()}
        o = po.parse_chunks(data, offs, fmt=po.CSV, **okw)
        h = pyemu.parse(data, offs, "csv", **kw)
        failed = check_fail(h, "csv", offs)
        assert (o["status"] != 0) == failed, (it, data[:300], offs, o["msg"], h["error"])
        if not failed:
            assert diff(h, o) == [], (it, diff(h, o), data[:300])
        paths[h["path"]] += 1
    assert paths["fast"] >= 12, paths


def test_emu_csv_fast_text_fields():
    """Text in CSV float columns on the single-pass kernel (csv_fast.h
    csv_junk_byte): header rows, text columns, words and numbers followed by
    text -- a field starting with text holds no value, text after a number
    ends it; "nan" / "inf" / "f" fields are values (also after a sign or
    blanks), text after blanks a 0, a BOM at a row start skipped, "NaN(...)"
    a NaN or the reference's literal error (round 6: no longer the exact
    kernels).  Multi-tile, odd chunkings, both ',' and ' ' delimiters."""
    rng = np.random.default_rng(77)
    paths = {"fast": 0, "exact": 0}
    for it in range(40):
        big = it % 8 == 7
        violate = it % 5 == 4
        delim = " " if it % 7 == 3 else ","
        data = fuzz_text.junk_csv(rng, 1200 if big else int(rng.integers(1, 40)), 40 if big else 12, delim=delim,
                                  header=it % 2 == 0, violate=violate)
        offs = fuzz_text.random_cuts(rng, data, 5, anywhere=it % 3 == 1)
        kw = {"delimiter": delim}
        o = po.parse_chunks(data, offs, fmt=po.CSV, **kw)
        h = pyemu.parse(data, offs, "csv", **kw)
        failed = check_fail(h, "csv", offs)
        assert (o["status"] != 0) == failed, (it, data[:300], offs, o["msg"], h["error"])
        if not failed:
            assert diff(h, o) == [], (it, diff(h, o), data[:300])
        paths[h["path"]] += 1
        if delim == ",":
            assert h["path"] == "fast", (it, data[:300])
    assert paths["fast"] >= 20, paths


@pytest.mark.parametrize("vt", [0, 1, 2])
def test_emu_csv_chunk_cut_edges(vt):
    """Chunk cuts inside blank runs and between a sign and its digits: the
    decoders stop at the chunk end (the reference's chunk buffer), so a blank
    field reaching it, or a sign whose digit lies in the next chunk, must not
    borrow the next chunk's bytes."""
    cases = [(b"1,-5,2\n", [0, 3, 7]), (b"1,+7\n4\n", [0, 3, 8]), (b"1,  \n 2,3\n", [0, 3, 11]),
             (b"1, 2,3\n", [0, 3, 7]), (b"5, ,  6\n", [0, 4, 8]), (b"-\n9,1\n", [0, 1, 6]),
             (b"1|  |2\n", [0, 3, 7]), (b" 7, 8\n 9\n", [0, 1, 10]),
             # inf / nan tokens cut by the chunk end: the letters after it are
             # the next chunk's (ParseFloat reads NUL there)
             (b"1,inf\n2,3\n", [0, 3, 10]), (b"1,nan(2)\n2\n", [0, 5, 11]), (b"1,-inf\n2\n", [0, 4, 9]),
             (b"x,1\ni\rinfo,9\n", [0, 6, 14]), (b"1,infinity\n", [0, 8, 11])]
    for data, offs in cases:
        kw = {"value_type": vt}
        okw = {"value_kind": vt}
        o = po.parse_chunks(data, offs, fmt=po.CSV, delimiter="|" if b"|" in data else ",", **okw)
        h = pyemu.parse(data, offs, "csv", delimiter="|" if b"|" in data else ",", **kw)
        failed = check_fail(h, "csv", offs)
        assert (o["status"] != 0) == failed, (data, offs, o["msg"], h["error"])
        if not failed:
            assert diff(h, o) == [], (data, offs, diff(h, o))


def test_emu_exact_gaps_across_segments():
    """The exact libsvm kernels classify each run's gap from the segment's
    masks (libsvm_core.h Seg.rc / rh) and read the bytes only for a segment's
    first run: ':' / '#' / blanks at every offset against the 32-byte segment
    and 8 KiB window edges, on the exact path, equal the oracle."""
    rng = np.random.default_rng(2024)
    checked = 0
    for it in range(40):
        rows = []
        for r in range(int(rng.integers(20, 200))):
            parts = ["%d" % (r % 3)]
            for j in range(int(rng.integers(0, 12))):
                gap = " " * int(rng.integers(1, 4))
                # (index-only runs among valued ones fail the reference's GetBlock CHECK:
                # every 4th input has no values at all instead)
                colon = "" if it % 4 == 3 else str(rng.choice([":", " :", ": ", " : ", "  :"],
                                                             p=[0.7, 0.1, 0.1, 0.05, 0.05]))
                parts.append("%s%d%s%s" % (gap, int(rng.integers(0, 999)), colon,
                                           ("%.4g" % rng.random()) if colon else ""))
            if rng.random() < 0.15:
                parts.append(" # c %d:%d" % (r, r))
            rows.append("".join(parts))
        data = (" " * int(rng.integers(0, 33)) + "\n".join(rows) + "\n").encode()
        offs = [0, len(data)]
        o = po.parse_chunks(data, offs, fmt=po.LIBSVM)
        h = pyemu.parse(data, offs, "libsvm", exact=True, tile_bytes=int(rng.choice([0, 4096, 9000])))
        failed = check_fail(h, "libsvm", offs)
        assert (o["status"] != 0) == failed, (it, o["msg"], h["error"])
        if not failed:
            assert diff(h, o) == [], (it, diff(h, o))
        checked += not failed
    assert checked >= 30, checked


def test_emu_fast_dirty_lines_vs_oracle():
    """Lines holding bytes outside the grammar (svm_fast.h dirty_lines): file
    headers mid-chunk, words, symbols, inf / nan values, across and near tile
    ends, with odd chunkings, CRLF and lone-CR line ends, and long dirty lines (the exact kernels' case):
    the single pass takes the short ones line by line, the rest goes to the
    exact kernels -- whichever path runs, the reference's result."""
    rng = np.random.default_rng(3131)
    paths = {"fast": 0, "exact": 0}
    for it in range(30):
        data = fuzz_text.dirty_libsvm(rng, 70000 if it % 3 else 3000, rate=0.01 if it % 2 else 0.05,
                                      long_frac=0.3 if it % 5 == 4 else 0.0, near_tile_end=it % 3 == 1,
                                      eol=(b"\n", b"\r\n", b"\n", b"\r")[it % 4])
        offs = fuzz_text.random_cuts(rng, data, 5, anywhere=it % 4 == 3)
        kw = {"index_bits": 64} if it % 7 == 1 else ({"indexing_mode": -1} if it % 7 == 2 else {})
        h = _emu_vs_oracle(data, offs, **kw)
        paths[h["path"]] += 1
    assert paths["fast"] >= 8 and paths["exact"] >= 3, paths


def test_emu_fast_dirty_rows_stay_single_pass():
    """Rows carrying words, symbols, bytes >= 0x80, a ':' behind a non-blank
    byte, and inf / nan values and labels (fuzz_text.dirty_rows_libsvm) at
    1/8, 1/2 and every row, long rows across tile ends, CRLF / lone-CR line
    ends, odd chunkings, 64-bit ids and indexing_mode -1 / 1: the single pass
    keeps every input (svm_fast.h dirty_rewrite -- no line walk, no exact
    path) and its result is the reference's."""
    rng = np.random.default_rng(6061)
    for it in range(18):
        width = int(rng.integers(4, 90))
        data = fuzz_text.dirty_rows_libsvm(rng, max(4, 60000 // (width * 16 + 4)), width,
                                           rate=(0.125, 0.5, 1.0)[it % 3], eol=(b"\n", b"\r\n", b"\r")[it % 3 == 1 and 1 or (2 if it % 5 == 4 else 0)],
                                           near_tile_end=it % 2 == 1, runs=it % 3 == 2)
        offs = fuzz_text.random_cuts(rng, data, 4, anywhere=False)
        kw = {"index_bits": 64} if it % 4 == 1 else ({"indexing_mode": -1} if it % 4 == 2 else
                                                      ({"indexing_mode": 1} if it % 4 == 3 else {}))
        h = _emu_vs_oracle(data, offs, **kw)
        assert h["path"] == "fast", (it, kw)


def test_emu_fast_file_headers():
    """Files with a "# ..." first line concatenated the way InputSplit reads a
    directory ('\\n' between files, input_split_base.cc:204-210): headers
    without digitchars are empty lines to the reference and stay on the single
    pass, also when they sit across a 16 KiB tile end."""
    rng = np.random.default_rng(909)
    for it in range(12):
        files = []
        for f in range(6):
            body = fuzz_text.uniform_libsvm(rng, int(rng.integers(50, 400)), 20).replace(b"\r", b"\n")
            files.append(b"# synth libsvm shard\n" + body.rstrip(b"\n") + b"\n")
        data = b"\n".join(files) + b"\n"
        if it % 2:  # move a header across a tile end
            k = data.index(b"# synth", 16384 - 2000) if len(data) > 20000 else -1
            if k > 0:
                pad = 16384 - 10 - k
                if pad > 0:
                    data = data[:k - 1] + b" " * pad + data[k - 1:]
        offs = fuzz_text.random_cuts(rng, data, 4, anywhere=False)
        h = _emu_vs_oracle(data, offs)
        assert h["path"] == "fast", it


@pytest.mark.parametrize("form", ["valued", "mid_pair", "dangling", "long_head", "index_only"])
def test_emu_exact_rows_past_the_records(form):
    """Rows over 32 KiB crossing exact tile ends at tile_bytes=4096: the
    write pass runs past the count pass's three recorded windows per tile and
    restores the role state and pending token from rec_meta
    (libsvm_core.h:406) -- equal to the oracle."""
    rng = np.random.default_rng({"valued": 1, "mid_pair": 2, "dangling": 3, "long_head": 4, "index_only": 5}[form])
    for it in range(3):
        data = fuzz_text.long_row_libsvm(rng, form)
        offs = fuzz_text.random_cuts(rng, data, 2, anywhere=False)
        o = po.parse_chunks(data, offs, fmt=po.LIBSVM)
        h = pyemu.parse(data, offs, "libsvm", exact=True, tile_bytes=4096)
        failed = check_fail(h, "libsvm", offs)
        assert (o["status"] != 0) == failed, (form, it, o["msg"], h["error"])
        if not failed:
            assert diff(h, o) == [], (form, it, diff(h, o))


def test_emu_csv_exact_wide_rows_past_the_records():
    """The CSV write pass recounts windows past its records (csv_core.h:451):
    rows over 32 KiB at tile_bytes=4096 equal the oracle."""
    rng = np.random.default_rng(77)
    for it in range(4):
        data = fuzz_text.wide_row_csv(rng)
        offs = fuzz_text.random_cuts(rng, data, 2, anywhere=False)
        o = po.parse_chunks(data, offs, fmt=po.CSV)
        h = pyemu.parse(data, offs, "csv", exact=True, tile_bytes=4096)
        failed = check_fail(h, "csv", offs)
        assert (o["status"] != 0) == failed, (it, o["msg"], h["error"])
        if not failed:
            assert diff(h, o) == [], (it, diff(h, o))


def test_emu_libfm_exact_records_vs_oracle():
    """libfm exact kernels with the count pass's window records (round 6,
    libfm_core.h): lines ending in a dangling "f:i:" (ParseTriple decodes the
    value at the line end) among value lines; inputs without values whose
    lines end in a dangling "f:" (the index decoded at the line end); both
    kinds mixed -- then windows whose 32-byte segments hold both carry no
    record and are walked again, and the reference's offset / value CHECK
    fails, as it must here too -- plus '-' fields (the sign error even for a
    dropped triple); multi-window tiles at the default, 4 KiB and odd exact
    tiles, random chunk cuts."""
    rng = np.random.default_rng(606)
    checked = 0
    for it in range(18):
        kind = it % 3  # 0: values + "f:i:" ends, 1: no values + "f:" ends, 2: both + signs
        rows = []
        for _ in range(int(rng.integers(300, 2500))):
            r = rng.random()
            lab = int(rng.integers(0, 3))
            f, i = int(rng.integers(0, 50)), int(rng.integers(0, 900))
            if r < 0.15 and kind != 0:
                rows.append("%d %d:" % (lab, f))
            elif r < 0.3 and kind != 1:
                rows.append("%d %d:%d:" % (lab, f, i))
            elif r < 0.31 and kind == 2:
                rows.append("%d -3:4:5" % lab)
            else:
                fmt = "%d:%d" if kind == 1 else "%d:%d:%.4g"
                trips = [(fmt % ((rng.integers(0, 50), rng.integers(0, 900)) if kind == 1 else
                                 (rng.integers(0, 50), rng.integers(0, 900), rng.random())))
                         for _ in range(int(rng.integers(0, 6)))]
                if rng.random() < 0.2:
                    trips.append("%d" % rng.integers(0, 50))
                rows.append(" ".join(["%d" % lab] + trips))
        data = ("\n".join(rows) + "\n").encode()
        offs = fuzz_text.random_cuts(rng, data, 4)
        o = po.parse_chunks(data, offs, fmt=po.LIBFM)
        h = pyemu.parse(data, offs, "libfm", exact=True, tile_bytes=[0, 4096, 9000][(it // 3) % 3])
        failed = check_fail(h, "libfm", offs)
        assert (o["status"] != 0) == failed, (it, o["msg"], h["error"])
        if kind != 2:
            assert not failed, (it, o["msg"])
            assert diff(h, o) == [], (it, diff(h, o))
        else:
            # the reference fails the block's CHECK, so its arrays cannot pin the walked
            # windows: the same call without records (every window walked) must agree
            os.environ["EMU_NOREC"] = "1"
            try:
                h2 = pyemu.parse(data, offs, "libfm", exact=True, tile_bytes=[0, 4096, 9000][(it // 3) % 3])
            finally:
                os.environ.pop("EMU_NOREC", None)
            for k in ("offset", "label", "weight", "field", "index", "value", "chunk_table"):
                assert np.array_equal(h[k], h2[k]), (it, k)
            assert h["error"] == h2["error"], it
        checked += not failed
    assert checked >= 12, checked
