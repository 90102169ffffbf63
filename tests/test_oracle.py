"""The CPU oracle (oracle/dmlc_oracle.c) pinned against the reference's goldens."""
import hashlib
import os

import numpy as np
import pytest

from golden_util import FIELDS, dec, diff, load_cases, load_floats, load_json
from oracle import pyoracle as po
from tools import synth

CASES = load_cases()


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_matches_reference_block(case):
    got = po.parse_block(case["data_latin1"], **case["params"])
    if case["status"]:
        assert got["status"] != 0, "reference raised (%s) but oracle did not" % case["msg"]
        return
    assert got["status"] == 0, got["msg"]
    exp = {k: dec(v) for k, v in case["expect"].items()}
    assert diff(got, exp) == []


def test_oracle_parse_float_goldens():
    strs, bits, used = load_floats()
    bad = []
    for s, b, u in zip(strs, bits, used):
        v, n = po.parse_float(s)
        if np.float32(v).view(np.uint32) != b or n != u:
            bad.append((s, hex(int(b)), hex(int(np.float32(v).view(np.uint32))), u, n))
    assert not bad, bad[:10]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("name", ["libsvm_10k_x128", "csv_10k_x256"])
def test_oracle_synthetic_config1(name):
    g = load_json("synth_cfg1.json")[name]
    fmt = synth.LIBSVM if g["format"] == "libsvm" else synth.CSV
    text, _ = synth.rows(fmt, g["rows"], g["width"], seed=g["seed"])
    assert len(text) == g["input_bytes"] and sha(text) == g["input_sha256"]
    chunks = po.split_text([text.tobytes()])
    offs = np.cumsum([0] + [len(c) for c in chunks])
    got = po.parse_chunks(b"".join(chunks), offs, fmt=po.LIBSVM if fmt == synth.LIBSVM else po.CSV)
    assert got["status"] == 0
    for k, h in g["sha256"].items():
        assert sha(got[k]) == h, k


SPLIT = load_json("split.json")["cases"]


def _files_for(case, name_to_bytes):
    return [name_to_bytes[fn] for fn in case["order"]]


def _regen_files(case):
    out = {}
    for fn, txt in case["files"].items():
        if txt is not None:
            out[fn] = txt.encode("latin-1")
    if len(out) != len(case["files"]):  # big generated files: rebuild exactly as make_golden did
        big, _ = synth.rows(synth.LIBSVM, 12000, 64, seed=7)
        big = big.tobytes()
        if case["name"] == "big_multi_chunk":
            out = {"a.libsvm": big, "b.libsvm": big[: len(big) // 3] + b"\n\r\n" + b"7 1:2"}
        elif case["name"] == "crlf_boundaries":
            out = {"a.libsvm": b"1 1:1\r\n" * 5000 + b"\r\n\r\n", "b.libsvm": b"\n\n2 2:2\r\n" * 3000}
    for fn, h in case["file_sha256"].items():
        assert hashlib.sha256(out[fn]).hexdigest() == h
    return out


@pytest.mark.parametrize("case", SPLIT, ids=["%s-%d/%d" % (c["name"], c["part"], c["nparts"]) for c in SPLIT])
def test_oracle_input_split(case):
    files = _regen_files(case)
    chunks = po.split_text(_files_for(case, files), case["part"], case["nparts"])
    assert [len(c) for c in chunks] == case["chunk_sizes"]
    assert [hashlib.sha256(c).hexdigest() for c in chunks] == case["chunk_sha256"]
    offs = np.cumsum([0] + [len(c) for c in chunks])
    fmt = po.LIBSVM if case["format"] == "libsvm" else po.CSV
    got = po.parse_chunks(b"".join(chunks), offs, fmt=fmt)
    assert len(got["offset"]) - 1 == case["num_row"]
    ncol = int(got["index"].max()) + 1 if len(got["index"]) else 0
    assert ncol == case["num_col"]
    for k, h in case["sha256"].items():
        assert sha(got[k]) == h, k


# ---- live cross-check against the genuine reference (build container only) ----

def _fuzz_line(rng, fmt):
    alpha = {po.LIBSVM: list("0123456789") * 6 + list(" :.-+eE#\tq") + ["qid:", "nan", "inf", "\r"],
             po.CSV: list("0123456789") * 6 + list(",,,,.-+eE \t") + ["nan", "inf", "0x", "\xef\xbb\xbf"],
             po.LIBFM: list("0123456789") * 6 + list(" ::.-+e#")}[fmt]
    n = int(rng.integers(0, 40))
    return "".join(alpha[int(i)] for i in rng.integers(0, len(alpha), n))


@pytest.mark.skipif(not po.ref_available(), reason="oracle/_ref not built (needs /root/reference)")
@pytest.mark.parametrize("fmt", [po.LIBSVM, po.CSV, po.LIBFM])
def test_oracle_fuzz_vs_reference(fmt):
    rng = np.random.default_rng(1000 + fmt)
    for it in range(400):
        text = "\n".join(_fuzz_line(rng, fmt) for _ in range(int(rng.integers(1, 6))))
        if rng.random() < 0.5:
            text += "\n"
        kw = {"fmt": fmt}
        if fmt == po.CSV and rng.random() < 0.3:
            kw["label_column"] = int(rng.integers(0, 3))
        if fmt == po.LIBSVM and rng.random() < 0.3:
            kw["indexing_mode"] = int(rng.integers(-1, 2))
        r = po.ref_parse_block(text, **kw)
        o = po.parse_block(text, **kw)
        assert (r["status"] != 0) == (o["status"] != 0), (text, r["msg"], o["msg"])
        if r["status"] == 0:
            assert diff(o, r) == [], repr(text)


# ---- FillData's nthread range split (text_parser.h:116-155) ----

FILLDATA = load_json("filldata.json")


@pytest.mark.parametrize("case", FILLDATA, ids=[c["name"] for c in FILLDATA])
def test_oracle_filldata_goldens(case):
    """The oracle's range split (dmo_parse_chunk with nthread) against the
    genuine reference's ParseNext: arrays, errors and per-block counts."""
    got = po.parse_chunks(case["data_latin1"], case["offs"], **case["params"])
    assert (got["status"] != 0) == bool(case["status"]), (got["msg"], case["msg"])
    if case["status"]:
        return
    exp = {k: dec(v) for k, v in case["expect"].items()}
    assert diff(got, exp) == []
    for k in ("rows", "index", "value"):
        assert got["blocks"][k].tolist() == case["blocks"][k], k


@pytest.mark.skipif(not po.ref_available(), reason="oracle/_ref not built (needs /root/reference)")
@pytest.mark.parametrize("fmt", [po.LIBSVM, po.CSV, po.LIBFM])
def test_oracle_filldata_fuzz_vs_reference(fmt):
    """Live: oracle == reference ParseNext for nthread 2..4 on multi-chunk input."""
    rng = np.random.default_rng(77 + fmt)
    for it in range(150):
        text = ("\n".join(_fuzz_line(rng, fmt) for _ in range(int(rng.integers(1, 9)))) + "\n").encode("latin-1")
        nl = [i + 1 for i, b in enumerate(text) if b == 10 and i + 1 < len(text)]
        cuts = sorted(set(rng.choice(nl, size=min(len(nl), int(rng.integers(0, 3))), replace=False).tolist())) if nl else []
        offs = [0] + cuts + [len(text)]
        kw = {"fmt": fmt, "nthread": int(rng.integers(2, 5))}
        if fmt != po.CSV:
            kw["indexing_mode"] = int(rng.integers(-1, 2))
        r = po.ref_parse_chunks(text, offs, **kw)
        o = po.parse_chunks(text, offs, **kw)
        assert (r["status"] != 0) == (o["status"] != 0), (text, kw, r["msg"], o["msg"])
        if r["status"] == 0:
            assert diff(o, r) == [], (text, kw)
            assert o["blocks"]["rows"].tolist() == r["blocks"]["rows"].tolist()


@pytest.mark.skipif(not po.ref_available(), reason="oracle/_ref not built (needs /root/reference)")
def test_oracle_csv_text_fields_vs_reference():
    """Live: CSV text fields (header words, text columns, "3.5kg", "feature",
    "-f", "name", "inf", "NaN(1)", text after blanks) -- what ParseFloat
    consumes of them (strtonum.h:95-264) -- oracle == the genuine reference."""
    import fuzz_text
    rng = np.random.default_rng(4040)
    for it in range(300):
        delim = ",;\t|"[it % 4]
        text = fuzz_text.junk_csv(rng, int(rng.integers(1, 12)), 10, delim=delim, header=it % 3 != 0,
                                  violate=it % 2 == 1).decode("latin-1")
        kw = {"fmt": po.CSV, "delimiter": delim}
        r = po.ref_parse_block(text, **kw)
        o = po.parse_block(text, **kw)
        assert (r["status"] != 0) == (o["status"] != 0), (text, r["msg"], o["msg"])
        if r["status"] == 0:
            assert diff(o, r) == [], repr(text)
