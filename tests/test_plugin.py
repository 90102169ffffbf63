"""The HIP parsers as a plugin of the UNMODIFIED reference.

oracle/_ref/host_api_test_ref is tests/cpp/host_api_test.cc compiled against
the reference's own headers and sources (src/data.cc registry, src/io
InputSplit) plus dmlc-core_amd/host/hip_plugin.cc, which registers
libsvm_hip / libfm_hip / csv_hip with DMLC_REGISTER_DATA_PARSER.  The GPU
tests call Parser<I,D>::Create(uri, part, nparts, "<fmt>_hip") and
RowBlockIter::Create through the reference's registry and compare every
array, every block's row count and NumCol with the reference's own CPU type
"<fmt>" run by the same binary on the same files (the unittest_inputsplit.cc
scenarios and synthetic multi-file, multi-part inputs).  The binary is built
in the build container (make -C oracle plugin) and travels to the GPU box.
"""
import os
import subprocess

import numpy as np
import pytest

from tools import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "oracle", "_ref", "host_api_test_ref")

pytestmark = pytest.mark.skipif(not os.path.exists(BIN), reason="make -C oracle plugin (needs /root/reference)")


def run(tmp_path, uri, fmt, part=0, nparts=1, index_bits=32, dtype="f32", iter_=False, tag="o"):
    o = str(tmp_path / tag)
    args = [BIN, uri, str(part), str(nparts), fmt, str(index_bits), dtype, o] + (["iter"] if iter_ else [])
    r = subprocess.run(args, capture_output=True, timeout=240)
    if r.returncode == 3:
        return {"error": open(o + ".error").read()}
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    it = np.uint64 if index_bits == 64 else np.uint32
    vt = {"f32": np.float32, "i32": np.int32, "i64": np.int64}[dtype]
    out = {}
    for k, t in (("offset", np.uint64), ("label", vt), ("weight", np.float32), ("qid", np.uint64),
                 ("index", it), ("value", vt), ("field", it), ("blocks", np.uint64), ("meta", np.uint64)):
        out[k] = np.fromfile(o + "." + k, t)
    return out


def same(a, b):
    if "error" in a or "error" in b:
        return ("error" in a) == ("error" in b)
    for k in ("offset", "label", "weight", "qid", "index", "value", "field", "blocks"):
        x, y = a[k], b[k]
        if x.dtype == np.float32:
            x, y = x.view(np.uint32), y.view(np.uint32)
        if not np.array_equal(x, y):
            return False
    return a["meta"][0] == b["meta"][0] and a["meta"][2] == b["meta"][2]


def write(d, files):
    d.mkdir(parents=True, exist_ok=True)
    for name, data in files.items():
        (d / name).write_bytes(data)
    return str(d)


def test_plugin_api_semantics_on_the_reference():
    """CPU: the C++ API checks of host_api_test.cc (RowBlock/Row CHECKs,
    MemCostBytes, a program-registered parser type) hold on the genuine
    reference -- the semantics this build's include/dmlc restates."""
    import tempfile
    text, _ = synth.rows(synth.LIBSVM, 2000, 30, seed=6)
    with tempfile.NamedTemporaryFile(suffix=".libsvm") as f:
        f.write(text.tobytes())
        f.flush()
        r = subprocess.run([BIN, "--api", f.name], capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr.decode()[-2000:]


@pytest.mark.gpu
def test_plugin_unittest_inputsplit_scenarios(tmp_path):
    """test/unittest_inputsplit.cc:41-147 through Parser::Create(..., "<fmt>_hip")
    in the reference's registry == the reference's own "<fmt>"."""
    cases = [
        ("csv", {"a.csv": b"0,1,2,3\n4,5,6,7\n", "b.csv": b"8,9,10,11\n12,13,14,15", "c.csv": b"16,17,18,19\n"}),
        ("libsvm", {"a.txt": b"1 1:1 2:2\n0 3:3\n1 4:4 5:5"}),
        ("libsvm", {"p%d" % i: b"".join(b"%d %d:1\n" % (j % 2, j) for j in range(2 * i, 2 * i + 2)) for i in range(5)}),
    ]
    for n, (fmt, files) in enumerate(cases):
        d = write(tmp_path / ("s%d" % n), files)
        for nparts in (1, 2):
            for part in range(nparts):
                ref = run(tmp_path, d, fmt, part, nparts, tag="r")
                hip = run(tmp_path, d, fmt + "_hip", part, nparts, tag="h")
                assert "error" not in ref and same(ref, hip), (n, part, nparts)


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", ["libsvm", "csv", "libfm"])
def test_plugin_synthetic_vs_reference(tmp_path, fmt):
    """Multi-file, multi-part synthetic inputs (several 8 MiB chunks for the
    big file), both index widths, Parser and RowBlockIter (NumCol)."""
    rng = np.random.default_rng({"libsvm": 1, "csv": 2, "libfm": 3}[fmt])
    if fmt == "libfm":
        import fuzz_text
        files = {"f%d" % i: fuzz_text.libfm_rows(rng, int(rng.integers(50, 3000)), 12) for i in range(3)}
    else:
        kind = synth.LIBSVM if fmt == "libsvm" else synth.CSV
        files = {"f%d" % i: synth.rows(kind, int(rng.integers(50, 4000)), 30, seed=i + 1)[0].tobytes()
                 for i in range(3)}
        big, _ = synth.rows(kind, 80000 if fmt == "libsvm" else 40000, 64, seed=9)
        files["big"] = big.tobytes()
    d = write(tmp_path / fmt, files)
    for bits in (32, 64):
        for nparts in (1, 3):
            for part in range(nparts):
                ref = run(tmp_path, d, fmt, part, nparts, index_bits=bits, tag="r")
                hip = run(tmp_path, d, fmt + "_hip", part, nparts, index_bits=bits, tag="h")
                assert "error" not in ref and same(ref, hip), (fmt, bits, part, nparts)
    if fmt == "csv":
        # the reference's BasicRowIter crashes on label-less CSV: Push copies
        # `size` labels from the block's NULL label pointer (row_block.h:128-130),
        # and RowBlockIter::Create drops the uri's ?label_column (data.cc:92-94)
        return
    ref = run(tmp_path, d, fmt, iter_=True, tag="r")
    hip = run(tmp_path, d, fmt + "_hip", iter_=True, tag="h")
    assert same(ref, hip) and ref["meta"][2] == hip["meta"][2] > 0


@pytest.mark.gpu
def test_plugin_args_auto_and_errors(tmp_path):
    """URI arguments, "auto" with format=<fmt>_hip, integer CSV DTypes, and a
    parse error surfacing as the reference's dmlc::Error."""
    d = write(tmp_path / "lab", {"x.csv": b"1,2,3\n4,5,6\n7,,9\n"})
    for dt in ("f32", "i32", "i64"):
        ref = run(tmp_path, d + "?label_column=0", "csv", dtype=dt, tag="r")
        hip = run(tmp_path, d + "?label_column=0", "csv_hip", dtype=dt, tag="h")
        assert same(ref, hip), dt
    ref = run(tmp_path, d + "?format=csv", "auto", tag="r")
    hip = run(tmp_path, d + "?format=csv_hip", "auto", tag="h")
    assert same(ref, hip)
    e = write(tmp_path / "neg", {"n.txt": b"1 3:1\n1 -3:1\n"})
    ref = run(tmp_path, e, "libsvm", tag="r")
    hip = run(tmp_path, e, "libsvm_hip", tag="h")
    assert "sign == true" in ref["error"] and "sign == true" in hip["error"]
    bad = run(tmp_path, d + "?bogus=1", "csv_hip", tag="h")
    assert "Cannot find argument" in bad["error"]


@pytest.mark.gpu
def test_disk_row_cache_pages_vs_reference(tmp_path):
    """uri#cachefile (DiskRowIter, disk_row_iter.h:40-137): the rows written
    once to 64 MB pages in RowBlockContainer::Save's format and read back.
    The reference's own "libsvm" type, the HIP parser as a plugin of the
    reference ("libsvm_hip"), and this build's drop-in API all write the same
    cache file byte for byte and iterate the same pages; an existing cache is
    reused without parsing."""
    from test_host_api import run_api
    text, _ = synth.rows(synth.LIBSVM, 100000, 128, seed=17)
    d = write(tmp_path / "cache_in", {"f0": text.tobytes()})
    caches = {k: str(tmp_path / ("%s.cache" % k)) for k in ("ref", "plugin", "dropin")}
    ref = run(tmp_path, d + "#" + caches["ref"], "libsvm", iter_=True, tag="r")
    plug = run(tmp_path, d + "#" + caches["plugin"], "libsvm_hip", iter_=True, tag="p")
    drop = run_api(tmp_path, d + "#" + caches["dropin"], iter_=True)
    raw = {k: open(v, "rb").read() for k, v in caches.items()}
    assert len(raw["ref"]) > 64 << 20 and raw["plugin"] == raw["ref"] and raw["dropin"] == raw["ref"]
    assert len(ref["blocks"]) >= 2  # pages
    assert same(ref, plug) and same(ref, drop)
    assert ref["meta"][2] == plug["meta"][2] == drop["meta"][2] > 0  # NumCol of a built cache
    again = run_api(tmp_path, d + "#" + caches["dropin"], iter_=True)  # reuse: no parse
    assert same(again, drop) and again["meta"][2] == drop["meta"][2]
    assert open(caches["dropin"], "rb").read() == raw["ref"]
