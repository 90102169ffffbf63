#!/usr/bin/env python3
"""Generate tests/golden/* from the GENUINE reference (oracle/_ref/libdmlc_ref.so).

Run in the build container (where /root/reference exists):
    make -C oracle ref && python tests/golden/make_golden.py

Outputs (data only -- inputs and the reference's outputs, no reference source):
  cases.json     every known-answer case of test/unittest_parser.cc, restated as
                 inputs, plus the Appendix-A quirk corpus of SURVEY.md; expected
                 arrays are what the reference's ParseBlock produced.
  floats.npz     ParseFloat goldens: strings -> (fp32 bits, bytes consumed).
  synth_cfg1.json BASELINE config 1 (10k x 128 libsvm, 10k x 256 csv) through
                 Parser<uint32_t>::Create on a real file: per-array SHA-256 and
                 the first/last 64 rows in full.
  split.json     InputSplit("text") chunk sizes/hashes and multi-part row counts.
  filldata.json  TextParserBase::FillData with nthread = 1..4 ranges per chunk
                 (text_parser.h:116-155) over multi-chunk inputs: every array
                 plus the per-block row/index/value counts the reference's
                 ParserImpl::Next hands out (one block per non-empty range).
"""
import hashlib
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import pyoracle as po  # noqa: E402
from tools import synth  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def enc(a):
    a = np.asarray(a)
    if a.dtype == np.float32:
        return {"dtype": "f32bits", "data": a.view(np.uint32).tolist()}
    return {"dtype": str(a.dtype), "data": a.tolist()}


QID_DATA = """3 qid:1 1:1 2:1 3:0 4:0.2 5:0
                           2 qid:1 1:0 2:0 3:1 4:0.1 5:1
                           1 qid:1 1:0 2:1 3:0 4:0.4 5:0
                           1 qid:1 1:0 2:0 3:1 4:0.3 5:0
                           1 qid:2 1:0 2:0 3:1 4:0.2 5:0
                           2 qid:2 1:1 2:0 3:1 4:0.4 5:0
                           1 qid:2 1:0 2:0 3:1 4:0.1 5:0
                           1 qid:2 1:0 2:0 3:1 4:0.2 5:0
                           2 qid:3 1:0 2:0 3:1 4:0.1 5:1
                           3 qid:3 1:1 2:1 3:0 4:0.3 5:0
                           4 qid:3 1:1 2:0 3:0 4:0.4 5:1
                           1 qid:3 1:0 2:1 3:1 4:0.5 5:0"""
QID_COMMENT = """# what does foo bar mean anyway
                           3 qid:1 1:1 2:1 3:0 4:0.2 5:0 # foo
                           2 qid:1 1:0 2:0 3:1 4:0.1 5:1
                           1 qid:1 1:0 2:1 3:0 4:0.4 5:0
                           1 qid:1 1:0 2:0 3:1 4:0.3 5:0
                           1 qid:2 1:0 2:0 3:1 4:0.2 5:0 # bar
                           2 qid:2 1:1 2:0 3:1 4:0.4 5:0
                           1 qid:2 1:0 2:0 3:1 4:0.1 5:0
                           1 qid:2 1:0 2:0 3:1 4:0.2 5:0
                           2 qid:3 1:0 2:0 3:1 4:0.1 5:1
                           3 qid:3 1:1 2:1 3:0 4:0.3 5:0
                           4 qid:3 1:1 2:0 3:0 4:0.4 5:1
                           1 qid:3 1:0 2:1 3:1 4:0.5 5:0"""
IDX4 = "1 1:1 2:-1\n0 1:-1 2:1\n1 1:-1 2:-1\n0 1:1 2:1\n"


def cases():
    L, C, F = po.LIBSVM, po.CSV, po.LIBFM
    c = []
    # ---- test/unittest_parser.cc known answers (inputs restated verbatim) ----
    c += [
        ("ut_csv_ignore_bom_a", C, "\xEF\xBB\xBF\x31\n\xEF\xBB\x32\n", {}),
        ("ut_csv_ignore_bom_b", C, "\xEF\xBB\xBF\x31\n\xEF\xBB\xBF\x32\n", {}),
        ("ut_csv_standard", C, "0,1,2,3\n4,5,6,7\n8,9,10,11\n", {}),
        ("ut_csv_missing_values", C, "0,,,3\n4,5,6,7\n8,9,10,11\n", {}),
        ("ut_csv_int32", C, "20000000,20000001,20000002,20000003\n20000004,20000005,20000006,20000007\n"
         "20000008,20000009,20000010,20000011\n", {"value_kind": po.I32}),
        ("ut_csv_int64", C, "2147483648,2147483649,2147483650,2147483651\n2147483652,2147483653,"
         "2147483654,2147483655\n2147483656,2147483657,2147483658,2147483659\n", {"value_kind": po.I64}),
        ("ut_csv_crlf", C, "0,1,2,3\r\n4,5,6,7\r\n8,9,10,11\r\n", {}),
        ("ut_csv_noeol", C, "0,1,2,3\r\n4,5,6,7\r\n8,9,10,11", {}),
        ("ut_csv_delimiter_space", C, "0 1 2 3\n4 5 6 7\n8 9 10 11", {"delimiter": " "}),
        ("ut_csv_weight_column", C, "0,1,2,3\n4,5,6,7\n8,9,10,11", {"weight_column": 2}),
        ("ut_csv_weight_column_2", C, "0,1,2,3\n4,5,6,7\n8,9,10,11", {}),
        ("ut_libsvm_qid", L, QID_DATA, {}),
        ("ut_libsvm_qid_comment", L, QID_COMMENT, {}),
        ("ut_libsvm_excess_digits", L, "0 1:17.065995780200002000000 4:17.0659957802 "
         "6:0.00017065995780200002 8:0.000170659957802\n", {}),
        ("ut_libsvm_index0", L, IDX4, {}),
        ("ut_libsvm_index1", L, IDX4, {"indexing_mode": 1}),
        ("ut_libsvm_index_auto", L, IDX4, {"indexing_mode": -1}),
        ("ut_libsvm_index_auto2", L, "1 1:1 2:-1\n0 0:-2 1:-1 2:1\n1 1:-1 2:-1\n0 1:1 2:1\n",
         {"indexing_mode": -1}),
        ("ut_libfm_index0", F, "1 1:1:1 1:2:-1\n0 1:1:-1 2:2:1\n1 2:1:-1 1:2:-1\n0 2:1:1 2:2:1\n", {}),
        ("ut_libfm_index1", F, "1 1:1:1 1:2:-1\n0 1:1:-1 2:2:1\n1 2:1:-1 1:2:-1\n0 2:1:1 2:2:1\n",
         {"indexing_mode": 1}),
        ("ut_libfm_index_auto", F, "1 1:1:1 1:2:-1\n0 1:1:-1 2:2:1\n1 2:1:-1 1:2:-1\n0 2:1:1 2:2:1\n",
         {"indexing_mode": -1}),
        ("ut_libfm_index_auto2", F, "1 1:1:1 1:2:-1\n0 0:0:-2 1:1:-1 2:2:1\n1 2:1:-1 1:2:-1\n0 2:1:1 2:2:1\n",
         {"indexing_mode": -1}),
    ]
    # ---- SURVEY.md Appendix A quirk corpus: libsvm ----
    q = [
        ("q_l0_comment", "# comment\n1 2:3\n"),
        ("q_later_comment_line", "1 2:3\n# comment\n"),
        ("q_later_hash_label", "1 1:1\n#7 comment e5\n"),
        ("q_blank_then_comment", "   # x 1:2\n3 4:5\n"),
        ("q_weight", "1:0.5 2:3\n0:2 1:1\n"),
        ("q_qid_tab", "1\tqid:3 2:1\n"),
        ("q_qid_after_weight_tab", "1:0.5\tqid:3 2:1\n"),
        ("q_qid_after_weight_space", "1:0.5 qid:3 2:1\n"),
        ("q_qid_space_value", "1 qid: 5 2:1\n"),
        ("q_qid_negative", "1 qid:-5 2:1\n"),
        ("q_qid_saturate", "1 qid:99999999999999999999 1:1\n0 qid:-99999999999999999999 1:1\n"),
        ("q_qid_hash", "1 qid:#x 1:1\n"),
        ("q_qid_newline", "1 qid:\n2 1:1\n"),
        ("q_qid_exp", "1 qid:5e3 1:1\n"),
        ("q_dangling_colon", "1 3:\n2 4:5\n"),
        ("q_dangling_label_colon", "1:\n3 1:1\n"),
        ("q_dangling_colon_comment", "1 3: # x\n4 5:6\n"),
        ("q_inline_comment", "1 1:2 # foo 3:4\n"),
        ("q_inline_not_comment", "1 1:2 x# 3:4\n"),
        ("q_glued_comment", "1 1:2#3:4\n"),
        ("q_chain", "1:2:3 4:5 6\n"),
        ("q_chain_long", "1 1:2:3:4:5 7:8\n"),
        ("q_sign_only", "1 1:-inf 2:+inf 3:nan 4:- 5:+ 6:-Infinity 7:NaN 8:+.\n"),
        ("q_skip_nondigit", "1 2:nan 3:1e3\n"),
        ("q_index_wrap32", "1 4294967297:1 3.7:2 +5:3 e7:4\n"),
        ("q_crlf", "1 1:1\r\n2 2:2\r\n"),
        ("q_blank_lines", "\n\n1 1:1\n   \n\t\n2 2:2"),
        ("q_noeol", "1 1:1\n2 2:2"),
        ("q_float_edges", "1 1:1e39 2:3.4028235e38 3:1e-45 4:123456789012345678901234 "
         "5:0.00000000000000000000001 6:1e-38 7:3.402823466e38 8:1.17549e-38 9:7e-39\n"),
        ("q_nan_paren", "1 1:nan(abc_1) 2:3\n"),
        ("q_formfeed", "1 1:\f2 3:\v4\n"),
        ("q_high_bytes", "1 1:\xff2 \xc3\xa93:4\n"),
        ("q_spaces_everywhere", "  1   1 :  2    3:4  \n"),
        ("q_label_only", "1\n2\n3 1:1\n"),
        ("q_many_colons", "1 ::2 3::4\n"),
        ("q_exponent_wrap", "1 1:1e4294967297 2:1e-4294967298\n"),
        ("q_long_fraction", "1 1:0.12345678901234567890123 2:99999999999999999999.5\n"),
        ("q_tabs", "1\t1:2\t3:4\n"),
        ("q_cr_only", "1 1:1\r2 2:2\r"),
        ("q_only_newlines", "\n\r\n"),
        ("q_empty", ""),
    ]
    c += [(n, L, d, {}) for n, d in q]
    c += [
        ("q_index64_wrap", L, "1 18446744073709551617:1 18446744073709551615:2\n", {"index_bits": 64}),
        ("q_auto_zero_block", L, "1 0:1\n2 3:4\n", {"indexing_mode": -1}),
        ("q_auto_positive", L, "1 5:1\n2 3:4\n", {"indexing_mode": -1}),
        ("q_mode1_zero_wrap", L, "1 0:1\n", {"indexing_mode": 1}),
        ("q_err_negative_index", L, "1 -3:1\n", {}),
        ("q_err_mixed_values", L, "1 1:1 2\n", {}),
        ("q_err_nan_paren", L, "1 1:nan(abc 2:3\n", {}),
    ]
    # ---- Appendix A.2 quirk corpus: csv ----
    cq = [
        ("c_ws_field_eol", "1,2, \n3,4\n", {}),
        ("c_ws_field_mid", "1,  ,2\n", {}),
        ("c_sign_dot_e", "1,-,3\n1,.,e5\n", {}),
        ("c_label0", "1,2,3\n4,5,6\n", {"label_column": 0}),
        ("c_label_last", "1,2,3\n4,5,6\n", {"label_column": 2}),
        ("c_label_weight", "1,0.5,2,3\n4,2,5,6\n", {"label_column": 0, "weight_column": 1}),
        ("c_weight_nan_err", "1,nan,2\n3,4,5\n", {"weight_column": 1}),
        ("c_label_missing_err", "1,2,3\n4\n", {"label_column": 2}),
        ("c_delim_not_found_err", "5\n", {"label_column": 0}),
        ("c_int_prefixes", "0x10,010,-5,+7, 12 ,0x,08,0X1f\n", {"value_kind": po.I32}),
        ("c_int_prefixes64", "0x10,010,-5,+7, 12 ,0x,08,0X1f\n", {"value_kind": po.I64}),
        ("c_int_overflow64", "99999999999999999999,-99999999999999999999,9223372036854775808\n",
         {"value_kind": po.I64}),
        ("c_int_trunc32", "4294967297,-2147483649,2147483648\n", {"value_kind": po.I32}),
        ("c_int_label", "7,1,2\n8,3,4\n", {"value_kind": po.I32, "label_column": 0}),
        ("c_int_weightcol_is_value", "7,1,2\n8,3,4\n", {"value_kind": po.I64, "weight_column": 1}),
        ("c_bom_only_line", "\xEF\xBB\xBF\n1,2\n", {}),
        ("c_tab", "1\t2\t3\n4\t5\t6\n", {"delimiter": "\t"}),
        ("c_semicolon", "1;2;3\n4;;6\n", {"delimiter": ";"}),
        ("c_empty_lines", "1,2\n\n\n3,4\n\r\n5,6", {}),
        ("c_cr_mix", "\r\r\n1,2\r\r3,4\n", {}),
        ("c_trailing_delim", "1,2,\n3,4,\n", {}),
        ("c_space_double", "1  2 3\n4 5  6\n", {"delimiter": " "}),
        ("c_junk_fields", "abc,1,x2,3y\n", {}),
        ("c_inf_nan", "inf,-inf,nan,NAN(x),-0\n", {}),
        ("c_float_edges", "1e39,3.4028235e38,1e-45,0.1,1e-38\n", {}),
        ("c_index64", "1,2,3\n", {"index_bits": 64}),
        ("c_only_newlines", "\n\n\r\n", {}),
    ]
    c += [(n, C, d, kw) for n, d, kw in cq]
    fq = [
        ("f_pair_only", "1 1:2 3:4:5\n"),
        ("f_single", "1 1 2:3:4\n"),
        ("f_weight", "1:2 1:2:3\n"),
        ("f_comment_not_special", "# x\n1 1:2:3\n"),
    ]
    c += [(n, F, d, {}) for n, d in fq]
    return c


def gen_cases():
    out = []
    for name, fmt, data, kw in cases():
        kw = dict(kw)
        kw["fmt"] = fmt
        r = po.ref_parse_block(data, **kw)
        rec = {"name": name, "data_latin1": data, "params": kw, "status": int(r["status"] != 0),
               "msg": r["msg"]}
        if r["status"] == 0:
            rec["expect"] = {k: enc(r[k]) for k in ("offset", "label", "weight", "qid", "field",
                                                      "index", "value")}
        out.append(rec)
    with open(os.path.join(OUT, "cases.json"), "w") as f:
        json.dump(out, f, indent=0)
    print("cases.json:", len(out), "cases,", sum(r["status"] for r in out), "error cases")


def gen_floats():
    rng = np.random.default_rng(12345)
    strs = []
    bits = rng.integers(0, 2 ** 32, size=6000, dtype=np.uint64).astype(np.uint32)
    fl = bits.view(np.float32)
    strs += ["%.9g" % float(x) for x in fl if np.isfinite(x)]
    strs += ["%.6g" % float(x) for x in fl[:2000] if np.isfinite(x)]
    for _ in range(6000):  # fixed notation, 1..25 digits
        ni, nf = int(rng.integers(0, 12)), int(rng.integers(0, 25))
        s = "".join(str(int(d)) for d in rng.integers(0, 10, ni)) or "0"
        if nf:
            s += "." + "".join(str(int(d)) for d in rng.integers(0, 10, nf))
        if rng.random() < 0.3:
            s = "-" + s
        if rng.random() < 0.2:
            s += "e%+d" % int(rng.integers(-45, 45))
        strs.append(s)
    u = rng.random(4000, dtype=np.float32)
    strs += ["%.9g" % float(x) for x in u]
    strs += ["%.9g" % float(x) for x in (u * 2 - 1)]
    strs += ["0", "-0", "+0", ".5", "5.", "1e", "1e+", "-e", "+", "-", ".", "e", "E5", "1E5",
             "inf", "-INF", "Infinity", "-infinity", "infinit", "nan", "NaN", "nan(1_a)",
             "3.4028235e38", "3.402823466e38", "3.4028235e+38", "1e38", "1e39", "1e-38", "1e-39",
             "1e-45", "1e-46", "1.17549435e-38", "1.175494351e-38", "1.175494350e-38",
             "123456789012345678901234", "18446744073709551615", "18446744073709551616",
             "0.99999999999999999999999", "9.999999999999999999999e37", "1.5f", "2F", "  7",
             "\t\n8", "0x10", "1,5", "1.2.3", "1e5e3", "12-3", "--1", "+-1"]
    vals, used = [], []
    for s in strs:
        v, n = po.ref_parse_float(s)
        vals.append(np.float32(v).view(np.uint32))
        used.append(n)
    np.savez_compressed(os.path.join(OUT, "floats.npz"),
                        text=np.frombuffer("\0".join(strs).encode("latin-1"), dtype=np.uint8),
                        bits=np.array(vals, dtype=np.uint32), used=np.array(used, dtype=np.int32))
    print("floats.npz:", len(strs), "strings")


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def gen_synth():
    res = {}
    with tempfile.TemporaryDirectory(dir="/dev/shm" if os.path.isdir("/dev/shm") else None) as td:
        for name, fmt, rows, width, ptype in (("libsvm_10k_x128", synth.LIBSVM, 10000, 128, "libsvm"),
                                              ("csv_10k_x256", synth.CSV, 10000, 256, "csv")):
            text, _ = synth.rows(fmt, rows, width, seed=1)
            path = os.path.join(td, name + "." + ptype)
            with open(path, "wb") as f:
                f.write(text.tobytes())
            r = po.ref_parse_uri(path, 0, 1, ptype)
            assert r["status"] == 0, r["msg"]
            n = len(r["label"])
            o = r["offset"]
            head = {k: enc(r[k][: int(o[64])] if k in ("index", "value") else r[k][:65 if k == "offset" else 64])
                    for k in ("offset", "label", "index", "value")}
            tail_i0 = int(o[n - 64])
            tail = {"offset": enc(r["offset"][n - 64:]), "label": enc(r["label"][n - 64:]),
                    "index": enc(r["index"][tail_i0:]), "value": enc(r["value"][tail_i0:])}
            res[name] = {
                "format": ptype, "rows": rows, "width": width, "seed": 1,
                "input_bytes": int(len(text)), "input_sha256": sha(text),
                "sha256": {k: sha(r[k]) for k in ("offset", "label", "weight", "qid", "index", "value")},
                "sizes": {k: int(len(r[k])) for k in ("offset", "label", "weight", "qid", "index", "value")},
                "head": head, "tail": tail,
            }
    with open(os.path.join(OUT, "synth_cfg1.json"), "w") as f:
        json.dump(res, f, indent=0)
    print("synth_cfg1.json written")


def gen_split():
    res = {"cases": []}
    line = ("1 3:1 10:1 11:1 21:1 30:1 34:1 36:1 40:1 41:1 53:1 58:1 65:1 69:1 "
            "77:1 86:1 88:1 92:1 95:1 102:1 105:1 117:1 124:1")
    big, _ = synth.rows(synth.LIBSVM, 12000, 64, seed=7)  # ~12 MB -> 2 chunks of 8 MiB
    big = big.tobytes()
    setups = {
        # unittest_inputsplit.cc:41-147, restated as files
        "csv_noeol": ({"train_0.csv": b"0,1,1,1", "train_1.csv": b"0,1,1,2\n", "train_2.csv": b"0,1,1,2\n"},
                      "csv", [1]),
        "libsvm_noeol": ({"train_0.libsvm": (line + "\n").encode(), "train_1.libsvm": line.encode()},
                         "libsvm", [1]),
        "libsvm_5files": ({"test_%d.libsvm" % i: (line + "\n").encode() for i in range(5)}, "libsvm", [1]),
        "libsvm_distributed": ({"test_%d.libsvm" % i: ((line + "\n") * (6 if i == 0 else 1)).encode()
                                for i in range(5)}, "libsvm", [2]),
        "big_multi_chunk": ({"a.libsvm": big, "b.libsvm": big[: len(big) // 3] + b"\n\r\n" + b"7 1:2"},
                            "libsvm", [1, 2, 3]),
        "crlf_boundaries": ({"a.libsvm": b"1 1:1\r\n" * 5000 + b"\r\n\r\n", "b.libsvm": b"\n\n2 2:2\r\n" * 3000},
                            "libsvm", [1, 2, 5]),
    }
    with tempfile.TemporaryDirectory() as td:
        for name, (files, ptype, nparts_list) in setups.items():
            d = os.path.join(td, name)
            os.makedirs(d)
            for fn in sorted(files):
                with open(os.path.join(d, fn), "wb") as f:
                    f.write(files[fn])
            # listing order the reference used (readdir order) is recorded explicitly
            for nparts in nparts_list:
                for part in range(nparts):
                    chunks = po.ref_split_chunks(d, part, nparts)
                    r = po.ref_parse_uri(d, part, nparts, ptype)
                    ncol = int(r["index"].max()) + 1 if len(r["index"]) else 0
                    res["cases"].append({
                        "name": name, "format": ptype, "part": part, "nparts": nparts,
                        "order": [x for x in os.listdir(d)],
                        "files": {fn: files[fn].decode("latin-1") if len(files[fn]) < 4096 else None
                                  for fn in files},
                        "file_sha256": {fn: hashlib.sha256(files[fn]).hexdigest() for fn in files},
                        "chunk_sizes": [len(c) for c in chunks],
                        "chunk_sha256": [hashlib.sha256(c).hexdigest() for c in chunks],
                        "num_row": int(len(r["offset"]) - 1), "num_col": ncol,
                        "sha256": {k: sha(r[k]) for k in ("offset", "label", "index", "value")},
                    })
    with open(os.path.join(OUT, "split.json"), "w") as f:
        json.dump(res, f, indent=0)
    print("split.json:", len(res["cases"]), "cases")


def _fd_text(rng, fmt):
    alpha = {po.LIBSVM: list("0123456789") * 6 + list("  ::.-+eE#\t") + ["qid:", "\r", " 0:1", " 1:2"],
             po.CSV: list("0123456789") * 6 + list(",,,,.-+eE \t") + ["nan", "\xef\xbb\xbf"],
             po.LIBFM: list("0123456789") * 6 + list("  :::.-+eE#\t") + ["\r", " 0:0:1", " 1:1:1"]}[fmt]

    def structured():
        if fmt == po.CSV:
            return ",".join("%.4g" % rng.random() if rng.random() < 0.9 else "" for _ in range(int(rng.integers(1, 8))))
        toks = ["%d" % rng.integers(0, 2)]
        if fmt == po.LIBSVM and rng.random() < 0.2:
            toks.append("qid:%d" % rng.integers(0, 9))
        for _ in range(int(rng.integers(0, 8))):
            v = "%.3g" % rng.random()
            i = int(rng.integers(0, 20))
            toks.append("%d:%s" % (i, v) if fmt == po.LIBSVM else "%d:%d:%s" % (rng.integers(0, 4), i, v))
        line = " ".join(toks)
        if rng.random() < 0.15:
            line += " # c"
        return line

    lines = []
    for _ in range(int(rng.integers(1, 14))):
        if rng.random() < 0.7:
            lines.append(structured())
        else:
            lines.append("".join(alpha[int(i)] for i in rng.integers(0, len(alpha), int(rng.integers(0, 50)))))
    return ("\n".join(lines) + "\n").encode("latin-1")


def _fd_chunks(rng, data):
    nl = [i + 1 for i, b in enumerate(data) if b in (10, 13) and i + 1 < len(data)]
    k = int(rng.integers(0, min(4, len(nl)) + 1)) if nl else 0
    cuts = sorted(set(rng.choice(nl, size=k, replace=False).tolist())) if k else []
    return [0] + cuts + [len(data)]


def gen_filldata():
    """FillData range-split goldens (the reference's ParseNext with nthread
    ranges per chunk; DMLC_REF_NPROCS lifts its omp_get_num_procs cap)."""
    rng = np.random.default_rng(20261016)
    L, C, F = po.LIBSVM, po.CSV, po.LIBFM
    fixed = [
        # min index per range decides the 1-based shift (libsvm_parser.h:165-171)
        ("zero_in_first_half", L, b"1 0:1 2:3\n0 5:1\n1 1:2 7:1\n0 3:4\n", -1),
        ("zero_in_second_half", L, b"1 1:1 2:3\n0 5:1\n1 0:2 7:1\n0 3:4\n", -1),
        ("tiny_chunk_empty_ranges", L, b"1 1:1\n", -1),
        ("qid_newline_at_cut", L, b"1 qid:\n7 3:1\n0 qid:\n9 2:2\n", 0),
        ("comment_first_line", L, b"# head\n1 1:1\n0 2:2 # tail\n1 3:3\n", -1),
        ("libfm_dangling_at_cut", F, b"1 1:2:3 4:\n5:6 7:8:9\n0 2:\n3:1:1\n", -1),
        ("libfm_zero_field", F, b"1 0:1:1 2:2:2\n0 3:3:3\n1 1:1:1\n0 2:2:2\n", -1),
        ("csv_blank_field_at_cut", C, b"1,2, \n\n3,4\n5, \n6,7\n", 0),
    ]
    out = []

    def record(name, fmt, data, offs, nthread, kw):
        kw = dict(kw, fmt=fmt, nthread=nthread)
        r = po.ref_parse_chunks(data, offs, **kw)
        rec = {"name": name, "data_latin1": data.decode("latin-1"), "offs": [int(x) for x in offs],
               "params": kw, "status": int(r["status"] != 0), "msg": r["msg"]}
        if r["status"] == 0:
            rec["expect"] = {k: enc(r[k]) for k in ("offset", "label", "weight", "qid", "field",
                                                      "index", "value")}
            rec["blocks"] = {k: [int(x) for x in r["blocks"][k]] for k in ("rows", "index", "value")}
        out.append(rec)

    for name, fmt, data, im in fixed:
        for nt in (1, 2, 3, 4):
            kw = {} if fmt == C else {"indexing_mode": im}
            record("%s_t%d" % (name, nt), fmt, data, [0, len(data)], nt, kw)
    for it in range(150):
        fmt = (L, C, F)[it % 3]
        data = _fd_text(rng, fmt)
        offs = _fd_chunks(rng, data)
        kw = {}
        if fmt != C:
            kw["indexing_mode"] = int(rng.integers(-1, 2))
            if rng.random() < 0.2:
                kw["index_bits"] = 64
        elif rng.random() < 0.3:
            kw["label_column"] = int(rng.integers(0, 2))
        record("fuzz%03d" % it, fmt, data, offs, int(rng.integers(1, 5)), kw)
    with open(os.path.join(OUT, "filldata.json"), "w") as f:
        json.dump(out, f, indent=0)
    print("filldata.json:", len(out), "cases,", sum(r["status"] for r in out), "error cases")


if __name__ == "__main__":
    if not po.ref_available():
        sys.exit("build the reference first: make -C oracle ref")
    only = sys.argv[1:]
    for name, fn in (("cases", gen_cases), ("floats", gen_floats), ("synth", gen_synth), ("split", gen_split),
                     ("filldata", gen_filldata)):
        if not only or name in only:
            fn()
