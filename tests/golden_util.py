"""Helpers to load tests/golden/* fixtures."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def dec(e):
    if e["dtype"] == "f32bits":
        return np.array(e["data"], dtype=np.uint32).view(np.float32)
    return np.array(e["data"], dtype=e["dtype"])


def load_cases():
    with open(os.path.join(GOLDEN, "cases.json")) as f:
        return json.load(f)


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def load_floats():
    z = np.load(os.path.join(GOLDEN, "floats.npz"))
    strs = z["text"].tobytes().decode("latin-1").split("\0")
    return strs, z["bits"], z["used"]


def same(a, b):
    """Bit-exact array equality (floats compared by bit pattern, NaN == NaN)."""
    a, b = np.asarray(a), np.asarray(b)
    if a.shape != b.shape:
        return False
    if a.dtype == np.float32 or b.dtype == np.float32:
        return np.array_equal(a.astype(np.float32).view(np.uint32), b.astype(np.float32).view(np.uint32))
    return np.array_equal(a.astype(np.uint64) if a.dtype.kind == "u" else a, b.astype(a.dtype))


FIELDS = ("offset", "label", "weight", "qid", "field", "index", "value")


def diff(got, exp):
    """Return list of field names that differ."""
    return [k for k in FIELDS if k in exp and not same(got[k], exp[k])]


def blocks_of(h):
    """Per-block (rows, index, value) counts of a GPU / emulator result, from
    its per-unit table (one row per ParseBlock unit, dmlc_amd.h chunk_table):
    the blocks the reference's ParserImpl::Next hands out are the units with
    at least one row (parser.h:32-48)."""
    tab = np.asarray(h["chunk_table"], dtype=np.int64).reshape(-1, 8)
    tot = np.asarray(h["counts"][:8], dtype=np.int64)[None, :]
    per = np.vstack([tab[1:], tot]) - tab
    keep = per[:, 0] > 0
    return {"rows": per[keep, 0].tolist(), "index": per[keep, 1].tolist(), "value": per[keep, 2].tolist()}
