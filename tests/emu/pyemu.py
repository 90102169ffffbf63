"""TEST INFRASTRUCTURE ONLY: run the CPU emulation of the tile kernels (emu.cpp,
built with AddressSanitizer) on host bytes and return numpy arrays shaped like
dmlc_amd.parse_bytes()."""
import os
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
EXE = os.path.join(HERE, "_build", "emu_asan")
_FMT = {"libsvm": 0, "csv": 1, "libfm": 2}


_BUILT = False


def build():
    """(Re)build the emulator when its sources changed (make is a no-op otherwise)."""
    global _BUILT
    import fcntl
    os.makedirs(os.path.join(HERE, "_build"), exist_ok=True)
    # pytest-xdist workers share the build dir: one make at a time, so no worker
    # executes the binary while another is still linking it
    with open(os.path.join(HERE, "_build", ".lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.check_call(["make", "-s", "-C", HERE])
    _BUILT = True


def parse(data, chunk_offsets=None, fmt="libsvm", index_bits=32, value_type=0, indexing_mode=0,
          label_column=-1, weight_column=-1, delimiter=",", tile_bytes=0, exact=False, nthread=1):
    if not _BUILT:
        build()
    raw = data.encode("latin-1") if isinstance(data, str) else bytes(data)
    if chunk_offsets is None:
        chunk_offsets = [0, len(raw)] if raw else [0]
    f = _FMT[fmt] if isinstance(fmt, str) else fmt
    with tempfile.TemporaryDirectory() as td:
        tp, cp, op = os.path.join(td, "t"), os.path.join(td, "c"), os.path.join(td, "o")
        open(tp, "wb").write(raw)
        np.asarray(chunk_offsets, dtype=np.uint64).tofile(cp)
        d = ord(delimiter) if isinstance(delimiter, str) else int(delimiter)
        env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:exitcode=77")
        env.pop("EMU_EXACT", None)
        env["EMU_NTHREAD"] = str(int(nthread))
        if exact:
            env["EMU_EXACT"] = "1"
        r = subprocess.run([EXE, str(f), str(index_bits), str(int(value_type)), str(indexing_mode),
                            str(label_column), str(weight_column), str(d), str(tile_bytes), tp, cp, op],
                           capture_output=True, env=env)
        if r.returncode != 0:
            raise RuntimeError("emulator failed rc=%d\n%s" % (r.returncode, r.stderr.decode()[-4000:]))
        res = np.fromfile(op + ".res", dtype=np.uint64)
        it = np.uint32 if index_bits == 32 else np.uint64
        vt = {0: np.float32, 1: np.int32, 2: np.int64}[int(value_type) if f == 1 else 0]
        h = {
            "offset": np.fromfile(op + ".offset", dtype=np.uint64),
            "label": np.fromfile(op + ".label", dtype=vt),
            "weight": np.fromfile(op + ".weight", dtype=np.float32),
            "qid": np.fromfile(op + ".qid", dtype=np.uint64),
            "field": np.fromfile(op + ".field", dtype=it),
            "index": np.fromfile(op + ".index", dtype=it),
            "value": np.fromfile(op + ".value", dtype=vt),
            "chunk_table": np.fromfile(op + ".chunks", dtype=np.uint64).reshape(-1, 8),
            "error": int(res[8]),
            "counts": [int(x) for x in res[:8]],
            "path": "fast" if b"path=fast" in r.stderr else "exact",
        }
        return h
