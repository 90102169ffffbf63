"""CPU-side checks of the C-ABI library (no GPU needed)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "dmlc-core_amd", "lib", "libdmlc_amd.so")


def declared_symbols():
    syms = set()
    inc = os.path.join(ROOT, "include")
    for fn in os.listdir(inc):
        if fn.endswith(".h"):
            txt = open(os.path.join(inc, fn)).read()
            syms |= set(re.findall(r"^\w[\w\s\*]*?\b(dmlc_amd_\w+)\s*\(", txt, re.M))
    return syms


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        import subprocess
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "dmlc-core_amd")])
    return ctypes.CDLL(LIB)


def test_library_loads_and_exports_every_declared_symbol(lib):
    syms = declared_symbols()
    assert {"dmlc_amd_parse", "dmlc_amd_workspace_bytes", "dmlc_amd_strtof_batch"} <= syms
    for s in syms:
        assert hasattr(lib, s), s


def test_python_binding_lists_every_export():
    import dmlc_amd
    assert set(dmlc_amd.EXPORTED_SYMBOLS) == declared_symbols()


def test_abi_version_and_error_strings(lib):
    lib.dmlc_amd_abi_version.restype = ctypes.c_int
    assert lib.dmlc_amd_abi_version() == 2
    lib.dmlc_amd_error_string.restype = ctypes.c_char_p
    assert b"sign == true" in lib.dmlc_amd_error_string(1)
    assert b"NAN" in lib.dmlc_amd_error_string(2)


def test_workspace_and_argument_validation(lib):
    import dmlc_amd
    p = dmlc_amd.make_params("libsvm")
    ws = dmlc_amd.lib().dmlc_amd_workspace_bytes(1 << 30, 128, ctypes.byref(p))
    tile, _ = dmlc_amd.fast_geometry()
    # per single-pass tile a look-back record (8 words), plus per-chunk and per-exact-tile tables,
    # plus the exact libsvm count pass's window records (args.h exact_rec_bytes: at most the
    # text's size + 64 MiB, about half of it at the default 256 KiB exact tiles)
    assert 0 < ws < (1 << 30) // tile * 64 + (1 << 20) + (1 << 30) * 6 // 10
    c = dmlc_amd.make_params("csv")  # (CSV keeps window count records too)
    wc = dmlc_amd.lib().dmlc_amd_workspace_bytes(1 << 30, 128, ctypes.byref(c))
    assert 0 < wc < (1 << 30) // tile * 64 + (1 << 20) + (1 << 30) * 6 // 10
    fm = dmlc_amd.make_params("libfm")  # (libfm keeps the same records since round 6)
    wf = dmlc_amd.lib().dmlc_amd_workspace_bytes(1 << 30, 128, ctypes.byref(fm))
    assert 0 < wf < (1 << 30) // tile * 64 + (1 << 20) + (1 << 30) * 6 // 10
    small = dmlc_amd.make_params("libsvm", tile_bytes=64)  # tiny exact tiles: records off
    assert dmlc_amd.lib().dmlc_amd_workspace_bytes(1 << 30, 128, ctypes.byref(small)) < (1 << 30) * 2
    # records never exceed 5/8 of the text + 1 MiB (args.h exact_rec_on), whatever the exact tile;
    # libsvm and libfm keep the same tables and records, libsvm the lean kernel's look-back words too
    for tb in (4096, 9000, 65536, 1 << 18, 1 << 20):
        q = dmlc_amd.make_params("libsvm", tile_bytes=tb)
        base = dmlc_amd.make_params("libfm", tile_bytes=tb)
        for n in (1 << 16, 1 << 20, 32 << 20, 1 << 30):
            nft = (n + tile - 1) // tile
            extra = (dmlc_amd.lib().dmlc_amd_workspace_bytes(n, 128, ctypes.byref(q))
                     - dmlc_amd.lib().dmlc_amd_workspace_bytes(n, 128, ctypes.byref(base)))
            assert extra == (nft * 5 + 1) * 8, (tb, n, extra)
            ntiles = (n + tb - 1) // tb
            rec = ntiles * (tb // 8192 + 3) * (256 * 16 + 16)  # args.h exact_rec_bytes
            tables = dmlc_amd.lib().dmlc_amd_workspace_bytes(n, 128, ctypes.byref(base))
            if rec <= n // 8 * 5 + (1 << 20):  # records on: they are part of the workspace
                assert tables >= rec, (tb, n)
    # the CSV single pass keeps an 8-word look-back record per 16 KiB tile (args.h kCsvLbWords),
    # libfm 5 (kFastLbWords): with the exact kernels' records off (64-byte exact tiles) the
    # difference is those words alone -- round 6 sized CSV at 5 and its records ran into labsum
    n = 1 << 30
    nft = n // tile
    c64 = dmlc_amd.make_params("csv", tile_bytes=64)
    f64 = dmlc_amd.make_params("libfm", tile_bytes=64)
    d = (dmlc_amd.lib().dmlc_amd_workspace_bytes(n, 128, ctypes.byref(c64))
         - dmlc_amd.lib().dmlc_amd_workspace_bytes(n, 128, ctypes.byref(f64)))
    assert d == nft * 3 * 8, (d, nft)
    # bad index_bits is rejected before any device work
    bad = dmlc_amd.make_params("libsvm", index_bits=16)
    csr = dmlc_amd.Csr()
    rc = dmlc_amd.lib().dmlc_amd_parse(None, 0, None, 0, ctypes.byref(bad), ctypes.byref(csr), None,
                                      None, 0, None, None)
    assert rc == 32
    # csv label_column == weight_column is rejected (csv_parser.h:59-60)
    c = dmlc_amd.make_params("csv", label_column=1, weight_column=1)
    rc = dmlc_amd.lib().dmlc_amd_parse(None, 0, None, 0, ctypes.byref(c), ctypes.byref(csr), None,
                                      None, 0, None, None)
    assert rc == 32


def test_copy_n_dev_rejects_slot_past_the_counts(lib):
    """dmlc_amd_copy_n_dev reads d_counts[slot] on the device: slots past the
    DMLC_AMD_COPY_SLOTS words of dmlc_amd_result.count are refused before any
    launch (so no GPU is needed)."""
    f = lib.dmlc_amd_copy_n_dev
    f.restype = ctypes.c_int
    P = ctypes.c_void_p
    dst = (P * 1)(16)
    src = (P * 1)(32)
    cnt = (ctypes.c_uint64 * 8)()
    one = (ctypes.c_uint64 * 1)(1)
    big = (ctypes.c_uint64 * 1)(64)
    zero = (ctypes.c_uint64 * 1)(0)
    for s in (8, 9, 1 << 20):
        sl = (ctypes.c_int * 1)(s)
        assert f(dst, src, cnt, sl, one, zero, big, 1, None) == 32, s
    assert f(dst, src, cnt, (ctypes.c_int * 1)(0), one, zero, big, 17, None) == 32  # n > DMLC_AMD_COPY_MAX


def test_device_count_without_gpu(lib):
    lib.dmlc_amd_device_count.restype = ctypes.c_int
    assert lib.dmlc_amd_device_count() >= 0
