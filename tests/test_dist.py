"""Multi-process (world size 2, gloo, CPU) tests of the sharded path.

The GPU parse of each rank's part is covered by the -m gpu tests; here the
per-rank parse is the oracle (CPU), so these tests pin what multi-GPU adds:
the reference's byte-range split (InputSplitBase::ResetPartition +
LineSplitter::SeekRecordBegin) and the Push-style host concatenation of the
per-rank CSRs, gathered over torch.distributed (gloo).
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dmlc-core_amd", "python")]

import dmlc_amd_dist as dd  # noqa: E402
import fuzz_text  # noqa: E402
from oracle import pyoracle as po  # noqa: E402
from tools import synth  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_part_range_matches_reference_split():
    """part_range == the oracle InputSplit restatement (pinned to the
    reference's unittest_inputsplit scenarios in test_oracle.py)."""
    rng = np.random.default_rng(5)
    for it in range(60):
        data = fuzz_text.uniform_libsvm(rng, int(rng.integers(1, 200)), 20)
        if it % 5 == 0:
            data = data.replace(b"\n", b"\r\n")
        for world in (1, 2, 3, 4, 7):
            for rank in range(world):
                b, e = dd.part_range(data, rank, world)
                got = data[b:e]
                exp = b"".join(po.split_text([data], rank, world))
                # the InputSplit appends a '\n' when the input's last record has none
                if exp.endswith(b"\n") and not got.endswith(b"\n") and e == len(data) and e > b:
                    exp = exp[:-1]
                assert got == exp, (it, world, rank, b, e)


def test_concat_csr_equals_single_parse():
    text, _ = synth.rows(synth.LIBSVM, 3000, 40, seed=3)
    data = text.tobytes()
    whole = po.parse_chunks(data, [0, len(data)], fmt=po.LIBSVM)
    for world in (2, 3, 5):
        parts = []
        for r in range(world):
            b, e = dd.part_range(data, r, world)
            parts.append(po.parse_chunks(data[b:e], [0, e - b], fmt=po.LIBSVM))
        cat = dd.concat_csr(parts)
        for k in ("offset", "label", "index", "value"):
            assert np.asarray(cat[k]).tobytes() == np.asarray(whole[k]).astype(np.asarray(cat[k]).dtype).tobytes(), k


def _worker(rank, world, port, path, fmt, out_path):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    data = open(path, "rb").read()
    b, e = dd.part_range(data, rank, world)
    part = po.parse_chunks(data[b:e], [0, e - b] if e > b else [0], fmt=fmt)  # per-rank parse (CPU stand-in)
    part = {k: part[k] for k in ("offset", "label", "weight", "qid", "index", "value")}
    cat = dd.gather_concat(part)
    if rank == 0:
        np.savez(out_path, **cat)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("fmt", [po.LIBSVM, po.CSV])
def test_gloo_world2_gather_concat(tmp_path, fmt):
    import torch.multiprocessing as mp
    if fmt == po.LIBSVM:
        text, _ = synth.rows(synth.LIBSVM, 4000, 30, seed=11)
    else:
        text, _ = synth.rows(synth.CSV, 3000, 20, seed=11)
    data = text.tobytes()
    path = str(tmp_path / "in.txt")
    open(path, "wb").write(data)
    out = str(tmp_path / "cat.npz")
    mp.spawn(_worker, args=(2, _free_port(), path, fmt, out), nprocs=2, join=True)
    cat = np.load(out)
    whole = po.parse_chunks(data, [0, len(data)], fmt=fmt)
    for k in ("offset", "index", "value"):
        assert cat[k].tobytes() == np.asarray(whole[k]).astype(cat[k].dtype).tobytes(), k
