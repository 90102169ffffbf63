"""Multi-GPU sharding of the parse path (one process per GPU, no data-path
collective).

The reference shards text input by byte range: part k of n covers
[ceil(total/n)*k, ceil(total/n)*(k+1)), both ends moved forward to the next
record start (InputSplitBase::ResetPartition, src/io/input_split_base.cc:29-63;
LineSplitter::SeekRecordBegin, src/io/line_split.cc:11-36).  Each rank parses
its own part on its own GPU; per-rank CSR batches are concatenated on the host
with offset rebasing exactly as RowBlockContainer::Push(RowBlock) does
(src/data/row_block.h:126-168).  torch.distributed carries nothing on the data
path; gather_concat() is the optional host-side collection (gloo or RCCL) for
callers that want the whole CSR on one rank.
"""
import numpy as np

_NL = (10, 13)


def seek_record_begin(data, pos):
    """Bytes LineSplitter::SeekRecordBegin skips from pos: through the first
    '\\n'/'\\r' at or after pos, then over the newlines that follow it."""
    a = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    n = a.size
    if pos >= n:
        return 0
    nl = (a[pos:] == 10) | (a[pos:] == 13)
    first = int(np.argmax(nl)) if nl.any() else -1
    if first < 0:
        return n - pos  # read to the end without a newline
    step = first + 1
    rest = nl[first + 1:]
    if rest.size == 0:
        return step
    non = ~rest
    return step + (int(np.argmax(non)) if non.any() else rest.size)


def part_range(data, rank, world):
    """[begin, end) of part `rank` of `world` over one in-memory text, as the
    reference's text InputSplit computes it (align_bytes = 1)."""
    total = len(data)
    nstep = (total + world - 1) // world if world > 0 else total
    b = min(nstep * rank, total)
    e = min(nstep * (rank + 1), total)
    if b == e:
        return b, b
    if e != total:
        e += seek_record_begin(data, e)
    if b != 0:
        b += seek_record_begin(data, b)
    return b, max(b, e)


_ARRAYS = ("label", "weight", "qid", "field", "index", "value")


def concat_csr(parts):
    """RowBlockContainer::Push-style concatenation of per-rank CSR dicts
    (numpy arrays: offset, label, weight, qid, field, index, value): offsets
    rebased so the result equals one parse of the concatenated input."""
    offs = [np.zeros(1, np.uint64)]
    shift = np.uint64(0)
    for p in parts:
        o = np.asarray(p["offset"], dtype=np.uint64)
        if o.size:
            offs.append(o[1:] - o[0] + shift)
            shift = shift + (o[-1] - o[0])
    out = {"offset": np.concatenate(offs)}
    for k in _ARRAYS:
        arrs = [np.asarray(p[k]) for p in parts if k in p]
        out[k] = np.concatenate(arrs) if arrs else np.zeros(0)
    return out


def gather_concat(part, group=None, dst=0):
    """Collect every rank's CSR dict on rank `dst` (torch.distributed, any
    backend) and return the rebased concatenation there (None elsewhere)."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    bufs = [None] * world if dist.get_rank(group) == dst else None
    dist.gather_object(part, bufs, dst=dst, group=group)
    return concat_csr(bufs) if bufs is not None else None


def parse_part(text, rank, world, fmt="libsvm", chunk_bytes=8 << 20, **kw):
    """Parse part `rank` of `world` of a host text on this process's GPU:
    InputSplit-style chunks of the part, one dmlc_amd_parse call.  Returns a
    host CSR dict (dmlc_amd.parse_bytes)."""
    import dmlc_amd
    b, e = part_range(text, rank, world)
    part = np.frombuffer(text, dtype=np.uint8)[b:e] if not isinstance(text, np.ndarray) else text[b:e]
    starts = dmlc_amd.text_chunk_starts(part, chunk_bytes).tolist() if part.size else [0]
    return dmlc_amd.parse_bytes(part.tobytes(), starts, fmt=fmt, **kw)
