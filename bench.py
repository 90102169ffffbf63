"""Device-resident libsvm / CSV parse throughput on MI355X (BASELINE.json metric).

One step = one full dmlc_amd_parse call (flags 0) over this rank's
HBM-resident synthetic shard, into pre-allocated CSR outputs: the single-pass
kernel when the text is in its grammar, else the exact count -> scan -> write
kernels (forced for the *_exact configs by DMLC_AMD_FLAG_EXACT).  The text is made by the canonical
generator (tools/synth.c, splitmix64) and chunked exactly as dmlc-core's text
InputSplit would chunk it (8 MiB buffers cut after the last newline).

Multi-GPU (torchrun, one process per GPU): every rank parses its own shard of
rows (rank * rows .. (rank + 1) * rows); there is no data-path collective (the
reference's DP byte-range split exchanges nothing).  torch.distributed is used
only for the start/stop barriers and the max-over-ranks time.

Output: one JSON line on rank 0 (see DESIGN.md "Measurement").
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "dmlc-core_amd", "python")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import dmlc_amd  # noqa: E402
from tools import synth  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md

# name -> (format, rows per GPU, width, BASELINE.json config index); the index
# is 0-based into BASELINE.json "configs" (1 = SURVEY's "config 2", the
# headline libsvm 1M x 128; None = not a BASELINE config).  The JSON line
# carries it as config.baseline_config with config.baseline_config_note.
CONFIGS = {
    "libsvm_1m_x128": ("libsvm", 1 << 20, 128, 1),
    "csv_1m_x256": ("csv", 1 << 20, 256, 2),
    "libsvm_1m_x2048": ("libsvm", 1 << 20, 2048, 3),
    "libsvm_32m_x64": ("libsvm", 32 << 20, 64, 4),
    "libfm_1m_x64": ("libfm", 1 << 20, 64, None),  # SURVEY 8(f) row 3, not a BASELINE config
    "libsvm_qid_1m_x128": ("libsvm_qid", 1 << 20, 128, None),  # config 2's rows with qid: (ranking data)
    "libsvm_cmt_1m_x128": ("libsvm_cmt", 1 << 20, 128, None),  # config 2's rows with '#' comments
    # config 2 as a directory of 64 files read by the text InputSplit, each
    # starting with a "# synth libsvm shard" line (per-line fallback, svm_fast.h dirty_lines)
    "libsvm_hdrs_1m_x128": ("libsvm_hdrs", 1 << 20, 128, None),
    # config 2 with a word (" NA", " feature") or an "<id>:-inf" value on every
    # eighth row (svm_fast.h dirty_rewrite: the single pass keeps them)
    "libsvm_dirty_1m_x128": ("libsvm_dirty", 1 << 20, 128, None),
    # grammar variants of configs 2 / 3 (the rates real data hits
    # off the canonical shape)
    "libsvm_nt2_1m_x128": ("libsvm", 1 << 20, 128, None),  # config 2 at the reference's factory nthread = 2
    "libsvm_im1_1m_x128": ("libsvm", 1 << 20, 128, None),  # config 2 with ?indexing_mode=-1
    "libsvm_1b_im1_1m_x128": ("libsvm_1b", 1 << 20, 128, None),  # 1-based ids, ?indexing_mode=-1 (every id shifted)
    "csv_i32_1m_x256": ("csv", 1 << 20, 256, None),        # config 3 parsed as Parser<uint32_t, int32_t>
    "csv_sp_1m_x256": ("csv_sp", 1 << 20, 256, None),      # config 3 with ", " between values
    "csv_hdr_1m_x256": ("csv", 1 << 20, 256, None),        # config 3 behind a header row of column names
    "csv_nan_1m_x256": ("csv_nan", 1 << 20, 256, None),    # config 3 with 0.1 % "nan" fields and a BOM at the head
    "csv_dirty_1m_x256": ("csv_nanp", 1 << 20, 256, None),  # config 3 with a "NaN(x)" field on every 64th row
    # the exact kernels (the path input outside the single-pass grammar takes:
    # inf / nan tokens, BOM lines, '#' lines after a range's first line, qid
    # mixes) on configs 2 / 3, forced with DMLC_AMD_FLAG_EXACT
    "libsvm_exact_1m_x128": ("libsvm", 1 << 20, 128, None),
    "csv_exact_1m_x256": ("csv", 1 << 20, 256, None),
    "libfm_exact_1m_x64": ("libfm", 1 << 20, 64, None),
}
# parser arguments per config (dmlc_amd_params; the reference's URI args)
PARAMS = {
    "libsvm_nt2_1m_x128": {"nthread": 2},
    "libsvm_im1_1m_x128": {"indexing_mode": -1},
    "libsvm_1b_im1_1m_x128": {"indexing_mode": -1},
    "csv_i32_1m_x256": {"value_type": "i32"},
    "libsvm_exact_1m_x128": {"flags": dmlc_amd.FLAG_EXACT},
    "csv_exact_1m_x256": {"flags": dmlc_amd.FLAG_EXACT},
    "libfm_exact_1m_x64": {"flags": dmlc_amd.FLAG_EXACT},
}
DESC = {
    "libsvm_1m_x128": "libsvm 1M rows x 128 nnz/row, device-resident",
    "csv_1m_x256": "CSV dense 1M rows x 256 float cols, device-resident",
    "libsvm_1m_x2048": "libsvm 1M rows x 2048 nnz/row, device-resident",
    "libsvm_32m_x64": "libsvm 32M rows x 64 nnz/row, chunks sharded across GPUs",
    "libfm_1m_x64": "libfm 1M rows x 64 field:id:value/row, device-resident",
    "libsvm_qid_1m_x128": "libsvm 1M rows x 128 nnz/row with qid:<row/16> on every row, device-resident",
    "libsvm_cmt_1m_x128": "libsvm 1M rows x 128 nnz/row, a '# row <r>' comment on every row and a header, device-resident",
    "libsvm_hdrs_1m_x128": "libsvm 1M rows x 128 nnz/row as 64 files of 16384 rows, each headed by a '# synth libsvm shard' line, concatenated as InputSplit reads a directory ('\\n' between files), device-resident",
    "libsvm_dirty_1m_x128": "libsvm 1M rows x 128 nnz/row, every eighth row carrying a word (' NA' / ' feature') or an '<id>:-inf' value mid-row, device-resident",
    "libsvm_nt2_1m_x128": "libsvm 1M rows x 128 nnz/row, each InputSplit chunk cut into nthread=2 ParseBlock ranges (the reference's factory default, text_parser.h:32-35), device-resident",
    "libsvm_im1_1m_x128": "libsvm 1M rows x 128 nnz/row, indexing_mode=-1 (per-range 1-based detection), device-resident",
    "libsvm_1b_im1_1m_x128": "libsvm 1M rows x 128 nnz/row with 1-based ids, indexing_mode=-1 (every range detected 1-based and shifted), device-resident",
    "csv_i32_1m_x256": "CSV dense 1M rows x 256 cols parsed with DType int32 (strtoll), device-resident",
    "csv_sp_1m_x256": "CSV dense 1M rows x 256 float cols, ', ' separators, device-resident",
    "csv_hdr_1m_x256": "CSV dense 1M rows x 256 float cols behind a header row of column names, device-resident",
    "csv_nan_1m_x256": "CSV dense 1M rows x 256 float cols, 0.1% of fields \"nan\", UTF-8 BOM at the file head, device-resident",
    "csv_dirty_1m_x256": "CSV dense 1M rows x 256 float cols, every 64th row's middle field \"NaN(x)\" (ParseFloat's NAN(chars) form), device-resident",
    "libsvm_exact_1m_x128": "libsvm 1M rows x 128 nnz/row on the exact kernels (DMLC_AMD_FLAG_EXACT), device-resident",
    "csv_exact_1m_x256": "CSV dense 1M rows x 256 float cols on the exact kernels (DMLC_AMD_FLAG_EXACT), device-resident",
    "libfm_exact_1m_x64": "libfm 1M rows x 64 field:id:value/row on the exact kernels (DMLC_AMD_FLAG_EXACT), device-resident",
}
SYNTH = {"libsvm": synth.LIBSVM, "csv": synth.CSV, "libfm": synth.LIBFM, "libsvm_qid": synth.LIBSVM_QID,
         "libsvm_cmt": synth.LIBSVM_CMT, "csv_sp": synth.CSV_SP, "libsvm_1b": synth.LIBSVM_1B,
         "csv_nan": synth.CSV_NAN, "libsvm_hdrs": synth.LIBSVM_HDRS, "libsvm_dirty": synth.LIBSVM_DIRTY,
         "csv_nanp": synth.CSV_NANP}
# the arithmetic the path computes in (values decoded to f32 through the
# reference's f64 fraction divide; indices / fields as u32)
DTYPE = {"libsvm": "f32 values / u32 index", "libsvm_1b": "f32 values / u32 index",
         "libsvm_qid": "f32 values / u32 index / u64 qid",
         "libsvm_cmt": "f32 values / u32 index", "libsvm_hdrs": "f32 values / u32 index",
         "libsvm_dirty": "f32 values / u32 index",
         "csv": "f32 values", "csv_sp": "f32 values", "csv_nan": "f32 values", "csv_nanp": "f32 values",
         "libfm": "f32 values / u32 index / u32 field"}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def csr_bytes(counts, index_bits=32, vbytes=4):
    c = [int(x) for x in counts]
    ib = index_bits // 8
    return (8 * (c[dmlc_amd.ROWS] + 1) + vbytes * c[dmlc_amd.LABEL] + 4 * c[dmlc_amd.WEIGHT]
            + 8 * c[dmlc_amd.QID] + ib * c[dmlc_amd.FIELD] + ib * c[dmlc_amd.INDEX]
            + vbytes * c[dmlc_amd.VALUE])


def hbm_copy_rate(dev, nbytes=4 << 30, reps=5):
    """Achievable HBM rate on this GPU for context: a device-to-device
    copy of nbytes, (read + write bytes) / time, best of reps -- by the in-tree
    16-byte-per-lane copy kernel (csrc/copy.hip copy16_kernel via
    dmlc_amd_copy, four uint4 loads in flight per lane) and, for comparison,
    by torch's copy_; HIP events on the stream the copies run on."""
    import torch
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    st = torch.cuda.current_stream()
    L = dmlc_amd.lib()

    def kern():
        rc = L.dmlc_amd_copy(b.data_ptr(), a.data_ptr(), nbytes, st.cuda_stream)
        if rc:
            raise RuntimeError("dmlc_amd_copy rc %d" % rc)
    out = {}
    # the copy-shape probe (tools/ubench/hbm_copy.hip, built by build()): the
    # best of its grid / unroll / non-temporal shapes, one process of its own
    probe = os.path.join(ROOT, "tools", "_build", "hbm_copy")
    best_shape = None
    if os.path.exists(probe):
        import subprocess
        r = subprocess.run([probe], capture_output=True, text=True, timeout=120)
        shapes = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
        if r.returncode == 0 and shapes:
            best_shape = max(shapes, key=lambda d: d["GBps"])
    for name, fn in (("kernel", kern), ("torch", lambda: b.copy_(a))):
        fn()
        best = 1e30
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            fn()
            e1.record(st)
            e1.synchronize()
            best = min(best, e0.elapsed_time(e1) * 1e-3)
        out[name] = round(2 * nbytes / best / 1e9, 1)
    del a, b
    res = {"GBps": out["kernel"], "copy_kernel_GBps": out["kernel"], "torch_GBps": out["torch"],
           "what": "device copy of 4 GiB, (read+write)/time, best of %d: copy_kernel_GBps by the in-tree uint4 "
                   "copy kernel (dmlc_amd_copy), torch_GBps by torch copy_" % reps}
    if best_shape:
        res["GBps"] = max(out["kernel"], best_shape["GBps"])
        res["probe_best"] = best_shape
        res["what"] += ("; GBps: the best of those and of tools/ubench/hbm_copy.hip's 16-byte-lane copy shapes "
                        "(probe_best: its fastest)")
    return res


def cpu_model():
    """The host CPU's model name (the CPU baseline names its CPU)."""
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(text, starts, fmt, budget_s, wide=False):
    """Reference CPU parser (oracle/_ref when it travelled here, else the C
    restatement) over a bounded prefix of this shard's chunks.

    Thread model (oracle/ref_harness.cc ref_bench_blocks): T threads started
    once, each parsing whole chunks round-robin with the format's ParseBlock;
    T = the reference's factory cap min(max(nproc/2 - 4, 1), 2)
    (text_parser.h:32-35, data.cc:31), or with wide=True the uncapped
    max(nproc/2 - 4, 1); nproc = the CPUs this process may
    run on (omp_get_num_procs)."""
    from oracle import pyoracle as po
    f = {"libsvm": po.LIBSVM, "csv": po.CSV, "libfm": po.LIBFM}[fmt]
    nproc = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    use_ref = po.ref_available()
    nthread = max(nproc // 2 - 4, 1) if wide else min(max(nproc // 2 - 4, 1), 2)
    if not use_ref:
        nthread = 1
    # probe on a few chunks per thread, then size the sample to ~budget_s
    k0 = min(max(4, 2 * nthread), len(starts) - 1)
    t, _, _, _ = po.bench_chunks(text, starts[:k0 + 1], f, nthread, use_ref)
    per_chunk = t / max(k0, 1)
    k = int(min(len(starts) - 1, max(k0, budget_s / max(per_chunk, 1e-9))))
    secs, nnz, kind, thr = po.bench_chunks(text, starts[:k + 1], f, nthread, use_ref)
    nb = int(starts[k])
    passes = 1
    # the whole shard in well under the budget (many threads): pass over it
    # again until the sample is about half the budget long
    while secs < budget_s / 2 and passes < 64:
        s2, _, _, _ = po.bench_chunks(text, starts[:k + 1], f, nthread, use_ref)
        secs += s2
        passes += 1
    return {"value": round(nb * passes / secs / 1e9, 4), "unit": "GB/s", "cores": thr, "kind": kind,
            "cpu": cpu_model(), "nproc": nproc,
            "sample": "%d of %d InputSplit chunks (%.1f MB, %d nnz) of the same shard x %d pass(es), %d thread(s) "
                      "each parsing whole chunks round-robin with ParseBlock (%s, nproc=%d), %.1f s"
                      % (k, len(starts) - 1, nb / 1e6, nnz, passes, thr,
                         "uncapped max(nproc/2-4,1)" if wide else "reference cap min(max(nproc/2-4,1),2)",
                         nproc, secs)}


def spawn_ranks(n):
    """`bench.py --gpus N` without a launcher: start N rank processes (one per
    GPU) the way torch.distributed.run would, and exit with the first failing
    rank's status.  The parent makes no GPU call (device_count does not
    initialise the GPU on this image), so the children own their devices."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DMLC_AMD_BENCH_SPAWNED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    for pr in procs:
        c = pr.wait()
        if c and not rc:
            rc = c
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="libsvm_1m_x128", choices=sorted(CONFIGS))
    ap.add_argument("--rows", type=int, default=0, help="override rows per GPU")
    ap.add_argument("--tile-bytes", type=int, default=0)
    ap.add_argument("--label-column", type=int, default=-1, help="csv: CSVParserParam::label_column")
    ap.add_argument("--cpu-budget", type=float, default=15.0,
                    help="seconds of CPU-baseline parsing (rank 0, N=1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and not (world == 1 and args.gpus == 1):
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE %d" % (args.gpus, world))
    dist = None
    backend = None
    ndev = torch.cuda.device_count()
    if world > 1:
        import torch.distributed as dist
        if ndev >= world:  # one process per GPU: RCCL for the barriers and the max-over-ranks time
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:  # rehearsal with more ranks than GPUs (ranks share a card): gloo on the host
            torch.cuda.set_device(local % ndev)
            dist.init_process_group("gloo")
        backend = dist.get_backend()
        if dist.get_world_size() != args.gpus:
            raise SystemExit("bench.py: process group has %d ranks, --gpus %d" % (dist.get_world_size(), args.gpus))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    fmt, rows, width, cfg_idx = CONFIGS[args.config]
    if args.config == "libsvm_32m_x64":
        rows = rows // max(world, args.gpus, 1) if world > 1 else rows // 8
    if args.rows:
        rows = args.rows
    t0 = time.time()
    text, _ = synth.rows(SYNTH[fmt], rows, width, seed=1, row0=rank * rows)
    if args.config == "csv_hdr_1m_x256":  # a header row: a row without values (csv_fast.h csv_junk_byte)
        header = np.frombuffer((",".join("feature_%d" % j for j in range(width)) + "\n").encode(), np.uint8)
        text = np.concatenate([header, text])
    starts = dmlc_amd.text_chunk_starts(text)
    log("[rank %d] generated %s: %d rows, %.3f GB, %d chunks in %.1f s"
        % (rank, args.config, rows, text.size / 1e9, len(starts) - 1, time.time() - t0))

    d_text = torch.from_numpy(text).to(dev)
    d_starts = torch.from_numpy(starts).to(dev)
    nbytes = int(text.size)
    pfmt = {"libsvm_qid": "libsvm", "libsvm_cmt": "libsvm", "libsvm_1b": "libsvm", "libsvm_hdrs": "libsvm",
            "libsvm_dirty": "libsvm", "csv_sp": "csv", "csv_nanp": "csv",
            "csv_nan": "csv"}.get(fmt, fmt)
    pkw = dict(PARAMS.get(args.config, {}))
    if pfmt == "csv":
        pkw["label_column"] = args.label_column
    p = dmlc_amd.DeviceParser(pfmt, tile_bytes=args.tile_bytes, **pkw)
    res = torch.zeros(16, dtype=torch.int64, device=dev)
    counts = p.count(d_text, d_starts, result=res)
    out = p.alloc(counts)
    out["_csr"] = p.csr_of(out)
    vtype = pkw.get("value_type", "f32")
    b_out = csr_bytes(counts, vbytes=8 if vtype == "i64" else 4)
    dtype = DTYPE[fmt] if vtype == "f32" else "%s values (strtoll) / u32 index" % vtype

    def step():
        # one full dmlc_amd_parse call (flags 0) into pre-allocated outputs: the
        # single-pass kernel when the text is in the uniform grammar, else the
        # exact count -> scan -> write pipeline
        p.parse_into(d_text, d_starts, out, res)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    r = res.cpu().numpy().view(np.uint64)
    if int(r[8]) != 0:
        raise RuntimeError("parse error %#x" % int(r[8]))
    if [int(x) for x in r[:7]] != [int(x) for x in counts[:7]]:
        raise RuntimeError("count mismatch between calls")
    gate = int(r[9])
    if gate & 2:  # the look-back's safety valve handed the input to the exact kernels: not a valid fast-path number
        raise RuntimeError("look-back valve fired (result.path %d)" % gate)
    path = "exact tile kernels" if gate else "single-pass uniform-grammar kernel"

    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    dmlc_amd.profile_begin()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    kern_ms, launches, kern_name = dmlc_amd.profile_end()
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    r = res.cpu().numpy().view(np.uint64)
    if int(r[8]) != 0:
        raise RuntimeError("parse error %#x" % int(r[8]))
    if int(r[9]) != gate:
        raise RuntimeError("path changed inside the timed region (%d -> %d)" % (gate, int(r[9])))

    ms_per_step = elapsed * 1e3 / args.steps
    total_in = nbytes * world
    value = total_in * args.steps / elapsed / 1e9
    # dominant kernel: reads the text once and writes the CSR once (B_in + B_out)
    dom_ms = kern_ms / max(launches, 1)
    if gate:  # the exact pipeline produced the result: price the whole call (its several kernels)
        kern_name = "exact path (every kernel of the call: single-pass attempt, exact count, scan, exact write)"
        dom_ms = ms_per_step
    dom_bytes = nbytes + b_out
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    traffic = None
    build = dmlc_amd.build_id()
    traffic_src = None
    try:  # HBM bytes per launch measured by rocprofv3 PMC passes (tools/gpu_pmc.sh) on this kernel
        tr = json.load(open(os.path.join(ROOT, "profiles", "traffic.json"))).get(args.config)
        if tr and tr["kernel"] == kern_name and not args.rows and not args.tile_bytes:
            traffic = tr["hbm_bytes_per_launch"]
            # which build the PMC passes ran on (tools/traffic_update.py), and whether it is this one
            traffic_src = {"build": tr.get("build"), "same_build": tr.get("build") == build,
                           "source": tr.get("source")}
    except (OSError, ValueError):
        pass
    par = "shard%d" % world
    line = {
        "metric": "device-resident libsvm parse GB/s (input bytes) at 1/2/4/8 GPU; % HBM roofline",
        "value": round(value, 3),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": dtype,
        "data": "synthetic (tools/synth.c splitmix64 seed 1, %.9g values), HBM-resident",
        "config": {"workload": DESC[args.config], "baseline_config": cfg_idx,
                   "baseline_config_note": "0-based index into BASELINE.json configs (1 = SURVEY config 2)",
                   "format": pfmt,
                   "rows_per_gpu": rows, "width": width, "input_bytes_per_gpu": nbytes,
                   "csr_bytes_per_gpu": b_out, "nnz_per_gpu": int(counts[dmlc_amd.INDEX]),
                   "chunks_per_gpu": len(starts) - 1, "parallelism": par,
                   "nthread": int(p.params.nthread),  # ParseBlock ranges per chunk (FillData, text_parser.h:116-155)
                   **({"label_column": args.label_column} if args.label_column >= 0 else {}),
                   **{k: v for k, v in pkw.items() if k not in ("label_column", "nthread")}},
        "hbm_frac_input": round(value / world / HBM_PEAK_GBS, 4),
        "hbm_frac_in_out": round((total_in + b_out * world) * args.steps / elapsed / 1e9
                                 / world / HBM_PEAK_GBS, 4),
        "path": path,
        "roofline": {"bound": "hbm", "kernel": kern_name, "achieved": round(achieved, 2),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "bytes_per_launch": dom_bytes, "avg_ms": round(dom_ms, 4),
                     "traffic_measured_on": traffic_src},
        "build": build,
        "cpu_baseline": None,
    }
    if world > 1:
        line["ranks"] = {"world_size": world, "backend": backend, "devices_visible": ndev,
                         "launcher": "bench.py --gpus" if os.environ.get("DMLC_AMD_BENCH_SPAWNED") else "external",
                         "note": "one rank per GPU" if ndev >= world else
                                 "rehearsal: %d ranks share %d card(s), gloo barriers" % (world, ndev)}
    if rank == 0 and world == 1:
        try:
            line["hbm_copy"] = hbm_copy_rate(dev)
        except Exception as e:  # context only, never fatal
            line["hbm_copy"] = {"error": repr(e)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            line["cpu_baseline"] = cpu_baseline(text, starts, pfmt, args.cpu_budget)
            if line["cpu_baseline"].get("kind") == "reference":
                line["cpu_baseline_max_threads"] = cpu_baseline(text, starts, pfmt, args.cpu_budget / 2, wide=True)
        except Exception as e:  # reported, never fatal for the GPU number
            line["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
