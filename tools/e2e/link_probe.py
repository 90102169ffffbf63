"""Host link rates on the GPU box: what the end-to-end pipeline
can reach.  Page-locked host buffers <-> HBM, 1 GiB each way:
  * h2d / d2h alone, by copy kernel (dmlc_amd_copy) and by DMA (hipMemcpyAsync)
  * both directions at once on two streams (the pipeline's steady state:
    batch k's CSR out while batch k+1's text comes in)
One JSON line per measurement (best of 3).  Diagnostic only."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dmlc-core_amd", "python")]
import torch  # noqa: E402

import dmlc_amd  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 and int(sys.argv[1]) > 0 else 1 << 30
    L = dmlc_amd.lib()
    host_in = torch.empty(n, dtype=torch.uint8).pin_memory()
    host_out = torch.empty(n, dtype=torch.uint8).pin_memory()
    dev_in = torch.empty(n, dtype=torch.uint8, device="cuda")
    dev_out = torch.ones(n, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def kcopy(dst, src, s):
        assert L.dmlc_amd_copy(dst.data_ptr(), src.data_ptr(), n, s.cuda_stream) == 0

    def dcopy(dst, src, s):
        with torch.cuda.stream(s):
            dst.copy_(src, non_blocking=True)

    cases = {
        "h2d_kernel": [(kcopy, dev_in, host_in, s1)],
        "d2h_kernel": [(kcopy, host_out, dev_out, s1)],
        "h2d_dma": [(dcopy, dev_in, host_in, s1)],
        "d2h_dma": [(dcopy, host_out, dev_out, s1)],
        "both_kernel": [(kcopy, dev_in, host_in, s1), (kcopy, host_out, dev_out, s2)],
        "both_dma": [(dcopy, dev_in, host_in, s1), (dcopy, host_out, dev_out, s2)],
        "h2d_kernel_d2h_dma": [(kcopy, dev_in, host_in, s1), (dcopy, host_out, dev_out, s2)],
        "h2d_dma_d2h_kernel": [(dcopy, dev_in, host_in, s1), (kcopy, host_out, dev_out, s2)],
    }
    for name, ops in cases.items():
        best = 1e30
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for f, d, s_, st in ops:
                f(d, s_, st)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        moved = n * len(ops)
        print(json.dumps({"case": name, "bytes": moved, "s": round(best, 5), "GBps": round(moved / best / 1e9, 2)}),
              flush=True)


def batched(nb=40 << 20, reps=24):
    """The pipeline's shape: reps batches of nb bytes in, nb/2 out, two
    workers (streams) each copying its batch in, then its CSR out; by copy
    kernel and by DMA.  GB/s of input moved."""
    L = dmlc_amd.lib()
    h_in = [torch.empty(nb, dtype=torch.uint8).pin_memory() for _ in range(2)]
    h_out = [torch.empty(nb // 2, dtype=torch.uint8).pin_memory() for _ in range(2)]
    d_in = [torch.empty(nb, dtype=torch.uint8, device="cuda") for _ in range(2)]
    d_out = [torch.ones(nb // 2, dtype=torch.uint8, device="cuda") for _ in range(2)]
    ss = [torch.cuda.Stream(), torch.cuda.Stream()]
    for mode in ("kernel", "dma", "dma_in_kernel_out"):
        best = 1e30
        for _ in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for r in range(reps):
                w = r % 2
                s = ss[w]
                if mode == "kernel":
                    assert L.dmlc_amd_copy(d_in[w].data_ptr(), h_in[w].data_ptr(), nb, s.cuda_stream) == 0
                    assert L.dmlc_amd_copy(h_out[w].data_ptr(), d_out[w].data_ptr(), nb // 2, s.cuda_stream) == 0
                else:
                    with torch.cuda.stream(s):
                        d_in[w].copy_(h_in[w], non_blocking=True)
                        if mode == "dma":
                            h_out[w].copy_(d_out[w], non_blocking=True)
                    if mode != "dma":
                        assert L.dmlc_amd_copy(h_out[w].data_ptr(), d_out[w].data_ptr(), nb // 2, s.cuda_stream) == 0
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        print(json.dumps({"case": "batched_" + mode, "batch_bytes": nb, "GBps_in": round(nb * reps / best / 1e9, 2)}),
              flush=True)


def host_memcpy(n=1 << 30, threads=(1, 4, 8, 16)):
    """Host DRAM copy rate (what the reader's page-cache -> pinned copy and the
    links' DMA share): (read + write bytes) / time, best of 3."""
    import concurrent.futures
    import numpy as np
    a = np.ones(n, dtype=np.uint8)
    b = np.empty_like(a)
    for t in threads:
        step = n // t
        best = 1e30
        with concurrent.futures.ThreadPoolExecutor(t) as ex:
            for _ in range(3):
                t0 = time.perf_counter()
                list(ex.map(lambda i: np.copyto(b[i * step:(i + 1) * step], a[i * step:(i + 1) * step]), range(t)))
                best = min(best, time.perf_counter() - t0)
        print(json.dumps({"case": "host_memcpy", "threads": t, "GBps_rw": round(2 * n / best / 1e9, 1)}), flush=True)


def sweep(sizes_mib=(4, 16, 64, 256, 1024), total=2 << 30):
    """Copy-size sweep: per copy size, direction, engine
    (copy kernel / DMA) and stream count (one stream; two streams taking
    alternate copies), back-to-back copies moving `total` bytes, timed from
    the first enqueue to the sync: the rate a pipeline of that batch size can
    get from the link.  Also both directions at once (two streams, one per
    direction) per size."""
    L = dmlc_amd.lib()
    big = max(sizes_mib) << 20
    host = [torch.empty(big, dtype=torch.uint8).pin_memory() for _ in range(2)]
    dev = [torch.ones(big, dtype=torch.uint8, device="cuda") for _ in range(2)]
    ss = [torch.cuda.Stream(), torch.cuda.Stream()]

    def one(eng, dst, src, nb, s):
        if eng == "kernel":
            assert L.dmlc_amd_copy(dst.data_ptr(), src.data_ptr(), nb, s.cuda_stream) == 0
        else:
            with torch.cuda.stream(s):
                dst[:nb].copy_(src[:nb], non_blocking=True)

    for mib in sizes_mib:
        nb = mib << 20
        reps = max(2, total // nb)
        for eng in ("kernel", "dma"):
            for direction in ("h2d", "d2h", "both"):
                for nstream in ((1, 2) if direction != "both" else (2,)):
                    best = 1e30
                    for _ in range(2):
                        torch.cuda.synchronize()
                        t0 = time.perf_counter()
                        for r in range(reps):
                            w = r % nstream
                            if direction == "both":
                                one(eng, dev[0], host[0], nb, ss[0])
                                one(eng, host[1], dev[1], nb, ss[1])
                            elif direction == "h2d":
                                one(eng, dev[w], host[w], nb, ss[w])
                            else:
                                one(eng, host[w], dev[w], nb, ss[w])
                        torch.cuda.synchronize()
                        best = min(best, time.perf_counter() - t0)
                    moved = nb * reps * (2 if direction == "both" else 1)
                    print(json.dumps({"case": "sweep", "copy_mib": mib, "engine": eng, "dir": direction,
                                      "streams": nstream, "copies": reps * (2 if direction == "both" else 1),
                                      "GBps": round(moved / best / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    what = sys.argv[2:] or ["main", "batched", "host"]
    if "main" in what:
        main()
    if "batched" in what:
        batched()
        for nb in (4 << 20, 16 << 20, 64 << 20, 256 << 20):
            batched(nb=nb, reps=max(8, (1 << 30) // nb))
    if "sweep" in what:
        sweep()
    if "host" in what:
        host_memcpy()
