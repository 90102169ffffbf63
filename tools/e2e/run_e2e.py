"""End-to-end measurement (DESIGN.md "End to end"): synthetic file on the
host -> dmlc::Parser<uint32_t,float> (host InputSplit, pinned staging,
hipMemcpyAsync H2D, MI355X parse, D2H into pinned RowBlocks) -> Next() loop.
Next to it: the genuine reference's file -> Parser path (oracle/_ref, built
from /root/reference sources) on a bounded sample, when that library is here.

usage: python tools/e2e/run_e2e.py [config ...]   (default: libsvm_1m_x128 csv_1m_x256)
"""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dmlc-core_amd", "python")]
from tools import synth  # noqa: E402

CFG = {"libsvm_1m_x128": ("libsvm", 1 << 20, 128), "csv_1m_x256": ("csv", 1 << 20, 256)}


def main():
    names = sys.argv[1:] or ["libsvm_1m_x128", "csv_1m_x256"]
    exe = os.path.join(ROOT, "tools", "e2e", "_build", "e2e_bench")
    tmp = os.environ.get("TMPDIR", tempfile.gettempdir())
    for name in names:
        fmt, rows, width = CFG[name]
        text, _ = synth.rows(synth.LIBSVM if fmt == "libsvm" else synth.CSV, rows, width, seed=1)
        path = os.path.join(tmp, "e2e_%s.txt" % name)
        with open(path, "wb") as f:
            f.write(text.tobytes())
        del text
        r = subprocess.run([exe, path, fmt, "3"], capture_output=True, text=True, timeout=600)
        if r.returncode:
            raise RuntimeError(r.stderr)
        line = json.loads(r.stdout)
        line["config"] = name
        # one more pass with the engine's per-stage times (DMLC_AMD_STATS): seconds summed over
        # batches; the reader, the workers' H2D / parse / D2H and the consumer overlap
        r2 = subprocess.run([exe, path, fmt, "3"], capture_output=True, text=True, timeout=600,
                            env=dict(os.environ, DMLC_AMD_STATS="1"))  # stats of the last (warm) pass
        st = [json.loads(x) for x in r2.stderr.splitlines() if x.startswith('{"dmlc_amd_stats"')]
        line["stages"] = st[-1]["dmlc_amd_stats"] if st else None
        td = [json.loads(x) for x in r2.stderr.splitlines() if x.startswith('{"dmlc_amd_teardown"')]
        line["teardown"] = td[-1]["dmlc_amd_teardown"] if td else None
        line["stages_pass_s"] = json.loads(r2.stdout)["best_s"] if r2.returncode == 0 else None
        line["cpu_reference"] = None
        try:
            from oracle import pyoracle as po
            if po.ref_available():
                # genuine reference, file -> Parser::Create -> full iteration, on a bounded sample
                srows = rows // 16
                stext, _ = synth.rows(synth.LIBSVM if fmt == "libsvm" else synth.CSV, srows, width, seed=1)
                spath = os.path.join(tmp, "e2e_%s_sample.txt" % name)
                with open(spath, "wb") as f:
                    f.write(stext.tobytes())
                t0 = time.perf_counter()
                po.ref_parse_uri(spath, 0, 1, fmt)
                dt = time.perf_counter() - t0
                line["cpu_reference"] = {"GBps": round(stext.size / dt / 1e9, 4), "bytes": int(stext.size),
                                         "rows": srows, "kind": "reference (oracle/_ref, Parser::Create, "
                                         "nthread cap min(max(nproc/2-4,1),2))"}
                os.remove(spath)
        except Exception as e:  # reported, never fatal
            line["cpu_reference"] = {"error": repr(e)}
        os.remove(path)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
