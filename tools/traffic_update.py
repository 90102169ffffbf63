"""Record a PMC-measured HBM traffic figure in profiles/traffic.json together
with the build it was measured on (bench.py prices roofline.traffic from it
and says whether that build is the one running).
usage: python tools/traffic_update.py <config> <summary.json> <pmc bench log>
  summary.json: tools/summarize_prof.py output (hbm_bytes_per_launch.total,
  dominant_kernel); the log: a PMC pass's bench.py output (its JSON line
  carries the build id)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(cfg, summ, log):
    s = json.load(open(summ))
    line = [ln for ln in open(log) if ln.startswith("{")][-1]
    b = json.loads(line)
    path = os.path.join(ROOT, "profiles", "traffic.json")
    t = json.load(open(path))
    t[cfg] = {"kernel": s["dominant_kernel"], "hbm_bytes_per_launch": s["hbm_bytes_per_launch"]["total"],
              "build": b.get("build"),
              "source": "%s (tools/gpu_pmc.sh: FETCH_SIZE x2 + WRITE_SIZE, KiB->B, gfx950 correction per "
                        "MI355X_MICROARCH.md)" % os.path.relpath(summ, ROOT)}
    json.dump(t, open(path, "w"), indent=1)
    print(cfg, t[cfg])


if __name__ == "__main__":
    main(*sys.argv[1:4])
