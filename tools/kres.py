"""Per-kernel resources from a hipcc -S listing (amdhsa metadata):
python tools/kres.py <file.s> [name-filter]"""
import re
import sys

s = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
meta = s[s.index("amdhsa.kernels:"):]
for blk in re.split(r"\n  - ", meta)[1:]:
    d = dict(re.findall(r"\.(\w+):\s+(\S+)", blk))
    name = d.get("name", "?")
    if flt in name:
        print("%-60s vgpr %3s sgpr %3s vspill %3s sspill %3s lds %6s scratch %4s" % (
            name[-60:], d.get("vgpr_count"), d.get("sgpr_count"), d.get("vgpr_spill_count"),
            d.get("sgpr_spill_count"), d.get("group_segment_fixed_size"), d.get("private_segment_fixed_size")))
