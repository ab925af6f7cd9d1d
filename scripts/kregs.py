"""Register usage per kernel from a hipcc -S (--cuda-device-only) listing: python scripts/kregs.py x.s [filter]"""
import re
import sys

s = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
meta = s[s.index("amdhsa.kernels"):]
for blk in re.split(r"\n  - \.", meta)[1:]:
    m = re.search(r"\.name:\s+(\S+)", blk)
    if not m or flt not in m.group(1):
        continue
    g = lambda k: (re.search(r"\." + k + r":\s+(\d+)", blk) or [None, "?"])[1]
    print(f"{m.group(1)[:60]:60s} vgpr={g('vgpr_count')} agpr={g('agpr_count')} sgpr={g('sgpr_count')} "
          f"vspill={g('vgpr_spill_count')} sspill={g('sgpr_spill_count')} lds={g('group_segment_fixed_size')}")
