"""Print per-kernel VGPR/AGPR/SGPR/LDS/scratch usage from a gfx950 .s (hipcc --save-temps)."""
import re
import sys

text = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
meta = text[text.find("amdhsa.kernels:"):]
for blk in meta.split("\n  - ")[1:]:
    d = dict(re.findall(r"^\s+\.(\w+):\s+(\S+)", blk, re.M))
    name = d.get("name", "?")
    if pat and not re.search(pat, name):
        continue
    print(f"{d.get('vgpr_count','?'):>4} v {d.get('agpr_count','?'):>4} a {d.get('sgpr_count','?'):>4} s "
          f"{d.get('group_segment_fixed_size','?'):>6} lds {d.get('private_segment_fixed_size','?'):>4} scr  {name[:110]}")
