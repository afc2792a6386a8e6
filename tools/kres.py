#!/usr/bin/env python
"""Compile one .hip file for gfx950 and print per-kernel VGPR / AGPR / spill / LDS / occupancy.

usage: python tools/kres.py csrc/kernels/conv.hip [name-filter]
"""
import re
import subprocess
import sys


def main():
    src = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-munsafe-fp-atomics", "-fPIC", "-c",
           src, "-o", "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    cur, rows = None, []
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        if cur is None:
            continue
        for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("spill", r"VGPRs Spill: (\d+)"),
                         ("lds", r"LDS Size \[bytes/block\]: (\d+)"), ("occ", r"Occupancy \[waves/SIMD\]: (\d+)")):
            m = re.search(pat, line)
            if m:
                cur[key] = int(m.group(1))
        if "error" in line:
            print(line)
    for r in rows:
        if filt in r["name"]:
            dm = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
            dm = re.sub(r"\(.*", "", dm)
            print(f"{r.get('vgpr', 0):4d}v {r.get('agpr', 0):3d}a spill {r.get('spill', 0):3d} lds {r.get('lds', 0):6d} "
                  f"occ {r.get('occ', 0):2d}  {dm}")


if __name__ == "__main__":
    main()
