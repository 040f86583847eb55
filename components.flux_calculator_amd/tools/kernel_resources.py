#!/usr/bin/env python3
"""VGPRs / scratch / occupancy of every kernel in fcx_kernels.hip (compiler remarks).

  python tools/kernel_resources.py [filter]
"""
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "..", "csrc", "fcx_kernels.hip")
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
       "-I" + os.path.join(HERE, "..", "csrc"), "-I" + os.path.join(HERE, "..", "..", "include"), "-c", SRC,
       "-o", "/tmp/fcx_kernels_res.o", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[2:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur, rows = None, []
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
        continue
    for key, pat in (("vgpr", r" VGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                     ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
        m = re.search(pat, line)
        if m and cur is not None:
            cur[key] = int(m.group(1))
flt = sys.argv[1] if len(sys.argv) > 1 else ""
for r in rows:
    if flt in r["name"]:
        print(f"{r.get('vgpr', '?'):>4} vgpr {r.get('scratch', '?'):>4} scratch {r.get('occ', '?'):>2} waves "
              f"{r.get('lds', 0):>6} lds  {r['name'].split('(')[0]}")
