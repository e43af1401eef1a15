#!/usr/bin/env python3
"""Summarise hipcc per-kernel resource remarks: python tools/resources.py file.hip [hipcc flags]"""
import re, subprocess, sys
f, extra = sys.argv[1], sys.argv[2:]
out = subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", f, "-o", "/tmp/_res.o",
                      "-Rpass-analysis=kernel-resource-usage", *extra], capture_output=True, text=True).stderr
cur = {}
for line in out.splitlines():
    m = re.search(r"remark: +(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
    if m:
        key, val = m.group(1).split()[0], m.group(2)
        if key == "Function":
            if cur: print(cur)
            cur = {"fn": re.sub(r"^_ZN3nrk\d+", "", val)[:70]}
        else:
            cur[key] = val
    elif "error" in line:
        print(line)
if cur: print(cur)
