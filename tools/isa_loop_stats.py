#!/usr/bin/env python3
"""Instruction mix of the main (LDS-DMA issuing) loop of kernels in a hipcc -save-temps .s file.
usage: python tools/isa_loop_stats.py FILE.s NAME_SUBSTRING"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
for n in sorted(set(re.findall(r"^(_Z\w+):", s, re.M))):
    if sys.argv[2] not in n:
        continue
    i = s.index(n + ":")
    j = s.index(".Lfunc_end", i)
    body = s[i:j].split("\n")
    seg = s[s.find(".amdhsa_kernel " + n):][:4000]
    best = None
    for k, l in enumerate(body):
        if "Loop Header" not in l:
            continue
        hdr = l.split(":")[0]
        be = [m for m, x in enumerate(body) if hdr in x and ("s_cbranch" in x or "s_branch" in x) and m > k]
        if not be:
            continue
        loop = body[k:be[-1] + 1]
        if any("global_load_lds" in x for x in loop) and (best is None or len(loop) > len(best)):
            best = loop
    c = collections.Counter()
    for l in best or []:
        t = l.strip().split()
        if not t or t[0].startswith(";") or t[0].startswith("."):
            continue
        op = t[0]
        key = ("mfma" if op.startswith("v_mfma") else "acc" if op.startswith("v_accvgpr") else "valu" if op.startswith("v_")
               else "ds" if op.startswith("ds_") else "wait" if op == "s_waitcnt" else "salu" if op.startswith("s_") else op)
        c[key] += 1
    print(n[:60], "vgpr", re.findall(r"\.amdhsa_next_free_vgpr (\d+)", seg), "scratch",
          re.findall(r"private_segment_fixed_size (\d+)", seg), dict(c))
