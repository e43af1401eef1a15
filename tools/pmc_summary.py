"""Summarise tools/pmc_sq.sh output: per kernel (name filter), the mean of
every counter over its dispatches, and the derived fractions of wave time
(SQ_WAVE_CYCLES = WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY, quad-cycles).
usage: python tools/pmc_summary.py gpurun_out/pmc_TAG [kernel-substring]"""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "din_rerank"
vals = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if pat in r["Kernel_Name"]:
                k = r["Kernel_Name"][:60]
                vals[k][(r["Counter_Name"], r["Dispatch_Id"])].append(float(r["Counter_Value"]))
for k, d in vals.items():
    per = defaultdict(list)
    for (c, _disp), v in d.items():
        per[c].append(sum(v))  # sum over XCD / SE instances of one dispatch
    mean = {c: sum(v) / len(v) for c, v in per.items()}
    print(k)
    for c in sorted(mean):
        print(f"  {c:28s} {mean[c]:16.1f}  (n={len(per[c])})")
    wc = mean.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                  "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_MISC"):
            if c in mean:
                print(f"  {c:28s} {mean[c] / wc:7.3f} of wave cycles")
