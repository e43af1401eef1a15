#!/usr/bin/env python3
"""Print the kernels of one graph-replayed step from a rocprofv3 kernel trace.
usage: python tools/step_breakdown.py TRACE.csv LAST_KERNEL_SUBSTRING"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
key = sys.argv[2]
names = [re.sub(r"\(.*", "", r["Kernel_Name"]) for r in rows]
idx = [i for i, n in enumerate(names) if key in n]
i1, i2 = idx[-2], idx[-1]
t0 = int(rows[i1]["End_Timestamp"])
tot = 0.0
for i in range(i1 + 1, i2 + 1):
    dur = (int(rows[i]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"])) / 1e3
    tot += dur
    print(f"{names[i][:64]:64s} {dur:8.1f} us  start+{(int(rows[i]['Start_Timestamp']) - t0) / 1e3:8.1f}")
print(f"sum of kernel durations {tot:.1f} us; step span {(int(rows[i2]['End_Timestamp']) - t0) / 1e3:.1f} us")
