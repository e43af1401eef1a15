"""Compare rocprofv3 kernel_stats CSVs: python tools/kstats.py A.csv [B.csv ...]
(per-kernel average us, nrk kernels with >= 20 calls)."""
import csv, re, sys
tabs = []
for f in sys.argv[1:]:
    d = {}
    for r in csv.DictReader(open(f)):
        if int(r["Calls"]) < 20:
            continue
        n = re.sub(r"\(.*", "", r["Name"]).replace("void ", "").replace("nrk::", "")
        d[n] = (float(r["AverageNs"]) / 1e3, int(r["Calls"]))
    tabs.append(d)
names = sorted(set().union(*tabs), key=lambda n: -max(t.get(n, (0, 0))[0] for t in tabs))
for n in names:
    print(f"{n[:70]:70s}", " ".join(f"{t[n][0]:7.2f}({t[n][1]:3d})" if n in t else "      -     " for t in tabs))
print(f"{'sum of averages':70s}", " ".join(f"{sum(v[0] for v in t.values()):7.2f}     " for t in tabs))
