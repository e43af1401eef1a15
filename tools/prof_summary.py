#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output into profiles/.

  python tools/prof_summary.py --stats DIR/trace_kernel_stats.csv \
      --fetch DIR/pmc_counter_collection.csv --write DIR2/pmc_counter_collection.csv \
      --out profiles/r01_... [--key "nb=...,gpus=1"]

HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE come from separate --pmc passes (TCC slots), both in KB; on gfx950
FETCH_SIZE reports 1/2 of the bytes of wide coalesced streaming reads, so it
is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.
"""
import argparse
import collections
import csv
import json
import re


def short(name):
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "").replace("nrk::", "")


def pmc(path, counter):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            per[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stats")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--out", required=True)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    summary = {}
    if a.stats:
        rows = list(csv.DictReader(open(a.stats)))
        summary["kernel_stats"] = [
            {"kernel": short(r["Name"]), "calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
             "min_us": float(r["MinNs"]) / 1e3, "max_us": float(r["MaxNs"]) / 1e3, "pct": float(r["Percentage"])}
            for r in rows[: a.top]]
    if a.fetch or a.write:
        f = pmc(a.fetch, "FETCH_SIZE") if a.fetch else {}
        w = pmc(a.write, "WRITE_SIZE") if a.write else {}
        summary["hbm_per_launch"] = {
            k: {"FETCH_SIZE_KB": f.get(k), "WRITE_SIZE_KB": w.get(k),
                "hbm_bytes_corrected": (2 * 1024 * f.get(k, 0.0)) + 1024 * w.get(k, 0.0)}
            for k in sorted(set(f) | set(w))}
    json.dump(summary, open(a.out, "w"), indent=1)
    print(json.dumps(summary, indent=1)[:3000])


if __name__ == "__main__":
    main()
