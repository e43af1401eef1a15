"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output (stdin):
one line per kernel with VGPRs, AGPRs, spills, scratch and occupancy."""
import re
import sys

cur = None
rows = []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    if cur is None:
        continue
    for key in ("VGPRs", "AGPRs", "VGPRs Spill", "ScratchSize \\[bytes/lane\\]", "Occupancy \\[waves/SIMD\\]"):
        m = re.search(r"remark:\s+" + key + r": (\d+)", line)
        if m:
            cur[key.split(" ")[0] + ("_spill" if "Spill" in key else "")] = int(m.group(1))
for r in rows:
    n = r["name"]
    print(f"{n[:70]:70s} vgpr {r.get('VGPRs', '?'):>3} agpr {r.get('AGPRs', '?'):>3} spill {r.get('VGPRs_spill', '?'):>3} "
          f"scratch {r.get('ScratchSize', '?'):>4} occ {r.get('Occupancy', '?')}")
