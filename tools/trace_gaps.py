#!/usr/bin/env python3
"""Per-kernel durations and the idle gaps before each launch, from a
rocprofv3 kernel_trace.csv: the last ``n`` dispatches (a steady-state loop)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
tail = rows[-n:]
prev_end = None
for r in tail:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    print(f"{r['Kernel_Name'][:70]:70s} dur {(e - s) / 1e3:8.2f} us  gap {gap:8.2f} us  grid {r.get('Grid_Size_X', r.get('Grid_Size', ''))}")
    prev_end = e
span = (int(tail[-1]["End_Timestamp"]) - int(tail[0]["Start_Timestamp"])) / 1e3
print(f"span of the last {n} dispatches: {span:.1f} us")
