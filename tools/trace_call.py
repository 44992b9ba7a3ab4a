#!/usr/bin/env python3
"""One call's kernel sequence from a rocprofv3 kernel_trace.csv: the kernels
between the last two launches whose name contains ``anchor`` (one per call),
with start offsets, durations and the idle gap before each (development
tool).  argv: trace.csv anchor."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if sys.argv[2] in r["Kernel_Name"]]
a, b = idx[-2], idx[-1]
win = rows[a:b]
t0 = int(win[0]["Start_Timestamp"])
prev = None
busy = 0
for r in win:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    busy += e - s
    print(f"{(s - t0) / 1e3:9.1f} gap {gap:7.1f} dur {(e - s) / 1e3:7.1f}  {r['Kernel_Name'][:90]}")
    prev = e
span = int(rows[b]["Start_Timestamp"]) - t0
print(f"call span {span / 1e3:.1f} us, kernels {busy / 1e3:.1f} us, idle {(span - busy) / 1e3:.1f} us")
