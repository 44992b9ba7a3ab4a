#!/usr/bin/env python3
"""Print the kernel timeline of one bo_cholesky_inverse call from a rocprofv3
kernel trace (the last call: from its last potrf_block #0 on)."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "potrf_block" in r["Kernel_Name"]]
# the start of a call: a potrf launch preceded by a non-potrf/non-gemm kernel (memset)
starts = [i for i in idx if i > 0 and "gemm" not in rows[i - 1]["Kernel_Name"]
          and "potrf" not in rows[i - 1]["Kernel_Name"]]
which = int(sys.argv[2]) if len(sys.argv) > 2 else -1
s = starts[which]
e = starts[which + 1] if which + 1 < len(starts) and which != -1 else len(rows)
t0 = int(rows[s]["Start_Timestamp"])
tot = {}
for r in rows[s:e]:
    name = re.sub(r"\(.*", "", r["Kernel_Name"])[:60]
    st, en = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    grid = f'{r["Grid_Size_X"]}x{r["Grid_Size_Y"]}'
    if len(sys.argv) > 3:
        print(f"{st/1e3:9.1f} {en/1e3:9.1f} {(en-st)/1e3:7.1f}us q{r['Queue_Id']} {grid:>12} {name}")
    tot.setdefault(name, [0, 0.0])
    tot[name][0] += 1
    tot[name][1] += (en - st) / 1e3
last = max(int(r["End_Timestamp"]) for r in rows[s:e]) - t0
print(f"span {last/1e3:.1f} us")
for k, (c, t) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
    print(f"{t:9.1f} us  {c:4d}x  {k}")
