"""Print the kernel timeline of one step from a rocprofv3 kernel_trace.csv:
the kernels between the N-th and (N+1)-th launch of a marker kernel
(development tool).  argv: trace.csv marker N"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if sys.argv[2] in r["Kernel_Name"]]
n = int(sys.argv[3])
a, b = idx[n], idx[n + 1]
t0 = int(rows[a + 1]["Start_Timestamp"])
busy = 0
for r in rows[a + 1:b + 1]:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    e = (int(r["End_Timestamp"]) - t0) / 1e3
    busy += e - s
    print(f"{s:8.1f} {e:8.1f} {e - s:7.1f} g={r['Grid_Size_X']:>7} {r['Kernel_Name'][:70]}")
print("period", (int(rows[b]["End_Timestamp"]) - int(rows[a]["End_Timestamp"])) / 1e3, "busy", round(busy, 1))
