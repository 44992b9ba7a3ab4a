"""Kernel stats (calls, total / average / min / max ns, share) from a rocprofv3
rocpd SQLite database (development tool; the same columns as --stats'
kernel_stats.csv).  Usage: rocpd_stats.py results.db [out.csv]"""
import csv
import sqlite3
import sys


def stats(db):
    con = sqlite3.connect(db)
    tabs = [r[0] for r in con.execute("select name from sqlite_master where type='table'")]
    disp = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
    sym = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
    cols = [r[1] for r in con.execute(f"pragma table_info({sym})")]
    name_col = "kernel_name" if "kernel_name" in cols else ("display_name" if "display_name" in cols else "name")
    rows = con.execute(f"select s.{name_col}, d.end - d.start from {disp} d join {sym} s "
                       f"on d.kernel_id = s.id").fetchall()
    agg = {}
    for name, dur in rows:
        a = agg.setdefault(name, [0, 0, None, 0])
        a[0] += 1
        a[1] += dur
        a[2] = dur if a[2] is None else min(a[2], dur)
        a[3] = max(a[3], dur)
    total = sum(a[1] for a in agg.values()) or 1
    out = [(n, a[0], a[1], a[1] / a[0], 100.0 * a[1] / total, a[2], a[3]) for n, a in agg.items()]
    out.sort(key=lambda r: -r[2])
    return out


if __name__ == "__main__":
    res = stats(sys.argv[1])
    w = csv.writer(open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for r in res:
        w.writerow(r)
