#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs per kernel into one JSON file.

usage: python tools/pmc_summary.py [--meta key=value ...] OUT.json DIR [DIR ...]
``_meta`` records the creation time and the --meta pairs (bench.py reads
``restarts``: the launch size the passes ran at).  Each DIR holds a run_counter_collection.csv from one `rocprofv3 --pmc ...`
pass (FETCH_SIZE and WRITE_SIZE need separate passes on gfx950).

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half of the bytes of a wide coalesced read, so it
is doubled; WRITE_SIZE is taken as is.  MFMA utilisation =
SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x GRBM_GUI_ACTIVE / XCDs) (GRBM_GUI_ACTIVE is
summed over the 8 XCDs; MFMA busy cycles over all 1024 SIMDs).
"""
import collections
import csv
import json
import os
import re
import sys
import time

SIMDS, XCDS = 1024, 8


def short(name: str) -> str:
    m = re.search(r"(\w+_kernel(?:<[^>(]*>)?)", name)
    return m.group(1) if m else name.split("(")[0][-60:]


def main():
    argv = sys.argv[1:]
    meta = {"created": time.time()}
    while argv and argv[0] == "--meta":
        k, v = argv[1].split("=", 1)
        meta[k] = int(v) if v.isdigit() else v
        argv = argv[2:]
    out, dirs = argv[0], argv[1:]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        path = os.path.join(d, "run_counter_collection.csv")
        for r in csv.DictReader(open(path)):
            agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    summary = {}
    for k, cs in agg.items():
        e = {c: sum(v) / len(v) for c, v in cs.items()}
        e["dispatches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in e:
            e["hbm_read_bytes"] = e["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in e:
            e["hbm_write_bytes"] = e["WRITE_SIZE"] * 1024
        if "hbm_read_bytes" in e and "hbm_write_bytes" in e:
            e["hbm_bytes"] = e["hbm_read_bytes"] + e["hbm_write_bytes"]
        if "SQ_VALU_MFMA_BUSY_CYCLES" in e and e.get("GRBM_GUI_ACTIVE"):
            e["mfma_util"] = e["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * e["GRBM_GUI_ACTIVE"] / XCDS)
        summary[k] = e
    summary["_meta"] = meta
    json.dump(summary, open(out, "w"), indent=1, sort_keys=True)
    for k, e in sorted(((k, e) for k, e in summary.items() if k != "_meta"),
                       key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0)):
        print(f"{k:50s} n={e['dispatches']:4d} hbm={e.get('hbm_bytes', 0) / 1e6:10.2f} MB "
              f"mfma={e.get('mfma_util', float('nan')):.3f}")


if __name__ == "__main__":
    main()
