#!/usr/bin/env python3
"""Roofline of qehvi_kernel at C4 from EXECUTED work: a rocprofv3 kernel-trace
--stats directory and a --pmc directory of the same tools/c4_qehvi.py command.

usage: python tools/qehvi_roofline.py OUT.json STATS_DIR PMC_DIR [cells]

The kernel prunes: a (sample, subset, cell) term whose subset holds a point
with an empty box in the cell is skipped (the reference's dense sum minus exact
zeros), so the dense count b x S x (2^q - 1) x K x m x 3 is NOT work the kernel
does and is reported only as ``dense_flops`` (no fraction is taken of it).
What bounds the kernel is VALU issue -- most of its instructions are integer
and control (subset masks, min/max bookkeeping); fp64 arithmetic is a small
share -- so the roofline is the VALU pipe:

* executed VALU wave-instructions per launch = SQ_INSTS_VALU (summed over the
  SQs), of which SQ_INSTS_VALU_{FMA,ADD,MUL,TRANS}_F64 are fp64;
* issue cycles: a wave64 32-bit VALU instruction occupies its SIMD 2 cycles
  (MI355X_MICROARCH.md, 32 lanes/cycle), an fp64 one 4 (the 78.6 TFLOP/s fp64
  vector rate = 16 FMA lanes/cycle/SIMD);
* peak = 1024 SIMDs x 2.4 GHz of issue cycles; frac = executed issue cycles /
  (peak x average launch time).
Executed fp64 flops (x 64 lanes, FMA x 2) are reported beside it against the
78.6 TFLOP/s fp64 vector peak."""
import csv
import json
import os
import sys

B, Q, S, M = 128, 8, 128, 3
SIMDS, CLOCK = 1024, 2.4e9
PEAK_F64 = 78.6e12
F64 = ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
       "SQ_INSTS_VALU_TRANS_F64")


def main():
    out, stats_dir, pmc_dir = sys.argv[1:4]
    cells = int(sys.argv[4]) if len(sys.argv) > 4 else 294
    fwd_ns = bwd_ns = None
    for r in csv.DictReader(open(os.path.join(stats_dir, "run_kernel_stats.csv"))):
        if "qehvi_kernel" in r["Name"]:
            fwd_ns = float(r["AverageNs"])
        if "qehvi_backward" in r["Name"]:
            bwd_ns = float(r["AverageNs"])
    cnt, n_disp = {}, {}
    for r in csv.DictReader(open(os.path.join(pmc_dir, "run_counter_collection.csv"))):
        nm = r["Kernel_Name"]
        if "qehvi_kernel" not in nm or "backward" in nm:
            continue
        c = r["Counter_Name"]
        cnt[c] = cnt.get(c, 0.0) + float(r["Counter_Value"])
        n_disp[c] = n_disp.get(c, 0) + 1
    per = {c: v / n_disp[c] for c, v in cnt.items()}
    res = {"kernel": "qehvi_kernel", "config": "C4 qEHVI ModelListGP(3) DTLZ2 n=2048 q=8 S=128 b=128",
           "cells": cells, "avg_ns": fwd_ns, "backward_avg_ns": bwd_ns, "bound": "valu-issue",
           "dense_flops": B * S * (2 ** Q - 1) * cells * M * 3,
           "dense_flops_note": "the reference's dense inclusion-exclusion count; the kernel skips "
                               "empty-box terms, so this is not executed work"}
    if per:
        n_valu = per.get("SQ_INSTS_VALU", 0.0)
        n_f64 = sum(per.get(c, 0.0) for c in F64)
        issue = 2.0 * (n_valu - n_f64) + 4.0 * n_f64
        f64_flops = 64 * (2 * per.get("SQ_INSTS_VALU_FMA_F64", 0) + per.get("SQ_INSTS_VALU_ADD_F64", 0)
                          + per.get("SQ_INSTS_VALU_MUL_F64", 0) + per.get("SQ_INSTS_VALU_TRANS_F64", 0))
        res.update(pmc=per, executed_valu_insts=n_valu, executed_valu_f64_insts=n_f64,
                   f64_share_of_valu_insts=n_f64 / n_valu if n_valu else None,
                   executed_issue_cycles=issue, executed_valu_f64_flops=f64_flops,
                   peak_issue_cycles_per_s=SIMDS * CLOCK, unit="VALU issue cycles/s")
        if fwd_ns:
            t = fwd_ns * 1e-9
            res["achieved"] = issue / t
            res["peak"] = SIMDS * CLOCK
            res["frac"] = issue / t / (SIMDS * CLOCK)
            res["executed_f64_tflops"] = f64_flops / t / 1e12
            res["executed_f64_frac"] = f64_flops / t / PEAK_F64
        if per.get("SQ_BUSY_CYCLES") and per.get("SQ_ACTIVE_INST_VALU"):
            res["valu_active_per_busy"] = per["SQ_ACTIVE_INST_VALU"] / per["SQ_BUSY_CYCLES"]
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
