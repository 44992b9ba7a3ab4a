#!/usr/bin/env python3
"""VALU-fp64 roofline of qehvi_kernel at C4 from a rocprofv3 kernel-trace
--stats directory and a --pmc directory of the same tools/c4_qehvi.py command.

usage: python tools/qehvi_roofline.py OUT.json STATS_DIR PMC_DIR [cells]

algorithmic flops per forward launch:
b x S x (2^q - 1) x K x m x 3 (min over the subset, clip against the cell,
product of the m side lengths: about 3 flops per (sample, subset, cell,
output)); peak: 78.6 TFLOP/s fp64 vector (the MI355X fp64 VALU rate, the same
figure as the dense fp64 matrix peak).  The PMC pass counts executed fp64 VALU
instructions per wave (SQ_INSTS_VALU_{FMA,ADD,MUL,TRANS}_F64, summed over all
SQs); x 64 lanes, FMA x 2, gives the executed fp64 flops, which include the
kernel's own bookkeeping (the running subset minima, the sign fold)."""
import csv
import json
import os
import sys

B, Q, S, M = 128, 8, 128, 3
PEAK = 78.6e12


def main():
    out, stats_dir, pmc_dir = sys.argv[1:4]
    cells = int(sys.argv[4]) if len(sys.argv) > 4 else 294
    fwd_ns = bwd_ns = None
    for r in csv.DictReader(open(os.path.join(stats_dir, "run_kernel_stats.csv"))):
        if "qehvi_kernel" in r["Name"]:
            fwd_ns = float(r["AverageNs"])
        if "qehvi_backward" in r["Name"]:
            bwd_ns = float(r["AverageNs"])
    cnt = {}
    n_disp = {}
    for r in csv.DictReader(open(os.path.join(pmc_dir, "run_counter_collection.csv"))):
        nm = r["Kernel_Name"]
        if "qehvi_kernel" not in nm or "backward" in nm:
            continue
        c = r["Counter_Name"]
        cnt[c] = cnt.get(c, 0.0) + float(r["Counter_Value"])
        n_disp[c] = n_disp.get(c, 0) + 1
    per = {c: v / n_disp[c] for c, v in cnt.items()}
    alg = B * S * (2 ** Q - 1) * cells * M * 3
    res = {"kernel": "qehvi_kernel", "config": "C4 qEHVI ModelListGP(3) DTLZ2 n=2048 q=8 S=128 b=128",
           "cells": cells, "algorithmic_flops": alg, "avg_ns": fwd_ns, "backward_avg_ns": bwd_ns,
           "peak": PEAK, "unit": "TFLOP/s", "bound": "valu-fp64"}
    if fwd_ns:
        res["achieved_tflops"] = alg / (fwd_ns * 1e-9) / 1e12
        res["frac"] = alg / (fwd_ns * 1e-9) / PEAK
    if per:
        lanes = 64
        f64 = lanes * (2 * per.get("SQ_INSTS_VALU_FMA_F64", 0) + per.get("SQ_INSTS_VALU_ADD_F64", 0)
                       + per.get("SQ_INSTS_VALU_MUL_F64", 0) + per.get("SQ_INSTS_VALU_TRANS_F64", 0))
        res["pmc"] = per
        res["executed_valu_f64_flops"] = f64
        if fwd_ns:
            res["executed_tflops"] = f64 / (fwd_ns * 1e-9) / 1e12
            res["executed_frac"] = f64 / (fwd_ns * 1e-9) / PEAK
        if per.get("SQ_INSTS_VALU"):
            res["f64_share_of_valu_insts"] = (per.get("SQ_INSTS_VALU_FMA_F64", 0)
                                              + per.get("SQ_INSTS_VALU_ADD_F64", 0)
                                              + per.get("SQ_INSTS_VALU_MUL_F64", 0)
                                              + per.get("SQ_INSTS_VALU_TRANS_F64", 0)) / per["SQ_INSTS_VALU"]
        if per.get("SQ_BUSY_CYCLES") and per.get("SQ_ACTIVE_INST_VALU"):
            res["valu_active_per_busy"] = per["SQ_ACTIVE_INST_VALU"] / per["SQ_BUSY_CYCLES"]
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
