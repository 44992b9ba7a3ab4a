#!/usr/bin/env python3
"""One-line summary of a tools/trace_chol.py output file (its last line):
span, CRIT phase means and every sixth diagonal step's duration."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
tag = sys.argv[2] if len(sys.argv) > 2 else ""
print(tag, "span", d["span_us"], "crit", {k: round(x, 2) for k, x in d["crit_phase_us_mean"].items()},
      "pre", round(d["crit_pre_us_mean"], 1))
print([x[4] for x in d["crit_k_start_end_dur_step"][1::6]])
