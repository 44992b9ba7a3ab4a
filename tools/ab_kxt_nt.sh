#!/bin/bash
# K*x^T build with plain vs nontemporal stores (BO_KXT_NT): kernel stats of the
# forward-only C3 bench, interleaved twice.  The knob was reverted after this
# A/B (80.0/80.1 us plain, 80.2/80.1 us nontemporal; profiles/r04/kxt_nt), so
# on the current tree both legs run the plain store.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/kxt_nt; mkdir -p $O
for rep in 1 2; do
  for nt in 0 1; do
    BO_KXT_NT=$nt timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/nt${nt}_$rep -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extra --no-bwd --no-fit > $O/nt${nt}_$rep.log 2>&1 || exit $?
    python3 - "$O/nt${nt}_$rep" <<'PY'
import csv, json, sys
d = sys.argv[1]
rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
kx = [r for r in rows if "kxt_build" in r["Name"]]
pp = [r for r in rows if "post_partials_kernel<0, 6, false" in r["Name"]]
line = [l for l in open(d + ".log") if l.startswith("{")][-1]
print(d, "kxt_us", round(float(kx[0]["AverageNs"]) / 1e3, 1), "pp_us", round(float(pp[0]["AverageNs"]) / 1e3, 1),
      "ms_per_step", round(json.loads(line)["ms_per_step"], 4))
PY
  done
done
find $O -name '*_trace.csv' -delete
