#!/bin/bash
# GPU-box: C2 eager forward with two builds of libbotorch_amd.so (ab_libs/libA.so
# = before, libB.so = after), interleaved twice: wall ms per call and the
# per-kernel average durations.  Leaves libB.so in place.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/ab_lib_c2
mkdir -p $O
run() {  # tag
  local tag=$1
  cp ab_libs/lib${tag%%_*}.so botorch_amd/libbotorch_amd.so
  timeout -k 10 120 python tools/prof_small.py c2 > $O/$tag.plain 2>&1 || exit $?
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$tag -o run --output-format csv -- python tools/prof_small.py c2 > $O/$tag.log 2>&1 || exit $?
  echo "$tag $(grep 'C2 ms' $O/$tag.plain)"
  python - "$O/$tag/run_kernel_stats.csv" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(\w+_kernel)", r["Name"])
    if m and int(r["Calls"]) > 20:
        print("   %-32s n=%4s %8.1f us" % (m.group(1), r["Calls"], float(r["AverageNs"]) / 1e3))
PY
  find $O/$tag -name '*_trace.csv' -delete
}
for rep in 1 2; do run A_$rep; run B_$rep; done
cp ab_libs/libB.so botorch_amd/libbotorch_amd.so
