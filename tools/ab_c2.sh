#!/bin/bash
# GPU-box: C2 eager forward under A/B knobs: the R route's stream-K minimum
# share (BO_SK_MIN_SHARE) and the quad plan -- wall ms per call and
# per-kernel average durations.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/ab_c2b
mkdir -p $O
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 120 python tools/prof_small.py c2 > $O/$tag.plain 2>&1 || exit $?
  env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$tag -o run --output-format csv -- python tools/prof_small.py c2 > $O/$tag.log 2>&1 || exit $?
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
run quad BO_POST_QUAD=auto
for sh in 4 8 16 32 64; do run r_sk$sh BO_POST_QUAD=0 BO_SK_MIN_SHARE=$sh; done
