#!/bin/bash
# GPU-box: C3 forward bench with two builds of libbotorch_amd.so (ab_libs/libA.so
# = before, libB.so = after), interleaved twice: ms per step and the
# qmc_kernel / post_partials average durations.  Leaves libB.so in place.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/ab_lib_c3
mkdir -p $O
run() {  # tag
  local tag=$1
  cp ab_libs/lib${tag%%_*}.so botorch_amd/libbotorch_amd.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$tag -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra --no-bwd --no-fit > $O/$tag.log 2>&1 || exit $?
  python3 - "$O/$tag" <<'PY'
import csv, json, re, sys
d = sys.argv[1]
line = [l for l in open(d + ".log") if l.startswith("{")][-1]
out = [d.split("/")[-1], "ms_per_step %.4f" % json.loads(line)["ms_per_step"]]
for r in csv.DictReader(open(d + "/run_kernel_stats.csv")):
    m = re.search(r"(qmc_kernel|post_partials_kernel|kxt_build_kernel)", r["Name"])
    if m and int(r["Calls"]) >= 20:
        out.append("%s %.1f us" % (m.group(1), float(r["AverageNs"]) / 1e3))
print("  ".join(out))
PY
  find $O/$tag -name '*_trace.csv' -delete
}
for rep in 1 2; do run A_$rep; run B_$rep; done
cp ab_libs/libB.so botorch_amd/libbotorch_amd.so
