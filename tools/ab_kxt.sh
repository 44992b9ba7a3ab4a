#!/bin/bash
# A/B of kxt_build_kernel's training points per thread (tools/ab/lib_k{16,32,64}.so:
# the library relinked with post.hip built with -DKXT_K=16/32/64): kernel stats
# of the forward-only bench for each.  Measured 76.7 / 77.8 / 78.5 us: no effect.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/kxt
for K in 16 32 64; do
  cp tools/ab/lib_k$K.so botorch_amd/libbotorch_amd.so || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kxt/k$K -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extra --no-bwd --no-fit > gpurun_out/kxt/k$K.log 2>&1 || exit $?
  python3 - "$K" <<'PY'
import csv, json, sys
K = sys.argv[1]
rows = list(csv.DictReader(open(f"gpurun_out/kxt/k{K}/run_kernel_stats.csv")))
kx = [r for r in rows if "kxt_build" in r["Name"]]
pp = [r for r in rows if "post_partials_kernel<0, 6, false" in r["Name"]]
line = [l for l in open(f"gpurun_out/kxt/k{K}.log") if l.startswith("{")][-1]
d = json.loads(line)
print(K, "kxt_us", round(float(kx[0]["AverageNs"]) / 1e3, 1), "pp_us", round(float(pp[0]["AverageNs"]) / 1e3, 1), "ms_per_step", round(d["ms_per_step"], 4))
PY
done
find gpurun_out/kxt -name '*_trace.csv' -delete
