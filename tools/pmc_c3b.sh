#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the C3 forward alone at several t-batch counts
# (tools/c3_fwd.py), one summary per count: how the posterior GEMM's HBM
# traffic scales with the K*x^T row stride.  usage: tools/pmc_c3b.sh "512 576"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-pmc_c3b}
mkdir -p $O
for b in $1; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $O/b${b}_$c -o run -- python3 tools/c3_fwd.py 3 $b > $O/b${b}_$c.log 2>&1 || exit 1
  done
  python3 tools/pmc_summary.py --meta restarts=$b $O/b$b.json $O/b${b}_FETCH_SIZE $O/b${b}_WRITE_SIZE > /dev/null || exit 1
  find $O -name 'run_counter_collection.csv' -size +2M -delete
  python3 -c "
import json; d = json.load(open('$O/b$b.json'))
for k, e in d.items():
    if k.startswith('post_partials'): print($b, k, e['dispatches'], round(e['hbm_bytes'] / 1e9, 3))"
done
