#!/bin/bash
# GPU-box: post_small_kernel with 0 / 24 KB of LDS padding (BO_SMALL_LDS_PAD:
# one workgroup per CU) -- kernel stats of tools/prof_small.py c2 and the C2 bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/ab_small_pad
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
for v in 0 24576; do
  (cd /tmp && BO_SMALL_LDS_PAD=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p${v}_$r -o run -- python3 $R/tools/prof_small.py c2 > $O/p${v}_$r.log 2>&1) || exit 1
  python3 -c "
import csv,glob
f=glob.glob('$O/p${v}_$r/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'post_small' in r['Name']: print('pad=$v', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,2))"
done
done
