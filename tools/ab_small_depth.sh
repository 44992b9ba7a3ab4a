#!/bin/bash
# GPU-box: post_small_kernel with 2 (ab_libs/libD2.so) vs 3 (libD3.so) k-steps of
# operands in flight: kernel stats of tools/prof_small.py c2, the small-route tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/ab_small_depth
mkdir -p $O
cp botorch_amd/libbotorch_amd.so ab_libs/libORIG.so
cp ab_libs/libD3.so botorch_amd/libbotorch_amd.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_post_small.py tests/test_gpu_post_members.py > $O/tests_D3.log 2>&1 || { cp ab_libs/libORIG.so botorch_amd/libbotorch_amd.so; exit 1; }
export TMPDIR=/tmp
for r in 1 2; do
for v in D2 D3; do
  cp $R/ab_libs/lib$v.so $R/botorch_amd/libbotorch_amd.so
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${v}_$r -o run -- python3 $R/tools/prof_small.py c2 > $O/${v}_$r.log 2>&1) || exit 1
  python3 -c "
import csv,glob
f=glob.glob('$O/${v}_$r/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'post_small' in r['Name'] or 'qmc_kernel' in r['Name'] or 'kxt' in r['Name']: print('$v', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,2))"
done
done
cp ab_libs/libORIG.so botorch_amd/libbotorch_amd.so
