#!/bin/bash
# GPU-box: qmc_kernel's q x q Cholesky with the LDS column broadcast -- the
# acquisition / ladder tests, then qmc_kernel's time at C2 and C3 under
# rocprofv3 --kernel-trace --stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/ab_qmc
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_acquisition.py tests/test_gpu_full_configs.py tests/test_gpu_logei.py tests/test_gpu_graphs.py -q -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o run -- python3 tools/prof_small.py c2 > $O/c2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3 -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extra --no-bwd --no-fit > $O/c3.log 2>&1 || exit $?
for d in c2 c3; do
  python3 -c "
import csv
for r in csv.DictReader(open('$O/$d/run_kernel_stats.csv')):
    if 'qmc_kernel' in r['Name'] or 'post_partials' in r['Name'] or 'splitk' in r['Name']:
        print('$d', r['Name'][:60].replace('(anonymous namespace)::',''), r['Calls'], round(float(r['AverageNs'])/1e3, 2), 'us')"
done
grep '^{' $O/c3.log | cut -c1-200
find $O -name '*_trace.csv' -size +2M -delete
