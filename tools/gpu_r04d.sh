#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04d
mkdir -p $O
timeout -k 10 200 python3 tools/time_qmc_phases.py > $O/qmc_phases.log 2>&1 || exit $?
cat $O/qmc_phases.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
tail -3 $O/pytest.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o run -- python3 tools/prof_small.py c2 > $O/c2.log 2>&1 || exit $?
grep -h "qmc_kernel\|post_partials\|splitk\|kxt" $O/c2/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
grep "C2 ms" $O/c2.log
