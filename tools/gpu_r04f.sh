#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 200 python3 tools/time_qmc_phases.py > $O/qmc_phases.log 2>&1 || exit $?
cat $O/qmc_phases.log
timeout -k 10 200 python3 tools/host_eager.py > $O/host_eager.log 2>&1 || exit $?
cat $O/host_eager.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
tail -3 $O/pytest.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o run -- python3 tools/prof_small.py c2 > $O/c2.log 2>&1 || exit $?
grep "C2 ms" $O/c2.log
timeout -k 10 100 python3 tools/prof_small.py c2 > $O/c2_plain.log 2>&1 || exit $?
grep "C2 ms" $O/c2_plain.log
