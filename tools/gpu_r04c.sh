#!/bin/bash
# joint L-BFGS-B after the wide paths: phase clocks, then its GPU tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 300 python3 tools/prof_lbfgsb_joint.py > $O/lbfgsb_joint.log 2>&1 || exit $?
cat $O/lbfgsb_joint.log
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_lbfgsb.py tests/test_gpu_fit_optim.py tests/test_gpu_c1_end_to_end.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
tail -5 $O/pytest.log
