#!/bin/bash
# Cholesky: depth-2 prefetch of the batched updates -- tests, then interleaved A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_chol_dag.py tests/test_gpu_chol_batched.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest_chol.log 2>&1
rc=$?; tail -3 $O/pytest_chol.log
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2 3; do
  BO_CHOL_PREFETCH2=0 timeout -k 10 120 python3 tools/chol_time.py >> $O/ab.log 2>&1 || exit $?
  BO_CHOL_PREFETCH2=1 timeout -k 10 120 python3 tools/chol_time.py >> $O/ab.log 2>&1 || exit $?
done
grep '^{' $O/ab.log
