#!/bin/bash
# GPU-box: the Cholesky tests, the DAG Cholesky timed and traced, and the
# diagonal-tile probe (column-owner variants against the four-panel form).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab_potrf
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_chol_dag.py tests/test_gpu_chol_batched.py -q -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 1; do
  timeout -k 10 120 python tools/time_chol_batched.py > $O/time_$v.json 2>&1 || exit $?
  echo "rows=$v $(cat $O/time_$v.json | tail -1)"
done
for v in 1; do
  timeout -k 10 120 python tools/trace_chol.py > $O/trace_$v.json 2>&1 || exit $?
  python3 tools/trace_summary.py $O/trace_$v.json rows=$v
done
timeout -k 10 60 python tools/probe_potrf64.py > $O/probe.json 2>&1 || exit $?
tail -1 $O/probe.json
