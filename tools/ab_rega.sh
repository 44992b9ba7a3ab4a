#!/bin/bash
# GPU-box: register-operand batched updates (BO_CHOL_REGA) against the LDS-
# committed ones on the same build, and the committed build (ab_libs/libBASE.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab_rega
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_chol_dag.py tests/test_gpu_chol_batched.py > $O/tests_rega0.log 2>&1 || exit 1
BO_CHOL_REGA=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_chol_dag.py tests/test_gpu_chol_batched.py > $O/tests_rega1.log 2>&1 || exit 1
cp botorch_amd/libbotorch_amd.so ab_libs/libCUR.so
for r in 1 2; do
for v in BASE CUR0 CUR1; do
  case $v in BASE) cp ab_libs/libBASE.so botorch_amd/libbotorch_amd.so; R=0;; CUR0) cp ab_libs/libCUR.so botorch_amd/libbotorch_amd.so; R=0;; CUR1) cp ab_libs/libCUR.so botorch_amd/libbotorch_amd.so; R=1;; esac
  BO_CHOL_REGA=$R timeout -k 10 120 python tools/time_chol_batched.py > $O/time_${v}_$r.json 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('$O/time_${v}_$r.json').read().strip().splitlines()[-1])
print('$v', round(d['ms'], 4), [(b['nb'], b['n'], round(b['ms'], 3)) for b in d['batched']])"
done
done
cp ab_libs/libCUR.so botorch_amd/libbotorch_amd.so
