#!/bin/bash
# GPU-box: two library builds (ab_libs/lib$A.so, ab_libs/lib$B.so) swapped in
# turn: DAG tests on B, then Cholesky timings (n = 4096 + batched)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab_libs2
mkdir -p $O
cp botorch_amd/libbotorch_amd.so ab_libs/libORIG.so
cp ab_libs/lib$B.so botorch_amd/libbotorch_amd.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_chol_dag.py tests/test_gpu_chol_batched.py > $O/tests_$B.log 2>&1 || { cp ab_libs/libORIG.so botorch_amd/libbotorch_amd.so; exit 1; }
for r in 1 2; do
for v in $A $B; do
  cp ab_libs/lib$v.so botorch_amd/libbotorch_amd.so
  timeout -k 10 120 python tools/time_chol_batched.py > $O/time_${v}_$r.json 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('$O/time_${v}_$r.json').read().strip().splitlines()[-1])
print('$v', round(d['ms'], 4), [(b['nb'], b['n'], round(b['ms'], 3)) for b in d['batched']])"
done
done
cp ab_libs/libORIG.so botorch_amd/libbotorch_amd.so
