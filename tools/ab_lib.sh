#!/bin/bash
# GPU-box: ab_libs/libBASE.so against the working tree's library, swapped in
# turn: Cholesky timings (n = 4096 + batched) and the GP fit
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab_lib
mkdir -p $O
cp botorch_amd/libbotorch_amd.so ab_libs/libCUR.so
for r in 1 2; do
for v in BASE CUR; do
  cp ab_libs/lib$v.so botorch_amd/libbotorch_amd.so
  timeout -k 10 120 python tools/time_chol_batched.py > $O/time_${v}_$r.json 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('$O/time_${v}_$r.json').read().strip().splitlines()[-1])
print('$v', round(d['ms'], 4), [(b['nb'], b['n'], round(b['ms'], 3)) for b in d['batched']])"
  timeout -k 10 200 python tools/fit_breakdown.py one > $O/fit_${v}_$r.log 2>&1 || exit 1
  grep "rep 1" $O/fit_${v}_$r.log | sed "s/^/$v /"
done
done
cp ab_libs/libCUR.so botorch_amd/libbotorch_amd.so
