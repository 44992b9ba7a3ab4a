#!/bin/bash
# GPU-box: the DAG Cholesky's rows per single-step task (CH, one matrix) 4 (built, labelled 8) vs 2 / 3
# (tools/ab/lib_ch*.so swapped in), time_chol_batched A B C A B C.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab_ch
mkdir -p $O
cp botorch_amd/libbotorch_amd.so $O/lib_ch8.so
for rep in 1 2; do
  for v in 8 2 3; do  # 3 = CH 1 here
    if [ $v = 8 ]; then cp $O/lib_ch8.so botorch_amd/libbotorch_amd.so; else cp tools/ab/lib_ch$v.so botorch_amd/libbotorch_amd.so; fi
    timeout -k 10 120 python tools/time_chol_batched.py > $O/t_$v.json 2>&1 || exit $?
    python3 -c "
import json; d=json.loads(open('$O/t_$v.json').read().strip().splitlines()[-1])
print('ch=$v', round(d['ms'], 4), [(b['nb'], b['n'], round(b['ms'], 3)) for b in d['batched']])"
  done
done
cp $O/lib_ch8.so botorch_amd/libbotorch_amd.so
rm -f $O/lib_ch8.so
