#!/bin/bash
# GPU-box: the committed chol_dag (ab_libs/libHEAD.so) against the working tree's, swapped in turn
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab_head
mkdir -p $O
cp botorch_amd/libbotorch_amd.so ab_libs/libCUR.so
for r in 1 2 3; do
for v in HEAD CUR; do
  cp ab_libs/lib$v.so botorch_amd/libbotorch_amd.so
  BO_CHOL_CRIT_WG=0 timeout -k 10 120 python tools/time_chol_batched.py > $O/time_${v}_$r.json 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('$O/time_${v}_$r.json').read().strip().splitlines()[-1])
print('$v', round(d['ms'], 4), [(b['nb'], b['n'], round(b['ms'], 3)) for b in d['batched']])"
done
done
cp ab_libs/libCUR.so botorch_amd/libbotorch_amd.so
