#!/bin/bash
# GPU-box: first-chunk rows of the batched column updates (BO_CHOL_DIAG_CH):
# Cholesky timings (n = 4096 + batched) and the GP fit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab_diagch
mkdir -p $O
for r in 1 2; do
for c in ${CS:-0 1 2}; do
  BO_CHOL_DIAG_CH=$c timeout -k 10 120 python tools/time_chol_batched.py > $O/time_${c}_$r.json 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('$O/time_${c}_$r.json').read().strip().splitlines()[-1])
print('ch=$c', round(d['ms'], 4), [(b['nb'], b['n'], round(b['ms'], 3)) for b in d['batched']])"
done
done
for c in ${FS:-0 1}; do
  BO_CHOL_DIAG_CH=$c timeout -k 10 200 python tools/fit_only.py > $O/fit_$c.json 2>&1 || exit 1
  echo "fit ch=$c $(tail -1 $O/fit_$c.json | cut -c1-90)"
done
