#!/bin/bash
# GPU-box: DAG queue knobs swept on the n = 4096 factorisation + inverse
# (BO_CHOL_CH / BO_CHOL_CHB chunk rows, BO_CHOL_DIAG_CH, BO_CHOL_CRIT_W)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/sweep_chol
mkdir -p $O
run() {  # label env...
  local l=$1; shift
  env "$@" timeout -k 10 120 python tools/time_chol_batched.py > $O/$l.json 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('$O/$l.json').read().strip().splitlines()[-1])
print('$l', round(d['ms'], 4), [(b['nb'], b['n'], round(b['ms'], 3)) for b in d['batched']])"
}
for r in 1 2; do
  run base_$r X=1
  run chb3_$r BO_CHOL_CHB=3
  run chb6_$r BO_CHOL_CHB=6
  run ch1_$r BO_CHOL_CH=1
  run ch3_$r BO_CHOL_CH=3
  run dch1_$r BO_CHOL_DIAG_CH=1
  run dch3_$r BO_CHOL_DIAG_CH=3
  run cw05_$r BO_CHOL_CRIT_W=0.5
  run cw0_$r BO_CHOL_CRIT_W=0
done
