#!/bin/bash
# GPU-box: the batched queue's stagger (BO_CHOL_BATCH_STAGGER) and chunk rows on 3 x 2048 / 4 x 4096
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/sweep_chol_b
mkdir -p $O
run() {
  local l=$1; shift
  env "$@" timeout -k 10 120 python tools/time_chol_batched.py > $O/$l.json 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('$O/$l.json').read().strip().splitlines()[-1])
print('$l', round(d['ms'], 4), [(b['nb'], b['n'], round(b['ms'], 3)) for b in d['batched']])"
}
for r in 1 2; do
  run base_$r X=1
  run st0_$r BO_CHOL_BATCH_STAGGER=0
  run st05_$r BO_CHOL_BATCH_STAGGER=0.5
  run st1_$r BO_CHOL_BATCH_STAGGER=1
  run chb2_$r BO_CHOL_CHB=2
  run ch1_$r BO_CHOL_CH=1
done
