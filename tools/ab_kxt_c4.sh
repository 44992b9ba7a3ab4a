#!/bin/bash
# GPU-box: C4 bench line for the small-grid K*x^T points per thread (BO_KXT_SMALL)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab_kxt_c4
mkdir -p $O
for r in 1 2; do
for k in 2 4 8; do
  BO_KXT_SMALL=$k timeout -k 10 200 python bench.py --acq qehvi --steps 20 --warmup 3 --no-extra --no-fit > $O/c4_${k}_$r.log 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('$O/c4_${k}_$r.log').read().strip().splitlines()[-1])
print('kxt=$k', round(d['ms_per_step'], 4), 'fwd_bwd', round(d['fwd_bwd']['ms'], 4), 'check', d['check']['max_rel_err_nonzero'])"
done
done
