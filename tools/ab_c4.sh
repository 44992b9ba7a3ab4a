#!/bin/bash
# GPU-box: C4 qEHVI bench line (forward; fwd+bwd) with the small-grid route
# auto / forced (one launch for the three members)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab_c4
mkdir -p $O
for r in 1 2; do
for m in auto 1; do
  BO_POST_SMALL=$m timeout -k 10 200 python bench.py --acq qehvi --steps 20 --warmup 3 --no-extra --no-fit > $O/c4_${m}_$r.log 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('$O/c4_${m}_$r.log').read().strip().splitlines()[-1])
print('small=$m', round(d['ms_per_step'], 4), 'fwd_bwd', round(d['fwd_bwd']['ms'], 4), 'check', d['check']['max_rel_err_nonzero'])"
done
done
