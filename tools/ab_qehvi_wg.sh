#!/bin/bash
# GPU-box: C4 bench line with the qEHVI backward sample split targeting 256 / 512 / 1024 workgroups
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab_qehvi_wg
mkdir -p $O
for r in 1 2; do
for w in 256 512 1024; do
  BO_QEHVI_BWD_WG=$w timeout -k 10 200 python bench.py --acq qehvi --steps 20 --warmup 3 --no-extra --no-fit > $O/c4_${w}_$r.log 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('$O/c4_${w}_$r.log').read().strip().splitlines()[-1])
print('bwd_wg=$w', round(d['ms_per_step'], 4), 'fwd_bwd', round(d['fwd_bwd']['ms'], 4), 'check', d['check']['max_rel_err_nonzero'])"
done
done
