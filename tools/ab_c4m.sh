#!/bin/bash
# GPU-box: members-route tests, then the C4 bench line with the member-batched
# stream-K launch on / off
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab_c4m
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_post_members.py tests/test_gpu_post_small.py > $O/tests.log 2>&1 || exit 1
for r in 1 2; do
for m in 1 0; do
  BO_POST_MEMBERS=$m timeout -k 10 200 python bench.py --acq qehvi --steps 20 --warmup 3 --no-extra --no-fit > $O/c4_${m}_$r.log 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('$O/c4_${m}_$r.log').read().strip().splitlines()[-1])
print('members=$m', round(d['ms_per_step'], 4), 'fwd_bwd', round(d['fwd_bwd']['ms'], 4), 'check', d['check']['max_rel_err_nonzero'], 'kernel_ms', d['roofline']['kernel_ms'], d['roofline']['launches_per_step'])"
done
done
