#!/bin/bash
# GPU-box: the stream-K fix-up (BO_SK_FIXUP=1, default) against the separate
# split-k reduction kernel (0): posterior tests, the plan timings at C2 and the
# per-rank C3 shares, and the bench's other-config lines (C2 eager / graphed).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab_fixup
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_full_configs.py tests/test_gpu_graphs.py tests/test_gpu_acquisition.py -q -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  BO_SK_FIXUP=$v timeout -k 10 120 python tools/time_c2_plans.py > $O/c2_plans_$v.json 2>&1 || exit $?
  echo "fixup=$v c2_plans $(tail -1 $O/c2_plans_$v.json | cut -c1-300)"
  BO_SK_FIXUP=$v timeout -k 10 180 python tools/time_posterior.py > $O/time_posterior_$v.json 2>&1 || exit $?
  echo "fixup=$v posterior $(tail -1 $O/time_posterior_$v.json | cut -c1-400)"
done
for v in 1 0; do
  BO_SK_FIXUP=$v timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fit --no-bwd > $O/bench_$v.log 2>&1 || exit $?
  grep '^{' $O/bench_$v.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.readline()); oc=d['other_configs']
print('fixup=$v', {k: (round(v.get('gpu_ms', 0) or 0, 4), round(v.get('graphed_ms', 0) or 0, 4)) for k, v in oc.items() if k in ('C2', 'C4_qEHVI', 'C4_qNEHVI', 'C5_SAAS')}, 'W8', d['strong_scaling_projection'].get('W8'))"
done
