#!/bin/bash
# GPU-box: the GPU suite, then a short headline bench (no extras) and the
# posterior plan timings; every GPU step under its own limit, stop on a crash.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/chk
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -rf --timeout 120 --timeout-method thread > gpurun_out/chk/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/chk/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-extra --no-fit --no-cpu-baseline > gpurun_out/chk/bench.log 2>&1 || exit $?
python - <<'PY'
import json
for l in open('gpurun_out/chk/bench.log'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']
        print('ms/step %.4f kernel %.4f frac %.4f fwd_bwd %.4f chol %.4f' % (d['ms_per_step'], r['kernel_ms'], r['frac'], d['fwd_bwd']['ms'], d['cholesky']['ms']))
PY
if [ "${1:-}" = "tp" ]; then
timeout -k 10 300 python tools/time_posterior.py > gpurun_out/chk/time_posterior.json 2>&1 || exit $?
cat gpurun_out/chk/time_posterior.json
fi
