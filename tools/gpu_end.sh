#!/bin/bash
# GPU-box: end-of-session check of the committed tree -- the GPU suite, smoke()
# and the driver's default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/end
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -2 $O/smoke.log
timeout -k 10 900 python bench.py > $O/bench.log 2>&1 || exit $?
grep '^{' $O/bench.log | cut -c1-300
