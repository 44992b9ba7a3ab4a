#!/bin/bash
# GPU-box: quad plan tests, the GPU suite, then the quad timing (default rule and forced).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/quad
timeout -k 10 300 python -u -m pytest tests/test_gpu_acquisition.py -q -x -rf --timeout 120 --timeout-method thread -k "quad or deferred" > gpurun_out/quad/pytest_quad.log 2>&1
rc=$?; tail -3 gpurun_out/quad/pytest_quad.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -rf --timeout 120 --timeout-method thread > gpurun_out/quad/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/quad/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/time_quad.py > gpurun_out/quad/time_quad.json 2>&1 || exit $?
tail -1 gpurun_out/quad/time_quad.json
timeout -k 10 300 python tools/time_quad.py force > gpurun_out/quad/time_quad_force.json 2>&1 || exit $?
tail -1 gpurun_out/quad/time_quad_force.json
