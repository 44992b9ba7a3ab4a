#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_qnehvi.py tests/test_gpu_c1_end_to_end.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_qnehvi.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_qnehvi.log; exit $rc
