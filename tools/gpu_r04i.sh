#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04i
timeout -k 10 600 python -u -m pytest tests/test_gpu_qnehvi.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r04i/pytest_qnehvi.log 2>&1
rc=$?; tail -15 gpurun_out/r04i/pytest_qnehvi.log; exit $rc
