#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r04j
timeout -k 10 300 python3 tools/host_c2_breakdown.py > gpurun_out/r04j/host_c2.log 2>&1; rc=$?
tail -2 gpurun_out/r04j/host_c2.log; exit $rc
