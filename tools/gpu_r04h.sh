#!/bin/bash
# qNEHVI / C1 GPU tests, then the C2 K*x A/B (timing, and kernel stats of each arm)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04h
timeout -k 10 600 python -u -m pytest tests/test_gpu_qnehvi.py tests/test_gpu_c1_end_to_end.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r04h/pytest_qnehvi.log 2>&1
rc=$?; tail -5 gpurun_out/r04h/pytest_qnehvi.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 tools/ab_c2_kxt.py > gpurun_out/r04h/ab_c2_kxt.log 2>&1 || exit $?
tail -1 gpurun_out/r04h/ab_c2_kxt.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04h/prof -o run -- python3 tools/ab_c2_kxt.py > gpurun_out/r04h/prof.log 2>&1 || exit $?
find gpurun_out/r04h -name '*_trace.csv' -size +2M -delete
exit $rc
