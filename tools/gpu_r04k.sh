#!/bin/bash
# qmc ladder with rsq + readlane: full GPU suite, qmc phase timing, host
# breakdown of the eager C2 call, C2 A/B tool (op-level rate)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04k
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -rf --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python3 tools/time_qmc_phases.py > $O/qmc_phases.log 2>&1 || exit $?
tail -2 $O/qmc_phases.log
timeout -k 10 300 python3 tools/host_c2_breakdown.py > $O/host_c2.log 2>&1 || exit $?
tail -1 $O/host_c2.log
exit $rc
