#!/bin/bash
# full GPU suite, qmc phases, C2 host breakdown, then the Cholesky chunk A/B
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/gpu_r04k.sh || exit $?
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04k/c2 -o run -- python3 tools/prof_small.py c2 > gpurun_out/r04k/c2.log 2>&1 || exit $?
find gpurun_out/r04k -name '*_trace.csv' -size +2M -delete
bash tools/ab_chunks.sh > gpurun_out/ab_chunks_summary.log 2>&1 || exit $?
cat gpurun_out/ab_chunks_summary.log | cut -c1-200
