#!/bin/bash
# full GPU suite, qmc phases, C2 host breakdown, then the Cholesky chunk A/B
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/gpu_r04k.sh || exit $?
bash tools/ab_chunks.sh > gpurun_out/ab_chunks_summary.log 2>&1 || exit $?
cat gpurun_out/ab_chunks_summary.log | cut -c1-200
