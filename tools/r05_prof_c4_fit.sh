#!/bin/bash
# GPU-box: kernel stats of the C4 qEHVI forward/backward and of the GP-fit closure
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05_c4prof -o c4 -- python3 $R/tools/c4_qehvi.py 20 > $R/gpurun_out/r05_c4prof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05_fitprof2 -o fit -- python3 $R/tools/fit_only.py 1 > $R/gpurun_out/r05_fitprof2.log 2>&1 || exit 1
