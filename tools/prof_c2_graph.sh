#!/bin/bash
# GPU-box: kernel trace of the C2 eager calls and graph replays (tools/time_c2_graph.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/c2graph -o run -- python3 $R/tools/time_c2_graph.py > $R/gpurun_out/c2graph.log 2>&1
