#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG:-c4nprof} -o run -- python3 $R/tools/c4_qnehvi.py 10 > $R/gpurun_out/c4nprof.log 2>&1
