#!/bin/bash
# GPU-box: kernel trace of the C4 qEHVI forward/backward (tools/c4_qehvi.py)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
BO_POST_SMALL=${SMALL:-auto} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG:-c4prof} -o c4 -- python3 $R/tools/c4_qehvi.py 20 > $R/gpurun_out/${TAG:-c4prof}.log 2>&1
