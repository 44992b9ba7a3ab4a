#!/bin/bash
# GPU-box: PMC passes over the C2 forward (tools/prof_small.py c2): MFMA busy, HBM bytes, LDS
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_small
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/mfma -o run -- python3 $R/tools/prof_small.py c2 > $O/mfma.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $R/tools/prof_small.py c2 > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_ACTIVE_INST_ANY --output-format csv -d $O/wait -o run -- python3 $R/tools/prof_small.py c2 > $O/wait.log 2>&1 || exit 1
python3 $R/tools/pmc_summary.py --meta command=c2_small $O/pmc.json $O/mfma $O/fetch $O/wait || exit 1
find $O -name '*_trace.csv' -size +2M -delete
