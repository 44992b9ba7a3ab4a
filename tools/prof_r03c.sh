#!/bin/bash
# GPU-box: C4 qEHVI kernel trace + VALU-fp64 PMC (qehvi roofline), then the
# C3 fwd+bwd trace again (unmaterialised grads of the saved intermediates).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03c
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/c4 -o run --output-format csv -- python tools/c4_qehvi.py 5 > $O/c4.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $O/c4_pmc -o run --output-format csv -- python tools/c4_qehvi.py 3 > $O/c4_pmc.log 2>&1 || exit $?
python tools/qehvi_roofline.py $O/qehvi_roofline.json $O/c4 $O/c4_pmc > $O/qehvi_roofline.txt 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/bwd -o run --output-format csv -- python tools/prof_bwd.py > $O/bwd.log 2>&1 || exit $?
find $O -name '*_trace.csv' -size +2M -delete
find $O -name 'run_counter_collection.csv' -size +2M -delete
cat $O/qehvi_roofline.txt
