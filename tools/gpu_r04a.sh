#!/bin/bash
# Round 4, first GPU call: the GPU suite (with the config-size gradient, the
# fixed-feature capture and the 2-rank device tests), smoke, the default bench
# line, then the C4 qEHVI kernel trace + VALU PMC for the executed-work roofline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04a
mkdir -p $O
bash tools/gpu_run.sh test smoke || exit $?
cp gpurun_out/pytest_gpu.log gpurun_out/smoke.log $O/
timeout -k 10 700 python3 bench.py > $O/bench_default.log 2>&1 || exit $?
tail -c 3000 $O/bench_default.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/c4 -o run --output-format csv -- python3 tools/c4_qehvi.py 5 > $O/c4.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $O/c4_pmc -o run --output-format csv -- python3 tools/c4_qehvi.py 3 > $O/c4_pmc.log 2>&1 || exit $?
python3 tools/qehvi_roofline.py $O/qehvi_roofline.json $O/c4 $O/c4_pmc > $O/qehvi_roofline.txt 2>&1
find $O -name '*_trace.csv' -size +2M -delete
find $O -name 'run_counter_collection.csv' -size +2M -delete
cat $O/qehvi_roofline.txt
