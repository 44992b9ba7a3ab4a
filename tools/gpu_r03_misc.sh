#!/bin/bash
# GPU-box: the 2-rank strong-split bench rehearsed on one GPU (gloo, every
# rank on cuda:0: exercises the launcher, the split and the report, measures
# nothing), then PMC of the C3 forward + backward loop (the fused W -> dX pass).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03misc
mkdir -p $O
BO_BENCH_REHEARSE=1 timeout -k 10 300 python3 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-extra --no-fit --no-bwd > $O/rehearse_2ranks_strong.log 2>&1 || exit $?
grep '^{' $O/rehearse_2ranks_strong.log | cut -c1-400
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/bwd_fetch -o run -- python3 tools/prof_bwd.py > $O/bwd_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/bwd_write -o run -- python3 tools/prof_bwd.py > $O/bwd_write.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --output-format csv -d $O/bwd_mfma -o run -- python3 tools/prof_bwd.py > $O/bwd_mfma.log 2>&1 || exit $?
python3 tools/pmc_summary.py $O/pmc_bwd.json $O/bwd_fetch $O/bwd_write $O/bwd_mfma || exit $?
find $O -name 'run_counter_collection.csv' -delete
