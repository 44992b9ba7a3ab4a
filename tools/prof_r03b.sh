set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03b
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r03b/bwd -o run --output-format csv -- python tools/prof_bwd.py > gpurun_out/r03b/bwd.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r03b/fwd -o run --output-format csv -- python tools/c3_fwd.py 30 > gpurun_out/r03b/fwd.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/r03b/pmc_sq -o run --output-format csv -- python tools/c3_fwd.py 5 > gpurun_out/r03b/pmc_sq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r03b/pmc_fetch -o run --output-format csv -- python tools/c3_fwd.py 5 > gpurun_out/r03b/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r03b/pmc_write -o run --output-format csv -- python tools/c3_fwd.py 5 > gpurun_out/r03b/pmc_write.log 2>&1 || exit $?
python tools/pmc_summary.py gpurun_out/r03b/pmc_summary.json gpurun_out/r03b/pmc_sq gpurun_out/r03b/pmc_fetch gpurun_out/r03b/pmc_write > gpurun_out/r03b/pmc_summary.txt 2>&1
find gpurun_out/r03b -name '*_trace.csv' -size +2M -delete
find gpurun_out/r03b -name 'run_counter_collection.csv' -size +2M -delete
cat gpurun_out/r03b/pmc_summary.txt | head -8
