set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03a
timeout -k 10 60 rocprofv3 -L > gpurun_out/r03a/counters.txt 2>&1 || true
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r03a/c2 -o run --output-format csv -- python tools/prof_small.py c2 > gpurun_out/r03a/c2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/r03a/pmc_sq -o run --output-format csv -- python tools/c3_fwd.py 5 > gpurun_out/r03a/pmc_sq.log 2>&1 || exit $?
python tools/pmc_summary.py gpurun_out/r03a/pmc_sq.json gpurun_out/r03a/pmc_sq > gpurun_out/r03a/pmc_sq.txt 2>&1
find gpurun_out/r03a -name '*_trace.csv' -size +2M -delete
find gpurun_out/r03a -name 'run_counter_collection.csv' -size +2M -delete
ls -R gpurun_out/r03a | head -30
