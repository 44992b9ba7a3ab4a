#!/bin/bash
# Final round-3 measurement set on one MI355X: GPU suite + smoke, the driver's
# default bench line, rocprofv3 kernel stats of the bench (forward-only and
# with the GP fit), and the PMC passes (FETCH_SIZE, WRITE_SIZE, MFMA busy; one
# block group per run) summarised by tools/pmc_summary.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03final
mkdir -p $O
bash tools/gpu_run.sh test smoke || exit $?
timeout -k 10 700 python3 bench.py > $O/bench_default.log 2>&1 || exit $?
echo "bench: $(grep -c '^{' $O/bench_default.log) line(s)"
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra --no-bwd"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_fwd -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extra --no-bwd --no-fit > $O/stats_fwd.log 2>&1 || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_fit -o run -- $B > $O/stats_fit.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $B --no-fit > $O/fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $B --no-fit > $O/write.log 2>&1 || exit $?
timeout -s KILL 500 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --output-format csv -d $O/mfma -o run -- $B > $O/mfma.log 2>&1 || exit $?
python3 tools/pmc_summary.py $O/pmc_summary.json $O/fetch $O/write $O/mfma || exit $?
# the n = 4096 Cholesky alone: kernel trace and its PMC passes (single problems)
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/chol -o run -- python3 tools/chol_only.py > $O/chol.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/chol_fetch -o run -- python3 tools/chol_only.py > $O/chol_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/chol_write -o run -- python3 tools/chol_only.py > $O/chol_write.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d $O/chol_mfma -o run -- python3 tools/chol_only.py > $O/chol_mfma.log 2>&1 || exit $?
python3 tools/pmc_summary.py $O/pmc_chol.json $O/chol_fetch $O/chol_write $O/chol_mfma || exit $?
# C2 eager forward and the C4 qEHVI forward + backward, kernel traces
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o run -- python3 tools/prof_small.py c2 > $O/c2.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o run -- python3 tools/c4_qehvi.py 5 > $O/c4.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bwd -o run -- python3 tools/prof_bwd.py > $O/bwd.log 2>&1 || exit $?
find $O -name '*_trace.csv' -size +2M -delete
find $O -name 'run_counter_collection.csv' -delete
du -sh $O
