#!/bin/bash
# Round 4: joint L-BFGS-B phase clocks, then the forward bench's kernel stats
# and PMC passes (FETCH_SIZE / WRITE_SIZE / MFMA, one block group per run)
# summarised with the launch size recorded (bench.py's traffic field), C2 stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 300 python3 tools/prof_lbfgsb_joint.py > $O/lbfgsb_joint.log 2>&1 || exit $?
cat $O/lbfgsb_joint.log
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra --no-bwd --no-fit"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_fwd -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extra --no-bwd --no-fit > $O/stats_fwd.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $B > $O/fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $B > $O/write.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/mfma -o run -- $B > $O/mfma.log 2>&1 || exit $?
python3 tools/pmc_summary.py --meta restarts=512 --meta command=bench_fwd $O/pmc_summary.json $O/fetch $O/write $O/mfma || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o run -- python3 tools/prof_small.py c2 > $O/c2.log 2>&1 || exit $?
find $O -name '*_trace.csv' -size +2M -delete
find $O -name 'run_counter_collection.csv' -delete
grep -h "post_partials\|kxt\|qmc_kernel\|splitk" $O/stats_fwd/run_kernel_stats.csv $O/c2/run_kernel_stats.csv | cut -c1-200
