#!/bin/bash
# A round's measurement set on one MI355X (OUT names it, e.g. OUT=r06end):
# GPU suite + smoke (SKIP_SUITE=1: not),
# default bench line, rocprofv3 kernel stats of the forward bench, PMC passes
# of the forward bench (FETCH_SIZE / WRITE_SIZE / MFMA, one block group per
# run) summarised with the launch size recorded (bench.py reads it), the qmc
# phase timing and the Cholesky alone (kernel trace + PMC).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-round}
mkdir -p $O
if [ "${SKIP_SUITE:-0}" != 1 ]; then
  bash tools/gpu_run.sh test smoke || exit $?
  cp gpurun_out/pytest_gpu.log gpurun_out/smoke.log $O/
fi
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra --no-bwd --no-fit"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_fwd -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extra --no-bwd --no-fit > $O/stats_fwd.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $B > $O/fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $B > $O/write.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/mfma -o run -- $B > $O/mfma.log 2>&1 || exit $?
python3 tools/pmc_summary.py --meta restarts=512 --meta command=bench_fwd $O/pmc_summary.json $O/fetch $O/write $O/mfma || exit $?
timeout -k 10 200 python3 tools/time_qmc_phases.py > $O/qmc_phases.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/chol -o run -- python3 tools/chol_only.py > $O/chol.log 2>&1 || exit $?
# PMC of the single n = 4096 launch alone (one shape's bytes per problem)
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/chol_fetch -o run -- python3 tools/chol_only.py single > $O/chol_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/chol_write -o run -- python3 tools/chol_only.py single > $O/chol_write.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/chol_mfma -o run -- python3 tools/chol_only.py single > $O/chol_mfma.log 2>&1 || exit $?
python3 tools/pmc_summary.py --meta command=chol_only_single $O/pmc_chol.json $O/chol_fetch $O/chol_write $O/chol_mfma || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o run -- python3 tools/prof_small.py c2 > $O/c2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o run -- python3 tools/c4_qehvi.py 20 > $O/c4.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/c4_times.py 20 > $O/c4_times.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fit -o run -- python3 tools/fit_only.py 1 > $O/fit.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/fit_breakdown.py one > $O/fit_breakdown.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --acq qnei --steps 10 --warmup 2 --no-extra --no-fit > $O/bench_qnei.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --acq qehvi --steps 20 --warmup 3 --no-extra --no-fit > $O/bench_qehvi.log 2>&1 || exit $?
BO_LBFGSB_JOINT_W=0 timeout -k 10 300 python3 tools/prof_lbfgsb_joint.py > $O/lbfgsb_joint.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/host_c2_breakdown.py > $O/host_c2.log 2>&1 || exit $?
find $O -name '*_trace.csv' -size +2M -delete
find $O -name 'run_counter_collection.csv' -delete
du -sh $O
