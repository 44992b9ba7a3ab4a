set -o pipefail
mkdir -p gpurun_out/r02q
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra --no-bwd"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02q/stats -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra --no-bwd > gpurun_out/r02q/bench_stats.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r02q/fetch -o run -- $B --no-fit > gpurun_out/r02q/fetch.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r02q/write -o run -- $B --no-fit > gpurun_out/r02q/write.log 2>&1 || exit $?
timeout -s KILL 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r02q/mfma -o run -- $B > gpurun_out/r02q/mfma.log 2>&1 || exit $?
ls -R gpurun_out/r02q | head -40
