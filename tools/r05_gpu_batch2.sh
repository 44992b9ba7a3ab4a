#!/bin/bash
# round-5 GPU batch 2: suite, bench modes, default bench, fit + Cholesky profiles
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r05_suite3.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --acq qnei --steps 10 --warmup 2 --no-extra --no-fit > gpurun_out/r05_bench_qnei.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --acq qehvi --steps 10 --warmup 2 --no-extra --no-fit > gpurun_out/r05_bench_qehvi.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r05_bench_default.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r05_fitprof -o fit -- python3 $R/tools/fit_only.py 1 > $R/gpurun_out/r05_fitprof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r05_cholprof -o chol -- python3 $R/tools/chol_only.py > $R/gpurun_out/r05_cholprof.log 2>&1 || exit 1
