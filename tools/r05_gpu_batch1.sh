#!/bin/bash
# round-5 GPU batch: small-grid kernel tests + A/B, full suite, bench modes, fit profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_post_small.py tests/test_gpu_chol_batched.py tests/test_gpu_chol_dag.py > gpurun_out/r05_small.log 2>&1 || exit 1
for v in 0 1 auto; do BO_POST_SMALL=$v timeout -k 10 120 python tools/time_small.py >> gpurun_out/r05_small_ab.log 2>&1 || exit 1; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r05_suite2.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --acq qnei --steps 10 --warmup 2 --no-extra --no-fit > gpurun_out/r05_bench_qnei.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --acq qehvi --steps 10 --warmup 2 --no-extra --no-fit > gpurun_out/r05_bench_qehvi.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r05_fitprof -o fit -- python3 $GRAFT_REPO_ROOT/tools/fit_only.py 1 > $GRAFT_REPO_ROOT/gpurun_out/r05_fitprof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r05_cholprof -o chol -- python3 $GRAFT_REPO_ROOT/tools/chol_only.py > $GRAFT_REPO_ROOT/gpurun_out/r05_cholprof.log 2>&1 || exit 1
