#!/bin/bash
# N > 1 bench path rehearsed on one GPU (2 ranks on cuda:0 over gloo; the
# timings measure nothing), strong and weak; then the 2-rank device sharding test
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04n; mkdir -p $O
export BO_BENCH_REHEARSE=1
timeout -k 10 300 python3 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-extra --no-fit > $O/rehearse_2ranks_strong.log 2>&1 || exit $?
grep '^{' $O/rehearse_2ranks_strong.log | cut -c1-300
timeout -k 10 300 python3 bench.py --gpus 2 --weak --steps 5 --warmup 2 --no-cpu-baseline --no-extra --no-fit --no-bwd > $O/rehearse_2ranks_weak.log 2>&1 || exit $?
grep '^{' $O/rehearse_2ranks_weak.log | cut -c1-300
unset BO_BENCH_REHEARSE
timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py -v --timeout 200 --timeout-method thread > $O/pytest_distributed.log 2>&1; rc=$?
tail -3 $O/pytest_distributed.log; exit $rc
