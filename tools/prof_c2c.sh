#!/bin/bash
# GPU-box: the GPU suite, C2 kernel gaps + host cost, quad timings, C4 qEHVI trace.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c2c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -rf --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python tools/prof_small.py c2 > $O/trace.log 2>&1 || exit $?
timeout -k 10 120 python tools/prof_small.py c2 > $O/plain.log 2>&1 || exit $?
grep ms $O/plain.log
python tools/trace_gaps.py $O/trace/run_kernel_trace.csv 9 > $O/gaps.txt 2>&1
cat $O/gaps.txt
timeout -k 10 120 python tools/host_eager.py > $O/host_eager.json 2>&1 || exit $?
tail -1 $O/host_eager.json
timeout -k 10 300 python tools/time_quad.py > $O/time_quad.json 2>&1 || exit $?
tail -1 $O/time_quad.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/c4 -o run --output-format csv -- python tools/c4_qehvi.py 5 > $O/c4.log 2>&1 || exit $?
grep -E "qehvi" $O/c4/run_kernel_stats.csv | cut -d, -f1-6
