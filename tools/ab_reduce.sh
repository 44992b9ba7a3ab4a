#!/bin/bash
# GPU-box: the split-k reduction's two-chunks-per-round loop against the
# previous library (tools/ab/libbotorch_amd_base.so, swapped in for the B runs):
# posterior tests, then C2 / per-rank plan timings and the eager C2 call, A B A B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab_reduce
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
cp botorch_amd/libbotorch_amd.so $O/lib_new.so
for v in new base new base; do
  if [ $v = base ]; then cp tools/ab/libbotorch_amd_base.so botorch_amd/libbotorch_amd.so; else cp $O/lib_new.so botorch_amd/libbotorch_amd.so; fi
  timeout -k 10 120 python tools/time_c2_plans.py > $O/c2_$v.json 2>&1 || exit $?
  timeout -k 10 120 python tools/host_eager.py > $O/eager_$v.json 2>&1 || exit $?
  echo "$v c2 $(tail -1 $O/c2_$v.json | cut -c1-120) eager $(tail -1 $O/eager_$v.json | cut -c1-90)"
done
cp $O/lib_new.so botorch_amd/libbotorch_amd.so
rm -f $O/lib_new.so
