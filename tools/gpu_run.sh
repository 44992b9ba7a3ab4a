#!/bin/bash
# GPU-box driver: each GPU step under its own time limit; a crash, abort or
# timeout ends the script (test failures, rc=1, do not).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
}
for s in "$@"; do
  case $s in
    build) step build 600 make -j16 ;;
    test) step pytest_gpu 1200 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread ;;
    testx) step pytest_gpu 1200 python -u -m pytest tests -m gpu -q -x -rf --timeout 120 --timeout-method thread ;;
    testlog) step pytest_logei 600 python -u -m pytest tests/test_gpu_logei.py -q -rf --timeout 120 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ;;
    bench_short) step bench 600 python bench.py --steps 10 --warmup 2 ;;
    prof) step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-fit --no-extra --no-bwd ;;
    prof_fit) step prof_fit 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fit -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extra --no-bwd ;;
    pmc_fetch) step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fit --no-extra --no-bwd ;;
    pmc_write) step pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fit --no-extra --no-bwd ;;
    pmc_mfma) step pmc_mfma 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_mfma -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fit --no-extra --no-bwd ;;
    prof_small) step prof_small 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_small -o run --output-format csv -- python tools/prof_small.py c2 ;;
    prof_chol) export BO_ONLY=chol; step prof_chol 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_chol -o run --output-format csv -- python tools/bench_linalg.py ;;
    prof_bwd) step prof_bwd 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bwd -o run --output-format csv -- python tools/prof_bwd.py ;;
    potrf) step potrf 120 python tools/probe_potrf.py ;;
    linalg) step linalg 300 python tools/bench_linalg.py ;;
    probe) step probe 120 python tools/probe_rate.py ;;
    # summarise PMC passes on the box and drop the bulky per-dispatch traces
    # (gpurun copies gpurun_out/ back only below 64 MiB)
    finish) python tools/pmc_summary.py gpurun_out/pmc_summary.json gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_mfma || true
            find gpurun_out -name '*_trace.csv' -size +2M -delete
            find gpurun_out -name 'run_counter_collection.csv' -delete
            du -sh gpurun_out ;;
    *) step custom 900 bash -c "$s" ;;
  esac
done
