#!/bin/bash
# DAG Cholesky chunk rows (single-step / batched tasks of one matrix) with the
# depth-2 prefetch on: interleaved A/B of BO_CHOL_CH / BO_CHOL_CHB
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/ab_chunks; mkdir -p $O
for rep in 1 2; do
  for cfg in "2 4" "2 6" "2 8" "1 4" "3 4" "2 3" "4 8"; do
    set -- $cfg
    BO_CHOL_CH=$1 BO_CHOL_CHB=$2 timeout -k 10 120 python3 tools/chol_time.py >> $O/ab.log 2>&1 || exit $?
  done
done
grep '^{' $O/ab.log
