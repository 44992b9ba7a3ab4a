#!/bin/bash
# C2 eager call vs the stream-K minimum share (BO_SK_MIN_SHARE, read once per
# process), interleaved twice
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/ab_sk; mkdir -p $O
for rep in 1 2; do
  for sh in 4 2 3 6 8; do
    echo "share $sh $(BO_SK_MIN_SHARE=$sh timeout -k 10 120 python3 tools/host_c2_breakdown.py 2>/dev/null | tail -1 | cut -c1-80)" >> $O/ab.log || exit $?
  done
done
cat $O/ab.log
