#!/bin/bash
# GPU-box A/B driver (replaces the per-experiment ab_*.sh scripts of rounds
# 3-5, kept in git history).  Runs a measuring command once per variant, R
# rounds interleaved, output under gpurun_out/ab_<name>/.
#
#   tools/ab.sh NAME VAR "V1 V2 ..." CMD...
#
# VAR=LIB   swaps ab_libs/lib<V>.so in as botorch_amd/libbotorch_amd.so per
#           variant (CUR = the working tree's library), restored at the end;
# otherwise exports VAR=<V> (an environment knob) for the command.
# R (default 2) rounds; every step under its own time limit (T, default 200 s);
# the first failure ends the run.
# e.g.  tools/ab.sh diagch BO_CHOL_DIAG_CH "0 1 2" python tools/time_chol_batched.py
#       tools/ab.sh lib LIB "BASE CUR" python tools/fit_breakdown.py one
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
NAME=$1; VAR=$2; VALS=$3; shift 3
O=gpurun_out/ab_$NAME
mkdir -p $O
if [ "$VAR" = LIB ]; then
  mkdir -p ab_libs && cp botorch_amd/libbotorch_amd.so ab_libs/libCUR.so
fi
for r in $(seq 1 ${R:-2}); do
  for v in $VALS; do
    if [ "$VAR" = LIB ]; then
      cp ab_libs/lib$v.so botorch_amd/libbotorch_amd.so
      timeout -k 10 ${T:-200} "$@" > $O/${v}_$r.log 2>&1 || exit 1
    else
      env $VAR=$v timeout -k 10 ${T:-200} "$@" > $O/${v}_$r.log 2>&1 || exit 1
    fi
    echo "$VAR=$v round $r: $(tail -1 $O/${v}_$r.log | cut -c1-160)"
  done
done
[ "$VAR" = LIB ] && cp ab_libs/libCUR.so botorch_amd/libbotorch_amd.so
exit 0
