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
# PMC=1: one FETCH_SIZE / WRITE_SIZE pass per variant (PMC_CMD, default the
# measured command), summarised per variant by tools/pmc_summary.py
if [ "${PMC:-0}" = 1 ]; then
  export TMPDIR=/tmp
  if [ -n "$PMC_CMD" ]; then PC=($PMC_CMD); else PC=("$@"); fi
  for v in $VALS; do
    for c in FETCH_SIZE WRITE_SIZE; do
      if [ "$VAR" = LIB ]; then
        cp ab_libs/lib$v.so botorch_amd/libbotorch_amd.so
        timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${v}_$c -o run -- "${PC[@]}" > $O/pmc_${v}_$c.log 2>&1 || exit 1
      else
        env $VAR=$v timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${v}_$c -o run -- "${PC[@]}" > $O/pmc_${v}_$c.log 2>&1 || exit 1
      fi
    done
    python3 tools/pmc_summary.py $O/pmc_$v.json $O/pmc_${v}_FETCH_SIZE $O/pmc_${v}_WRITE_SIZE > $O/pmc_$v.txt 2>&1 || exit 1
    find $O/pmc_${v}_* -name 'run_counter_collection.csv' -size +2M -delete
    echo "PMC $v: $(head -c 600 $O/pmc_$v.txt)"
  done
fi
[ "$VAR" = LIB ] && cp ab_libs/libCUR.so botorch_amd/libbotorch_amd.so
exit 0
