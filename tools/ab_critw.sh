#!/bin/bash
# GPU-box: the DAG Cholesky timed for several CRIT weights of the queue priority.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab_critw
mkdir -p $O
for w in ${WS:-1 2 4 8 16}; do
  BO_CHOL_CRIT_W=$w timeout -k 10 120 python tools/time_chol_batched.py > $O/time_$w.json 2>&1 || exit $?
  python3 -c "
import json; d=json.loads(open('$O/time_$w.json').read().strip().splitlines()[-1])
print('w=$w', round(d['ms'], 4), [(b['nb'], b['n'], round(b['ms'], 3)) for b in d['batched']])"
done
BO_CHOL_CRIT_W=${WT:-4} timeout -k 10 120 python tools/trace_chol.py > $O/trace.json 2>&1 || exit $?
python3 tools/trace_summary.py $O/trace.json w=${WT:-4}
