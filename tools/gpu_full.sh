#!/bin/bash
# GPU-box: the GPU suite, then the default bench line (all configs).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/full
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u bench.py > $O/bench.log 2>&1 || exit $?
grep '^{' $O/bench.log | python -c "
import json,sys
d=json.loads(sys.stdin.readline())
r=d['roofline']; print('value %.4g ms/step %.4f kernel %.4f frac %.4f fwd_bwd %s chol %.4f' % (d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], d['fwd_bwd'], d['cholesky']['ms']))
oc=d.get('other_configs') or {}
for k,v in oc.items(): print(k, {kk:vv for kk,vv in v.items() if not isinstance(vv,(dict,list)) and kk!='config'})
"
