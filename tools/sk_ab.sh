#!/bin/bash
# One line for tools/ab.sh: C3-model forward + backward wall time at b = 2 and
# 8 (tools/small_fb.py) and C4 qEHVI forward / forward + backward
# (tools/c4_times.py) -- the stream-K plans' small grids.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
a=$(python3 tools/small_fb.py 200 2 2>/dev/null | tail -1)
b=$(python3 tools/small_fb.py 200 8 2>/dev/null | tail -1)
c=$(python3 tools/c4_times.py 20 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('c4 fwd %.3f fb %.3f qnehvi fb %.3f' % (d['qehvi']['fwd_ms'], d['qehvi']['fwd_bwd_ms'], d['qnehvi']['fwd_bwd_ms']))")
echo "$a | $b | $c"
