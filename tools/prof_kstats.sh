#!/bin/bash
# rocprofv3 kernel stats of one command, summarised as one JSON line of
# {kernel name prefix: [calls, average us]} (the A/B driver's last line).
#   tools/prof_kstats.sh python3 tools/c4_qehvi.py 20
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
D=$(mktemp -d /tmp/kst.XXXXXX)
export TMPDIR=/tmp
(cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- "$@") > $D/out.log 2>&1 || { tail -5 $D/out.log; exit 1; }
python3 - "$D" <<'PY'
import csv, glob, json, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
out = {}
for r in csv.DictReader(open(f)):
    name = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "")[:60]
    out[name] = [int(r["Calls"]), round(float(r["AverageNs"]) / 1e3, 2)]
print(json.dumps(dict(list(out.items())[:12])))
PY
rm -rf $D
