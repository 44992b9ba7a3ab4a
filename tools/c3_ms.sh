#!/bin/bash
# One short C3 forward bench, summarised on one line (A/B runs, tools/ab.sh):
# ms per step, the posterior GEMM's event-timed ms, its fraction of spec, the
# oracle check's max relative error.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
python3 bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-extra --no-bwd --no-fit > /tmp/c3_ms.json || exit 1
python3 - <<'PY'
import json
d = json.loads(open("/tmp/c3_ms.json").read().strip().splitlines()[-1])
r = d["roofline"]
c = (d.get("check") or {}).get("max_rel_err_nonzero", float("nan"))
print(f"ms_per_step {d['ms_per_step']:.4f} kernel_ms {r['kernel_ms']:.4f} frac {r['frac']:.4f} check {c:.2e}")
PY
