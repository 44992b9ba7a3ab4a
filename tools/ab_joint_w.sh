#!/bin/bash
# GPU-box: joint device L-BFGS-B on an 8- vs 16-wave workgroup (BO_LBFGSB_JOINT_W)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for w in 8 16; do
  BO_LBFGSB_JOINT_W=$w timeout -k 10 300 python tools/prof_lbfgsb_joint.py > gpurun_out/joint_w$w.log 2>&1 || exit 1
  grep joint gpurun_out/joint_w$w.log | sed "s/^/w=$w /"
done
