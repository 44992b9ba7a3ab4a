cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab_potrf && timeout -k 10 60 python tools/probe_potrf64.py > gpurun_out/ab_potrf/probe.json 2>&1; tail -1 gpurun_out/ab_potrf/probe.json
