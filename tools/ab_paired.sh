set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_full_configs.py tests/test_gpu_acquisition.py -q -x --timeout 120 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/ab/pytest.log
for i in 1 2; do
BO_POST_PAIRED=0 timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-extra --no-fit --no-cpu-baseline > gpurun_out/ab/unpaired$i.log 2>&1 || exit 1
BO_POST_PAIRED=1 timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-extra --no-fit --no-cpu-baseline > gpurun_out/ab/paired$i.log 2>&1 || exit 1
done
for f in gpurun_out/ab/*paired*.log; do python - "$f" <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']
        print(sys.argv[1], 'ms/step %.4f'%d['ms_per_step'], 'kernel %.4f'%r['kernel_ms'], 'frac %.4f'%r['frac'], 'fwd_bwd', d['fwd_bwd']['ms'])
PY
done
