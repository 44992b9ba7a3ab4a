"""bench.py's multi-GPU launcher on the CPU: ``python bench.py --gpus 2``
without torchrun's environment starts the two ranks itself (a
torch.distributed.run child), the N > 1 headline is the strong split of C3's
512 restarts, and rank 0 prints one JSON line.  BO_BENCH_REHEARSE=cpu swaps the
acquisition forward for a stub over gloo, so only the launch, the split, the
collectives and the report are exercised (the driver's 8-GPU run uses RCCL)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, extra_env=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(BO_BENCH_REHEARSE="cpu", OMP_NUM_THREADS="1", **(extra_env or {}))
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                         capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 4])
def test_bench_gpus_n_launches_n_ranks_strong(n):
    line = _run(["--gpus", str(n), "--steps", "3", "--warmup", "1"])
    assert line["n_gpus"] == n
    assert line["scaling"] == "strong"
    assert line["config"]["restarts_per_gpu"] == 512 // n
    assert line["steps"] == 3


def test_bench_gpus_2_weak_option():
    line = _run(["--gpus", "2", "--steps", "2", "--warmup", "1", "--weak"])
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["restarts_per_gpu"] == 512


def test_bench_world_size_mismatch_fails():
    env = {k: v for k, v in os.environ.items()}
    env.update(BO_BENCH_REHEARSE="cpu", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                         capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert out.returncode != 0 and "WORLD_SIZE" in out.stderr
