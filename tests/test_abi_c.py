"""The C ABI from a non-Python caller: tests/host/abi_driver.c (plain C99,
gcc) includes include/botorch_amd.h, links libbotorch_amd.so and checks the
records' layouts, host entry points and error reporting; on a GPU it runs the
device L-BFGS-B through hipMalloc'd buffers, with no PyTorch in the process."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build(tmp_path):
    exe = str(tmp_path / "abi_driver")
    subprocess.run(["gcc", "-std=c99", "-O1", "-Wall", "-Werror", "-o", exe,
                    os.path.join(ROOT, "tests", "host", "abi_driver.c"),
                    "-L" + os.path.join(ROOT, "botorch_amd"), "-lbotorch_amd",
                    "-L/opt/rocm/lib", "-lamdhip64",
                    "-Wl,-rpath," + os.path.join(ROOT, "botorch_amd"), "-Wl,-rpath,/opt/rocm/lib",
                    "-lm"], check=True)
    return exe


def test_c_caller_host(tmp_path):
    out = subprocess.run([_build(tmp_path), "host"], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    assert out.stdout.count("ok ") == 3, out.stdout


@pytest.mark.gpu
def test_c_caller_device_lbfgsb(tmp_path):
    out = subprocess.run([_build(tmp_path), "gpu"], capture_output=True, text=True, timeout=100)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "ok gpu lbfgsb" in out.stdout, out.stdout
