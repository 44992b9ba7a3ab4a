"""Host-code sanitizers: the threaded box decomposition
(csrc/boxdecomp.cpp, qNEHVI's per-sample partitions) built with
AddressSanitizer + UndefinedBehaviorSanitizer and with ThreadSanitizer and
driven on 8 worker threads against a one-thread run (tools/sanitize_host.sh,
tests/host/boxdecomp_driver.cpp).  GPU sanitizers are not available on the
pool; the device code is covered by the parity tests."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_boxdecomp_asan_ubsan_tsan_clean():
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize_host.sh")], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.count(" ok") == 8  # four cases under each sanitizer
