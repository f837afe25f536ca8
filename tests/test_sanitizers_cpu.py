"""Host-side race / memory checks of the native runtime: the store, bucket reducer,
host ring and watchdog self-test built with ASan+UBSan and with TSan (tools/sanitize.sh)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++ with sanitizer runtimes")
def test_runtime_selftest_asan_ubsan_tsan(tmp_path):
    p = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize.sh"), str(tmp_path)], capture_output=True,
                       text=True, timeout=900)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "sanitizers clean" in p.stdout
    assert "ERROR: AddressSanitizer" not in p.stderr and "WARNING: ThreadSanitizer" not in p.stderr
