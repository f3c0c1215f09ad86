"""Race / memory-error detection for the host runtime: the C++ self-test
(tests/native/runtime_selftest.cpp) built with ASan+UBSan and with TSan, driving the buffer manager from
several threads while the native WorkerQueue prefetches and flushes the same sets."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_runtime_under_asan_ubsan_tsan(tmp_path):
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "sanitize_native.sh"), str(tmp_path)],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "sanitizers clean" in r.stdout
