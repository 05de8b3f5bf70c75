"""ThreadSanitizer and AddressSanitizer+UBSan runs of the native CPU
runtime (loader producer/consumer ring with 1-8 workers, concurrent Go engine), including
determinism across worker counts and start_seq resume.  Host code only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_loader_and_engine_under_tsan_and_asan():
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize.sh")], capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.count("stress ok") == 2
