"""Host-runtime concurrency stress under AddressSanitizer + UBSan and ThreadSanitizer
(SURVEY.md section 5.2).  Builds csrc/runtime with csrc/runtime/tests/runtime_stress.cpp:
4 producer threads on two topic handles, 4 partition readers committing offsets, and the
ingest parser, all at once.  (Found and now guards against: appends from threads sharing a
handle were not serialised -- flock is a no-op within one open file description.)"""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_runtime_stress_under_sanitizers(tmp_path):
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "sanitize_runtime.sh"),
                        str(tmp_path)], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "sanitizers clean" in r.stdout
