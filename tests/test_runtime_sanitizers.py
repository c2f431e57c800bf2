"""Host-runtime concurrency stress under AddressSanitizer + UBSan and ThreadSanitizer
(SURVEY.md section 5.2).  Builds csrc/runtime (log, ingest, HTTP) with two drivers:

* csrc/runtime/tests/runtime_stress.cpp: 4 producer threads on two topic handles, 4 partition
  readers committing offsets, and the ingest parser, all at once;
* csrc/runtime/tests/runtime_stress2.cpp: oryx_log_append_fill writers (fill callbacks
  formatting into the mapped segment) on two handles with small segments, while a frame
  reader (poll_frames) and a text reader (read_text) tail the partition across the rolls;
  the native HTTP server with leader / follower handler threads under keep-alive, pipelined,
  chunked (small pieces), oversized (413), header-flood (431), malformed (400) and abruptly
  closing clients; oryx_topn_prep from 6 threads; the native thread pool entered from 6
  threads (blob hashing, content digests).

Found and guard against: appends from threads sharing a handle were not serialised (flock
is a no-op within one open file description); the HTTP handlers' timed waits used the steady
clock (pthread_cond_clockwait, which ThreadSanitizer does not intercept, so it reported a
double lock) -- they now wait on the system clock."""

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
