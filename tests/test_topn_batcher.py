"""Serving top-N micro-batcher (models/als/serving.py TopNBatcher): a lone client runs inline,
concurrent clients are batched into shared scans, and every request gets its own answer."""

import threading
import time

from oryx_amd.models.als.serving import TopNBatcher


class _FakeIndex:
    def __init__(self, delay=0.0):
        self.delay = delay
        self.scans = []
        self.threads = set()

    def scan(self, qs):
        self.scans.append(len(qs))
        self.threads.add(threading.current_thread().name)
        if self.delay:
            time.sleep(self.delay)
        return [("r", q) for q in qs]


def test_lone_client_runs_inline_cpu():
    idx = _FakeIndex()
    b = TopNBatcher(idx, max_batch=8, wait_s=0.0)
    for k in range(20):
        assert b.submit(k) == ("r", k)
    assert b.inline == 20 and b.requests == 20
    assert idx.threads == {threading.current_thread().name}
    b.close()


def test_concurrent_clients_are_batched_cpu():
    idx = _FakeIndex(delay=0.01)
    b = TopNBatcher(idx, max_batch=16, wait_s=0.0)
    out = {}
    errs = []

    def client(c):
        try:
            for k in range(15):
                q = (c, k)
                out[q] = b.submit(q)
        except Exception as e:   # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=client, args=(c,)) for c in range(6)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=60)
    assert not errs and len(out) == 90
    assert all(v == ("r", q) for q, v in out.items())
    assert b.requests == 90 and sum(idx.scans) == 90
    # queued-up requests shared launches
    assert max(idx.scans) > 1 and b.batches < 90
    b.close()


def test_pipelined_batches_keep_their_own_results_cpu():
    """An index without scan_async: batch B is launched before batch A is finished, so A's
    finisher must return A's results (regression: a late-bound closure handed A B's)."""
    idx = _FakeIndex(delay=0.002)
    b = TopNBatcher(idx, max_batch=3, wait_s=0.0)
    out = {}
    errs = []

    def client(c):
        try:
            for k in range(40):
                q = (c, k)
                out[q] = b.submit(q)
        except Exception as e:   # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=client, args=(c,)) for c in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=60)
    assert not errs and len(out) == 320
    bad = [q for q, v in out.items() if v != ("r", q)]
    assert not bad, bad[:5]
    b.close()


def test_wait_window_disables_inline_cpu():
    idx = _FakeIndex()
    b = TopNBatcher(idx, max_batch=8, wait_s=0.001)
    assert b.submit(1) == ("r", 1)
    assert b.inline == 0 and b.requests == 1
    b.close()
