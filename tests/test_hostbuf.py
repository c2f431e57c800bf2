"""Large host buffers unmapped on the runtime's reaper thread (oryx_amd/hostbuf.py,
csrc/runtime/oryx_hostbuf.cpp): a view keeps the mapping alive, the unmap is queued only when
the last reference goes, and the batch layer's text selections / concatenations use it."""

import gc

import numpy as np

from oryx_amd import hostbuf
from oryx_amd.textlines import TextLines, concat_lines


def test_views_keep_the_mapping_and_the_last_one_frees_it_cpu(monkeypatch):
    monkeypatch.setattr(hostbuf, "_MIN", 1 << 16)
    hostbuf.quiesce(10)
    before = hostbuf.stats()["freed_bytes"]
    n = 3 << 20
    a = hostbuf.empty(n)
    assert a.dtype == np.uint8 and a.shape == (n,) and a.flags.writeable
    assert not a[::4096].any()                       # a fresh mapping reads as zeros
    a[:] = 5
    v = a[100:200]
    del a
    gc.collect()
    assert hostbuf.quiesce(10) == 0
    assert hostbuf.stats()["freed_bytes"] == before  # the view still holds it
    assert int(v.sum()) == 500
    del v
    gc.collect()
    assert hostbuf.quiesce(10) == 0
    assert hostbuf.stats()["freed_bytes"] == before + n


def test_small_buffers_stay_numpy_cpu():
    a = hostbuf.empty(1000)
    assert a.base is None and a.shape == (1000,)


def test_text_selection_and_concat_on_native_buffers_cpu(monkeypatch):
    monkeypatch.setattr(hostbuf, "_MIN", 1 << 10)
    lines = ["%d,%d,%.3f" % (i, i * 7 % 13, i / 3) for i in range(5000)]
    tl = TextLines.from_strings(lines)
    mask = np.arange(5000) % 3 == 0
    sel = tl.take(mask)
    assert isinstance(sel.buf, np.ndarray) and sel.buf.base is not None
    assert list(sel) == [l for l, m in zip(lines, mask) if m]
    both = concat_lines([sel, tl.take(~mask)])
    assert len(both) == 5000
    assert sorted(both) == sorted(lines)
    del sel, both
    gc.collect()
    assert hostbuf.quiesce(10) == 0


def test_read_text_file_parallel_pieces_and_final_newline_cpu(tmp_path, monkeypatch):
    monkeypatch.setattr(hostbuf, "_MIN", 1 << 20)
    rs = np.random.default_rng(0)
    body = rs.integers(48, 58, size=(70 << 20) + 12345, dtype=np.uint8)   # > 2 pieces
    body[::97] = 10
    for tail in (b"", b"x", b"\n"):
        p = tmp_path / "part-00000.txt"
        data = body.tobytes() + tail
        p.write_bytes(data)
        got = hostbuf.read_text_file(str(p))
        want = data if data.endswith(b"\n") else data + b"\n"
        assert got.tobytes() == want
    p.write_bytes(b"")
    assert len(hostbuf.read_text_file(str(p))) == 0


def test_reaper_in_a_forked_child_cpu(monkeypatch):
    """A forked child gets a reaper of its own (the parent's thread does not exist there)."""
    import os
    monkeypatch.setattr(hostbuf, "_MIN", 1 << 20)
    a = hostbuf.empty(4 << 20)
    a[:] = 1
    del a
    gc.collect()
    assert hostbuf.quiesce(10) == 0
    pid = os.fork()
    if pid == 0:
        ok = False
        try:
            b = hostbuf.empty(4 << 20)
            b[:] = 2
            del b
            gc.collect()
            ok = hostbuf.quiesce(10) == 0 and hostbuf.stats()["freed_bytes"] == 4 << 20
        finally:
            os._exit(0 if ok else 3)
    _, st = os.waitpid(pid, 0)
    assert os.WEXITSTATUS(st) == 0
