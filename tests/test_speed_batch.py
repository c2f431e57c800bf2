"""The speed layer's native micro-batch path (ingest.SpeedBatch, csrc/runtime/oryx_ingest.cpp
``oryx_speed_*``) against the dictionary path it replaces on the GPU: same aggregated pairs
(ALSUpdate.aggregateScores semantics, deletes, quoted / JSON lines, IDs the stores lack) and
the same UP messages; and the update log's large-append path (mapped segment, preallocated
tail, publish-by-magic)."""

import json
import os

import numpy as np

from oryx_amd import ingest
from oryx_amd.models.als.batch import aggregate_scores
from oryx_amd.ops.textfmt import format_rows
from oryx_amd.textlines import TextLines
from oryx_amd.transport import log as tlog


def _stores(n_x=1000, n_y=500):
    xm, ym = ingest.RowMap(), ingest.RowMap()
    xids = ["U%d" % j for j in range(n_x)]
    yids = ["I%d" % j for j in range(n_y)]
    xrow = {k: 3 * j + 1 for j, k in enumerate(xids)}
    yrow = {k: 2 * j for j, k in enumerate(yids)}
    xm.set(xids, np.array([xrow[k] for k in xids]))
    ym.set(yids, np.array([yrow[k] for k in yids]))
    return xm, ym, xrow, yrow


def _lines(n, seed=1):
    g = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        u, it = "U%d" % g.integers(0, 1100), "I%d" % g.integers(0, 520)
        v = "" if g.random() < 0.03 else "%.2f" % (g.random() * 3)
        t = 1000 + int(g.integers(0, 50))
        r = g.random()
        if r < 0.05:
            out.append('"%s","%s",%s,%d' % (u, it, v, t))
        elif r < 0.1:
            out.append('["%s","%s",%s,%d]' % (u, it, v if v else '""', t))
        elif r < 0.12:
            out.append("%s,%s,%s" % (u, it, v or "1"))          # no timestamp
        else:
            out.append("%s,%s,%s,%d" % (u, it, v, t))
    return out


def test_speed_batch_matches_dictionary_path():
    xm, ym, xrow, yrow = _stores()
    lines = _lines(30000)
    tl = TextLines.from_strings(lines)
    sb = ingest.SpeedBatch()
    for implicit in (True, False):
        n = sb.parse(tl, xm, ym)
        u, i, s = sb.aggregate(implicit)
        users, items = ingest.IdDict(), ingest.IdDict()
        a, b, c, d = ingest.parse_ratings(tl, users, items, 0)
        assert n == len(a)
        au, ai, av = aggregate_scores(a, b, c, d, implicit)
        uk, ik = users.keys(), items.keys()
        want = {(uk[p], ik[q]): v for p, q, v in zip(au.tolist(), ai.tolist(), av.tolist())}
        assert len(u) == len(want)
        # rows resolve to the store's rows; IDs the stores lack are -1 and listed as new keys
        assert set((u[u >= 0] - 1) % 3) == {0} and set(i[i >= 0] % 2) == {0}
        new_u = set(ingest.blob_strings(*sb.new_keys(0)))
        new_i = set(ingest.blob_strings(*sb.new_keys(1)))
        assert new_u == {k for k in uk if k not in xrow}
        assert new_i == {k for k in ik if k not in yrow}
        # the assembled messages carry each pair's keys and value-ordered rows
        m = len(u)
        xr = format_rows(np.asarray(s, dtype=np.float32)[:, None].repeat(2, 1))
        yr = format_rows(np.asarray(s, dtype=np.float32)[:, None].repeat(3, 1))
        vx = np.ones(m, np.uint8)
        vy = (u >= 0).astype(np.uint8)
        blk = sb.assemble(0, m, xr, yr, vx, vy, True)
        msgs = [json.loads(x) for x in bytes(blk.buf).decode().strip().split("\n")]
        assert len(msgs) == int(vx.sum() + vy.sum()) == len(blk)
        got = {(mm[1], mm[3][0]): mm[2][0] for mm in msgs if mm[0] == "X"}
        assert set(got) == set(want)
        for key, v in got.items():
            assert abs(v - np.float32(want[key])) <= 1e-6 * max(1.0, abs(v))
        ys = [mm for mm in msgs if mm[0] == "Y"]
        assert all(mm[1] in yrow or mm[1] not in yrow for mm in ys)
        assert all(mm[3][0] in xrow for mm in ys)      # Y rows only for users in the store


def test_log_large_append_mapped_and_preallocated(tmp_path, monkeypatch):
    """A block past the mapped-append threshold lands through the segment mapping, the
    segment keeps a zero tail for the next block, readers stop at that tail, and a later
    append (large or small) continues at the data's end."""
    root = str(tmp_path)
    tlog.maybe_create_topic(root, "Up", 1, max_message=1 << 30)
    topic = tlog.Topic(root, "Up")
    big = ["x" * 300 + "%06d" % j for j in range(20000)]         # ~6 MB: mapped path
    topic.append_batch([("UP", v) for v in big])
    seg = [f for f in os.listdir(os.path.join(root, "Up", "0")) if f.endswith(".log")][0]
    size = os.path.getsize(os.path.join(root, "Up", "0", seg))
    assert topic.end_offset(0) == 20000
    assert size > sum(len(v) + 32 + 2 for v in big)          # preallocated zero tail
    topic.append(None, "small-after")
    topic.append_batch([("UP", v) for v in big[:100]])
    assert topic.end_offset(0) == 20101
    recs = []
    r = topic.reader(0, 0)
    while True:
        got = r.poll(50000, 50)
        if not got:
            break
        recs.extend(got)
    assert len(recs) == 20101
    assert recs[20000][3] == "small-after" and recs[20100][3] == big[99]
    topic.close()
    # reopened by another handle: the zero tail is not mistaken for corruption
    t2 = tlog.Topic(root, "Up")
    assert t2.append(None, "third") == 20101
    t2.close()


def test_log_unpublished_block_is_truncated(tmp_path):
    """A block whose writer died before publishing its first frame's magic (zero magic,
    written header) was never readable: the next append truncates it away."""
    root = str(tmp_path)
    tlog.maybe_create_topic(root, "T", 1)
    topic = tlog.Topic(root, "T")
    topic.append(None, "a")
    topic.close()
    seg = os.path.join(root, "T", "0", [f for f in os.listdir(os.path.join(root, "T", "0"))
                                         if f.endswith(".log")][0])
    import struct
    body = struct.pack("<qq", 1, 5) + struct.pack("<II", 0xFFFFFFFF, 3) + b"zzz"
    with open(seg, "ab") as fh:
        fh.write(struct.pack("<II", 0, 123) + body + b"\x01" * 64)
    t2 = tlog.Topic(root, "T")
    assert t2.end_offset(0) == 1
    assert t2.append(None, "b") == 1
    assert [x[3] for x in t2.reader(0, 0).poll(10, 10)] == ["a", "b"]
    t2.close()


def _read_all(topic):
    recs, r = [], topic.reader(0, 0)
    while True:
        got = r.poll(100000, 50)
        if not got:
            return recs
        recs.extend(got)


def test_deferred_block_formats_into_the_log(tmp_path):
    """A deferred UP block appended to a native topic (formatted by the log's writer
    threads in the segment, CRCs included) leaves exactly the records of the assembled
    block -- on the pwrite path and on the mapped large-append path, keys needing JSON
    escapes included; used after the batch's next parse it refuses."""
    import pytest
    xm, ym, _, _ = _stores()
    lines = _lines(20000) + ['["U\\"q","Iü",1.5,1001]', '["U1","I\\\\x",2,1002]']
    tl = TextLines.from_strings(lines)
    sb = ingest.SpeedBatch()
    sb.parse(tl, xm, ym)
    u, i, s = sb.aggregate(True)
    m = len(u)
    g = np.random.default_rng(3)
    xr = format_rows(g.normal(size=(m, 24)).astype(np.float32))
    yr = format_rows(g.normal(size=(m, 24)).astype(np.float32))
    vx = (g.random(m) < 0.9).astype(np.uint8)
    vy = (g.random(m) < 0.8).astype(np.uint8)
    for rep in range(2):
        # the full block (> 4 MB) takes the mapped append, the half one pwrite
        root = str(tmp_path / ("t%d" % rep))
        tlog.maybe_create_topic(root, "A", 1, max_message=1 << 24)
        tlog.maybe_create_topic(root, "B", 1, max_message=1 << 24)
        a, b = tlog.Topic(root, "A"), tlog.Topic(root, "B")
        for lo, hi, with_known in ((0, m, True), (17, m // 2, False)):
            a.append_block(sb.assemble(lo, hi, xr, yr, vx, vy, with_known), key="UP")
            blk = sb.deferred(lo, hi, xr, yr, vx, vy, with_known)
            assert len(blk) == int(vx[lo:hi].sum() + vy[lo:hi].sum())
            b.append_block(blk, key="UP")
        sizes = [os.path.getsize(os.path.join(root, "B", "0", f))
                 for f in os.listdir(os.path.join(root, "B", "0")) if f.endswith(".log")]
        assert max(sizes) > 4 << 20
        ra, rb = _read_all(a), _read_all(b)
        assert len(ra) == len(rb) > m
        assert [(x[2], x[3]) for x in ra] == [(x[2], x[3]) for x in rb]
        assert any('"U\\"q"' in x[3] for x in rb) and any("\\u00fc" in x[3] for x in rb)
        a.close()
        b.close()
    blk = sb.deferred(0, m, xr, yr, vx, vy, True)
    assert list(blk)[:3] == list(sb.assemble(0, m, xr, yr, vx, vy, True))[:3]
    stale = sb.deferred(0, m, xr, yr, vx, vy, True)
    sb.parse(tl, xm, ym)
    with pytest.raises(RuntimeError):
        stale.materialize()


def test_leaf_update_formatter_matches_json():
    """ingest.format_leaf_updates (the RDF speed layer's native formatter) writes the bytes of
    the reference-format messages json.dumps would: classification '[tree,ID,{"c":n,...}]'
    over the nonzero classes, regression '[tree,ID,mean,count]' with Python float repr."""
    g = np.random.default_rng(2)
    ids = ["r", "r-+", 'r-"q', "rü+-", "r--+-+-+"]
    blob, ends = ingest.strings_blob([json.dumps(i) for i in ids])
    n = 40
    idx = g.integers(0, len(ids), n)
    trees = g.integers(0, 50, n)
    counts = g.integers(0, 4, (n, 3)) * (g.random((n, 3)) < 0.7)
    counts[:, 0] += 1
    blk = ingest.format_leaf_updates(trees, blob, ends, idx, counts, 3)
    want = ['[%d,%s,{%s}]' % (t, json.dumps(ids[k]), ",".join('"%d":%d' % (c, v) for c, v in
                                                          enumerate(row) if v))
            for t, k, row in zip(trees.tolist(), idx.tolist(), counts.tolist())]
    assert list(blk) == want
    means = g.standard_normal(n) * 10.0 ** g.integers(-8, 8, n)
    cnt = g.integers(1, 1000, n)
    blk = ingest.format_leaf_updates(trees, blob, ends, idx, cnt, 0, means)
    want = [json.dumps([t, ids[k], m, c], separators=(",", ":"))
            for t, k, m, c in zip(trees.tolist(), idx.tolist(), means.tolist(), cnt.tolist())]
    assert list(blk) == want


def test_publish_blocks_order_errors_and_reuse():
    """layers.speed.publish_blocks: blocks land in order through the persistent writer, at
    most two wait, a failing append surfaces on the caller's thread and stops the rest, and
    the writer serves the next call afterwards."""
    import pytest
    from oryx_amd.api import MessageBlock
    from oryx_amd.layers.speed import publish_blocks

    class Prod:
        def __init__(self, fail_at=None):
            self.got, self.fail_at = [], fail_at

        def send_block(self, key, b):
            if self.fail_at is not None and len(self.got) == self.fail_at:
                raise IOError("disk full")
            self.got.append(list(b))

        def send_many(self, pairs):
            self.send_block("UP", [m for _, m in pairs])

    def block(msgs):
        ends = np.cumsum([len(m) + 1 for m in msgs]) - 1
        return MessageBlock(("\n".join(msgs) + "\n").encode(), ends)

    def blocks(n, made):
        for j in range(n):
            made.append(j)
            msgs = ["m%d-%d" % (j, k) for k in range(3)]
            yield block(msgs) if j % 2 else msgs

    p = Prod()
    st: dict = {}
    assert publish_blocks(p, blocks(7, []), st) == 21
    assert p.got == [["m%d-%d" % (j, k) for k in range(3)] for j in range(7)]
    assert st["write_ms"] >= 0 and st["tail_ms"] >= 0
    bad = Prod(fail_at=2)
    made: list = []
    with pytest.raises(IOError):
        publish_blocks(bad, blocks(50, made), {})
    assert len(bad.got) == 2 and len(made) < 50
    p2 = Prod()
    assert publish_blocks(p2, blocks(3, []), None) == 9 and len(p2.got) == 3


def _double_cases(n_random=200000, seed=7):
    g = np.random.default_rng(seed)
    bits = g.integers(0, 2 ** 63, n_random, dtype=np.int64).view(np.uint64)
    bits[: n_random // 2] |= np.uint64(1) << np.uint64(63)
    vals = [bits.view(np.float64)]
    ints = g.integers(-2 ** 60, 2 ** 60, 20000).astype(np.float64)
    vals += [ints, np.nextafter(ints, np.inf), g.integers(0, 10 ** 6, 20000) / 10.0 ** 3,
             np.ldexp(1.0, np.arange(-1074, 1024)), 10.0 ** np.arange(-300, 300),
             np.array([0.0, -0.0, np.nan, np.inf, -np.inf, 5e-324, 1.7976931348623157e308,
                       0.1, 0.2, 0.3, 1e16, 1e15, 123456789012345680.0, 1e-5, 1e-4, 9.5e-5])]
    return np.concatenate(vals)


def test_f64_repr_host_matches_python_repr():
    """The host double formatter (the reference for the device one) writes Python's repr
    (json.dumps spelling for NaN / Infinity)."""
    v = _double_cases(50000)
    slots, lens = ingest.f64_repr_slots(v)
    got = [bytes(slots[j, :lens[j]]).decode() for j in range(len(v))]
    want = [json.dumps(float(x)) for x in v.tolist()]
    assert got == want


def test_ryu_formatter_matches_host_formatter(tmp_path):
    """csrc/kernels/ryu_d2s.h (the device formatter's algorithm) compiled for the host equals
    the runtime's formatter byte for byte over random bit patterns, integers, short decimals,
    powers and running means (csrc/runtime/tests/ryu_check.cpp)."""
    import shutil
    import subprocess
    if shutil.which("g++") is None:
        import pytest
        pytest.skip("no g++")
    from oryx_amd import native
    native.runtime()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "oryx_amd", "_native")
    exe = str(tmp_path / "ryu_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(root, "csrc", "kernels"),
                    os.path.join(root, "csrc", "runtime", "tests", "ryu_check.cpp"),
                    "-L", lib, "-loryx_runtime", "-Wl,-rpath," + lib, "-o", exe], check=True)
    r = subprocess.run([exe, "2"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "all equal" in r.stdout, r.stdout + r.stderr
