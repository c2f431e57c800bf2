"""Transport and lambda-tier integration tests, ports of the reference's
``framework/kafka-util`` ITs (ProduceConsumeIT, LargeMessageIT, KafkaUtilsIT),
``framework/oryx-lambda`` ITs (BatchLayerIT, SpeedLayerIT with MockBatchUpdate /
MockSpeedModelManager), ``framework/oryx-ml`` SimpleMLUpdateIT (binomial check of the
train/test split) and ``app/oryx-app`` ALSSpeedIT (golden fold-in vectors to 1e-5).
The native append-only log (csrc/runtime/oryx_log.cpp) stands in for Kafka + ZooKeeper."""

import json
import threading
import time

import numpy as np
import pytest
from scipy import stats

from oryx_amd.api import BatchLayerUpdate, SpeedModelManager
from oryx_amd.layers.batch import BatchLayer
from oryx_amd.layers.speed import SpeedLayer
from oryx_amd.ml.mlupdate import MLUpdate
from oryx_amd.transport import log as tlog
from oryx_amd.transport.producer import LogTopicProducer
from oryx_amd.utils import config as cfg
from oryx_amd.utils import pmml as pmmlu


def _config(tmp_path, **extra):
    overlay = {
        "oryx.id": '"it"',
        "oryx.transport.log-dir": '"%s"' % (tmp_path / "log"),
        "oryx.batch.storage.data-dir": '"file:%s/"' % (tmp_path / "data"),
        "oryx.batch.storage.model-dir": '"file:%s/"' % (tmp_path / "model"),
        "oryx.gpu.device": '"cpu"',
    }
    overlay.update(extra)
    return cfg.overlay_on(overlay, cfg.get_default())


def _drain_topic(root, topic):
    t = tlog.Topic(root, topic)
    c = tlog.TopicConsumer(t, start="earliest")
    out = []
    while True:
        recs = c.poll(100000, 50)
        if not recs:
            break
        out.extend((k, v) for _, _, _, k, v in recs)
    c.close()
    t.close()
    return out


# ---------------------------------------------------------------- kafka-util ITs

def test_produce_consume(tmp_path):
    root = str(tmp_path)
    tlog.maybe_create_topic(root, "T", 4)
    assert tlog.topic_exists(root, "T") and not tlog.topic_exists(root, "U")
    topic = tlog.Topic(root, "T")
    consumer = tlog.TopicConsumer(topic, start="earliest")
    got = []
    done = threading.Event()

    def consume():
        while len(got) < 1000:
            for p, off, ts, k, v in consumer.poll(500, 100):
                got.append((p, k, v))
        done.set()

    th = threading.Thread(target=consume)
    th.start()
    prod = LogTopicProducer("log:" + root, "T", async_=True)
    for i in range(1000):
        prod.send(str(i % 37), "msg-%d" % i)
    prod.close()
    assert done.wait(30)
    th.join()
    consumer.close()
    assert sorted(v for _, _, v in got) == sorted("msg-%d" % i for i in range(1000))
    # a key always lands on the same partition, and per-partition order is append order
    part_of = {}
    for p, k, v in got:
        assert part_of.setdefault(k, p) == p
    for k in part_of:
        seq = [int(v.split("-")[1]) for p, kk, v in got if kk == k]
        assert seq == sorted(seq)
    assert len(set(part_of.values())) > 1
    topic.close()
    tlog.delete_topic(root, "T")
    assert not tlog.topic_exists(root, "T")


def test_large_message(tmp_path):
    root = str(tmp_path)
    max_size = 16 * 1024 * 1024
    tlog.maybe_create_topic(root, "Big", 1, max_message=max_size)
    topic = tlog.Topic(root, "Big")
    big = "x" * (max_size - 1024)
    topic.append("MODEL", big)
    with pytest.raises(tlog.MessageTooLargeError):
        topic.append("MODEL", "y" * (max_size + 1))
    recs = topic.reader(0, 0).poll(10, 1000)
    assert len(recs) == 1 and recs[0][2] == "MODEL" and recs[0][3] == big
    topic.close()


def test_offsets_get_set(tmp_path):
    root = str(tmp_path)
    tlog.maybe_create_topic(root, "In", 3)
    assert tlog.get_offsets(root, "In", "G", 3) == {}
    tlog.set_offsets(root, "In", "G", {0: 5, 2: 7})
    assert tlog.get_offsets(root, "In", "G", 3) == {0: 5, 2: 7}
    tlog.set_offsets(root, "In", "G", {0: 6, 1: 1, 2: 8})
    assert tlog.get_offsets(root, "In", "G", 3) == {0: 6, 1: 1, 2: 8}
    assert tlog.get_offsets(root, "In", "other", 3) == {}


def _segment_files(root, topic, part=0):
    import glob
    import os
    d = os.path.join(root, topic)
    files = [f for f in glob.glob(os.path.join(d, "**", "*"), recursive=True)
             if os.path.isfile(f) and os.path.basename(f) not in ("meta", "lock")
             and not os.path.basename(f).startswith(".")]
    return sorted(files)


@pytest.mark.timeout(60)
def test_torn_tail_is_truncated_not_spun_on(tmp_path):
    """A writer that died mid-append leaves a complete header with a short payload: the end
    offset ignores it, the next append truncates it, and readers never see it."""
    import os
    root = str(tmp_path)
    tlog.maybe_create_topic(root, "Torn", 1)
    topic = tlog.Topic(root, "Torn")
    for i in range(3):
        topic.append(None, "value-%d" % i)
    topic.append(None, "x" * 5000)          # the record that gets torn
    seg = max(_segment_files(root, "Torn"), key=os.path.getsize)
    size = os.path.getsize(seg)
    with open(seg, "r+b") as fh:
        fh.truncate(size - 2000)             # header intact, payload short
    topic.close()
    topic = tlog.Topic(root, "Torn")
    assert topic.end_offset(0) == 3
    assert topic.append(None, "after") == 3
    assert topic.end_offset(0) == 4
    recs = topic.reader(0, 0).poll(100, 100)
    assert [r[3] for r in recs] == ["value-0", "value-1", "value-2", "after"]
    vals, n = topic.reader(0, 0).read_text(4)
    assert n == 4 and vals == ["value-0", "value-1", "value-2", "after"]
    topic.close()


def _legacy_frame(offset, value, key=None, ts=1234):
    """One frame of the first log format ("ORYL", IEEE CRC-32 over offset|ts|key|value)."""
    import struct
    import zlib
    k = b"" if key is None else key
    body = struct.pack("<qq", offset, ts)
    crc = zlib.crc32(k + value, zlib.crc32(body))
    return (struct.pack("<II", 0x4F52594C, crc) + body
            + struct.pack("<II", 0xFFFFFFFF if key is None else len(k), len(value)) + k + value)


@pytest.mark.timeout(60)
def test_legacy_format_segment_is_read_and_appended_to(tmp_path):
    """A segment written by the first log format keeps its records: readers deliver them,
    the end offset counts them and a new append continues after them."""
    import os
    root = str(tmp_path)
    tlog.maybe_create_topic(root, "Old", 1)
    seg = os.path.join(root, "Old", "0", "%020d.log" % 0)
    with open(seg, "wb") as fh:
        for i in range(3):
            fh.write(_legacy_frame(i, b"old-%d" % i, key=b"k" if i == 1 else None))
    topic = tlog.Topic(root, "Old")
    assert topic.end_offset(0) == 3
    assert topic.append(None, "new-3") == 3
    recs = topic.reader(0, 0).poll(100, 100)
    assert [r[3] for r in recs] == ["old-0", "old-1", "old-2", "new-3"]
    assert recs[1][2] == "k"
    # the bulk text read defers keyed records to poll(); from offset 2 on there are none
    vals, n = topic.reader(0, 2).read_text(4)
    assert n == 2 and vals == ["old-2", "new-3"]
    topic.close()


@pytest.mark.timeout(60)
def test_unknown_frame_mid_segment_is_not_truncated(tmp_path):
    """Bytes of an unknown format with more data behind them are corruption, not a torn
    tail: an append fails loudly and leaves the segment as it was."""
    import os
    root = str(tmp_path)
    tlog.maybe_create_topic(root, "Bad", 1)
    topic = tlog.Topic(root, "Bad")
    topic.append(None, "good-0")
    topic.close()
    seg = _segment_files(root, "Bad")[0]
    junk = b"JUNK" + b"\x01" * 200
    with open(seg, "ab") as fh:
        fh.write(junk)
    size = os.path.getsize(seg)
    topic = tlog.Topic(root, "Bad")
    with pytest.raises(Exception, match="refusing to append"):
        topic.append(None, "after")
    assert os.path.getsize(seg) == size
    topic.close()


@pytest.mark.timeout(60)
def test_read_text_roll_then_poll_same_reader(tmp_path):
    """read_text rolling into the next segment drops the poll read-ahead block, so a later
    poll on the same reader continues in the new file instead of replaying the old one."""
    root = str(tmp_path)
    tlog.maybe_create_topic(root, "Roll", 1, segment_bytes=256)
    topic = tlog.Topic(root, "Roll")
    vals = ["rec-%03d-%s" % (i, "p" * 40) for i in range(40)]
    for v in vals:
        topic.append(None, v)
    assert len(_segment_files(root, "Roll")) > 3
    r = topic.reader(0, 0)
    first = r.poll(1, 50)
    assert first[0][3] == vals[0]
    got, n = r.read_text(25)
    assert n == 24 and got == vals[1:25]
    rest = []
    while True:
        recs = r.poll(100, 50)
        if not recs:
            break
        rest.extend(x[3] for x in recs)
    assert rest == vals[25:]
    topic.close()


def test_read_text_grows_for_one_huge_record(tmp_path):
    root = str(tmp_path)
    tlog.maybe_create_topic(root, "Huge", 1, max_message=64 << 20)
    topic = tlog.Topic(root, "Huge")
    big = "z" * (20 << 20)                   # larger than the 16 MB text buffer
    topic.append(None, "small")
    topic.append(None, big)
    topic.append(None, "tail")
    vals, n = topic.reader(0, 0).read_text(3)
    assert n == 3 and vals[0] == "small" and vals[1] == big and vals[2] == "tail"
    topic.close()


# ---------------------------------------------------------------- BatchLayerIT

class MockBatchUpdate(BatchLayerUpdate):
    """Records (timestamp, new data, past data) of every interval (MockBatchUpdate.java)."""
    intervals = []

    def __init__(self, config=None):
        pass

    def run_update(self, context, timestamp, new_data, past_data, model_dir, topic):
        MockBatchUpdate.intervals.append(
            (timestamp, new_data.values(), past_data.values() if past_data else []))


def test_batch_layer_new_and_past_data(tmp_path):
    MockBatchUpdate.intervals = []
    config = _config(tmp_path, **{"oryx.batch.update-class":
                                  "tests.test_lambda_framework.MockBatchUpdate"})
    root = str(tmp_path / "log")
    tlog.maybe_create_topic(root, "OryxInput", 4)
    tlog.maybe_create_topic(root, "OryxUpdate", 1)
    batch = BatchLayer(config)
    batch.run_interval()          # positions the consumer (nothing consumed yet)
    prod = LogTopicProducer("localhost:9092", "OryxInput", config, async_=False)
    produced = []
    for gen in range(3):
        for j in range(50 + 10 * gen):
            m = "g%d-%d" % (gen, j)
            prod.send(str(j), m)
            produced.append(m)
        batch.run_interval()
    batch.run_interval()          # an empty interval runs no update
    prod.close()
    batch.close()
    assert len(MockBatchUpdate.intervals) == 3
    seen = []
    for gen, (ts, new, past) in enumerate(MockBatchUpdate.intervals):
        assert sorted(new) == sorted(m for m in produced if m.startswith("g%d-" % gen))
        assert sorted(past) == sorted(seen)
        seen.extend(new)
    # every record was persisted under data-dir/oryx-<ts>.data
    from oryx_amd.layers.batch import read_past_data
    assert sorted(read_past_data(config.get_string("oryx.batch.storage.data-dir")).values()) == \
        sorted(produced)


class FlakyBatchUpdate(BatchLayerUpdate):
    """Fails its first update, then records like MockBatchUpdate."""
    calls = 0
    intervals = []

    def __init__(self, config=None):
        pass

    def run_update(self, context, timestamp, new_data, past_data, model_dir, topic):
        FlakyBatchUpdate.calls += 1
        if FlakyBatchUpdate.calls == 1:
            raise RuntimeError("injected update failure")
        FlakyBatchUpdate.intervals.append(
            (timestamp, new_data.values(), past_data.values() if past_data else []))


def test_failed_update_saves_no_data_and_retry_does_not_duplicate(tmp_path):
    """The interval's data is published into the past data only after its update succeeded
    (BatchLayer.java:103-124: update, then SaveToHDFSFunction, then UpdateOffsetsFn).  A
    failed update leaves no data dir behind and rewinds the consumer, so the next interval
    sees the same records once as new data and the past data holds them once."""
    import os
    from oryx_amd.layers.batch import read_past_data
    FlakyBatchUpdate.calls = 0
    FlakyBatchUpdate.intervals = []
    config = _config(tmp_path, **{"oryx.batch.update-class":
                                  "tests.test_lambda_framework.FlakyBatchUpdate"})
    root = str(tmp_path / "log")
    data_dir = config.get_string("oryx.batch.storage.data-dir")
    local = str(tmp_path / "data")
    tlog.maybe_create_topic(root, "OryxInput", 2)
    tlog.maybe_create_topic(root, "OryxUpdate", 1)
    batch = BatchLayer(config)
    batch.run_interval()
    prod = LogTopicProducer("localhost:9092", "OryxInput", config, async_=False)
    first = ["a%d" % j for j in range(40)]
    for j, m in enumerate(first):
        prod.send(str(j), m)
    with pytest.raises(RuntimeError, match="injected"):
        batch.run_interval(1000)
    assert not os.path.isdir(local) or not [d for d in os.listdir(local)
                                            if d.startswith("oryx-")]
    batch.run_interval(2000)                  # the retry: same records as new data
    second = ["b%d" % j for j in range(10)]
    for j, m in enumerate(second):
        prod.send(str(j), m)
    batch.run_interval(3000)
    prod.close()
    batch.close()
    assert [sorted(new) for _, new, _ in FlakyBatchUpdate.intervals] == \
        [sorted(first), sorted(second)]
    assert sorted(FlakyBatchUpdate.intervals[1][2]) == sorted(first)
    assert sorted(read_past_data(data_dir).values()) == sorted(first + second)
    assert sorted(os.listdir(local)) == ["oryx-2000.data", "oryx-3000.data"]


# ---------------------------------------------------------------- SpeedLayerIT

class MockSpeedModelManager(SpeedModelManager):
    """Echoes every input as an update; remembers what it consumed."""
    consumed = []

    def __init__(self, config=None):
        pass

    def consume(self, updates, context=None):
        for km in updates:
            MockSpeedModelManager.consumed.append((km.key, km.message))

    def build_updates(self, new_data):
        return ["echo-" + m for m in new_data.values()]


def test_speed_layer_echo(tmp_path):
    MockSpeedModelManager.consumed = []
    config = _config(tmp_path, **{"oryx.speed.model-manager-class":
                                  "tests.test_lambda_framework.MockSpeedModelManager"})
    root = str(tmp_path / "log")
    tlog.maybe_create_topic(root, "OryxInput", 4)
    tlog.maybe_create_topic(root, "OryxUpdate", 1)
    upd = LogTopicProducer("localhost:9092", "OryxUpdate", config, async_=False)
    # MockModelGenerator: MODEL every 10th record, UP otherwise
    for i in range(10):
        upd.send("MODEL" if i % 10 == 0 else "UP", str(i))
    speed = SpeedLayer(config).start(start_timer=False)
    try:
        deadline = time.time() + 20
        while len(MockSpeedModelManager.consumed) < 10 and time.time() < deadline:
            time.sleep(0.05)
        assert MockSpeedModelManager.consumed[:10] == \
            [("MODEL" if i == 0 else "UP", str(i)) for i in range(10)]
        inp = LogTopicProducer("localhost:9092", "OryxInput", config, async_=False)
        for i in range(100):
            inp.send(str(i), "in-%d" % i)
        inp.close()
        assert speed.run_interval() == 100
    finally:
        speed.close()
        upd.close()
    ups = [(k, v) for k, v in _drain_topic(root, "OryxUpdate")[10:]]
    assert sorted(v for _, v in ups) == sorted("echo-in-%d" % i for i in range(100))
    assert all(k == "UP" for k, _ in ups)


# ---------------------------------------------------------------- SimpleMLUpdateIT

class MockMLUpdate(MLUpdate):
    """Model = nothing; eval = test count (MockMLUpdate.java)."""
    train_counts, test_counts = [], []

    def build_model(self, context, train_data, hyper_parameters, candidate_path):
        MockMLUpdate.train_counts.append(len(train_data))
        return pmmlu.build_skeleton_pmml()

    def evaluate(self, context, model, model_parent_path, test_data, train_data):
        MockMLUpdate.test_counts.append(len(test_data))
        return float(len(test_data))


def test_ml_update_train_test_split_is_binomial(tmp_path):
    MockMLUpdate.train_counts, MockMLUpdate.test_counts = [], []
    frac = 0.2
    config = _config(tmp_path, **{"oryx.batch.update-class":
                                  "tests.test_lambda_framework.MockMLUpdate",
                                  "oryx.ml.eval.test-fraction": frac})
    root = str(tmp_path / "log")
    tlog.maybe_create_topic(root, "OryxInput", 4)
    tlog.maybe_create_topic(root, "OryxUpdate", 1)
    batch = BatchLayer(config)
    batch.run_interval()
    prod = LogTopicProducer("localhost:9092", "OryxInput", config, async_=False)
    sizes = [400, 700, 1000]
    for n in sizes:
        for j in range(n):
            prod.send(str(j), "d%d" % j)
        batch.run_interval()
    prod.close()
    batch.close()
    assert len(MockMLUpdate.train_counts) == 3 and len(MockMLUpdate.test_counts) == 3
    past = 0
    for n, train, test in zip(sizes, MockMLUpdate.train_counts, MockMLUpdate.test_counts):
        # train = past data + the new data not held out
        assert train + test == past + n
        dist = stats.binom(n, frac)
        p = dist.cdf(test) if test < dist.mean() else dist.sf(test - 1)
        assert p >= 0.001, (n, test, p)
        past += n
    # the winning model was published on the update topic
    ups = _drain_topic(root, "OryxUpdate")
    assert [k for k, _ in ups] == ["MODEL"] * 3


# ---------------------------------------------------------------- ALSSpeedIT

def _sid(i):
    """ALSUtilsTest.idToStringID: letter ('A' + i mod 26) followed by the number."""
    return chr(ord("A") + i % 26) + str(i)


X_INIT = {_sid(6 + j): v for j, v in enumerate([
    [-0.6790019, 0.1732324], [-0.8232442, -0.9200852], [-1.1865344, 0.44631857],
    [-0.20789514, 0.5303508]])}
Y_INIT = {_sid(1 + j): v for j, v in enumerate([
    [-0.7203235, 0.45654634], [-0.77601856, -0.34911805], [-0.5384191, 0.7197065],
    [-1.0381957, -0.22146331], [-0.31787223, -0.6780096]])}
A_KNOWN = {_sid(6): ["1", "4"], _sid(7): ["2", "4", "5"], _sid(8): ["1", "2", "3", "4"],
           _sid(9): ["3"]}
AT_KNOWN = {_sid(1): ["6", "8"], _sid(2): ["7", "8"], _sid(3): ["8", "9"],
            _sid(4): ["6", "7", "8"], _sid(5): ["7"]}
X_EXPECTED = {_sid(100 + j): v for j, v in enumerate([
    [-0.20859924, 0.25232133], [-0.22472803, -0.1929485], [-0.15592135, 0.3977631],
    [-0.3006522, -0.12239703], [-0.09205295, -0.37471837]])}
Y_EXPECTED = {_sid(105 + j): v for j, v in enumerate([
    [-0.19663288, 0.09574106], [-0.23840417, -0.50850725], [-0.34360975, 0.2466687],
    [-0.060204573, 0.29311115]])}


def test_als_speed_golden_vectors(tmp_path):
    """ALSSpeedIT: a MODEL + 9 UP messages (an SVD factorisation of a 4x5 matrix), then 9
    inputs that each pair a new user or item with a known one -> exactly 9 updates whose
    vectors match the reference's golden values to 1e-5."""
    _als_speed_golden(tmp_path)


@pytest.mark.gpu
def test_als_speed_golden_vectors_gpu(tmp_path, cuda):
    """The same golden ALSSpeedIT check through the fused HIP fold-in (device model)."""
    _als_speed_golden(tmp_path)


def _als_speed_golden(tmp_path):
    config = _config(tmp_path, **{
        "oryx.speed.model-manager-class": "com.cloudera.oryx.app.speed.als.ALSSpeedModelManager",
        "oryx.als.hyperparams.features": 2})
    root = str(tmp_path / "log")
    tlog.maybe_create_topic(root, "OryxInput", 4)
    tlog.maybe_create_topic(root, "OryxUpdate", 1)
    upd = LogTopicProducer("localhost:9092", "OryxUpdate", config, async_=False)
    doc = pmmlu.build_skeleton_pmml()
    doc.add_extension("features", 2)
    doc.add_extension("implicit", "true")
    doc.add_extension_content("XIDs", list(X_INIT))
    doc.add_extension_content("YIDs", list(Y_INIT))
    upd.send("MODEL", pmmlu.to_string(doc))
    for i in range(1, 10):          # MockALSModelUpdateGenerator ids 1..9
        sid = _sid(i)
        if i >= 6:
            upd.send("UP", json.dumps(["X", sid, X_INIT[sid], A_KNOWN[sid]]))
        else:
            upd.send("UP", json.dumps(["Y", sid, Y_INIT[sid], AT_KNOWN[sid]]))
    speed = SpeedLayer(config).start(start_timer=False)
    try:
        deadline = time.time() + 30
        while time.time() < deadline and (
                speed.manager.model is None or speed.manager.model.get_fraction_loaded() < 1.0
                or speed.manager.model.X.size() < 4 or speed.manager.model.Y.size() < 5):
            time.sleep(0.05)
        inp = LogTopicProducer("localhost:9092", "OryxInput", config, async_=False)
        now = int(time.time() * 1000)
        for i in range(9):              # MockALSInputGenerator
            large, small = _sid(100 + i), _sid(1 + i)
            inp.send(str(i), ("%s,%s,1,%d" % (large, small, now)) if i < 5 else
                     ("%s,%s,1,%d" % (small, large, now)))
        inp.close()
        assert speed.run_interval() == 9
    finally:
        speed.close()
        upd.close()
    ups = _drain_topic(root, "OryxUpdate")
    assert len(ups) == 19 and ups[0][0] == "MODEL"
    for k, m in ups[10:]:
        assert k == "UP"
        u = json.loads(m)
        expected = (X_EXPECTED if u[0] == "X" else Y_EXPECTED)[u[1]]
        np.testing.assert_allclose(u[2], expected, atol=1e-5)
        other = _sid(int(u[1][1:]) - 99)
        assert u[3] == [other]
