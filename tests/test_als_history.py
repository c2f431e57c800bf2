"""Resident parsed history (models/als/history.py): the cached per-part-file parse gives the
same codes and columns as one parse of the concatenated text, reuses keyed segments across
generations and drops aged-out ones."""

import os

import numpy as np
import pytest

from oryx_amd import ingest
from oryx_amd.api import Dataset
from oryx_amd.layers.batch import read_past_data
from oryx_amd.models.als import batch as als_batch
from oryx_amd.models.als.history import RatingsHistory
from oryx_amd.textlines import TextLines, concat_lines


def _lines(gen, n, users, items, with_ts=True, deletes=False):
    out = []
    for j in range(n):
        u = "u%d" % gen.integers(users) if gen.random() < 0.5 else str(gen.integers(users))
        i = "i%d" % gen.integers(items)
        if deletes and gen.random() < 0.05:
            v = ""
        else:
            v = "%.3f" % gen.uniform(-1, 5)
        if with_ts and gen.random() < 0.8:
            out.append("%s,%s,%s,%d" % (u, i, v, 1_600_000_000_000 + int(gen.integers(10**9))))
        else:
            out.append("%s,%s,%s" % (u, i, v))
    return out


def _write_parts(root, gen, n_parts, per_part):
    paths = []
    for p in range(n_parts):
        d = os.path.join(root, "oryx-%d.data" % (1000 + p))
        os.makedirs(d)
        path = os.path.join(d, "part-00000.txt")
        with open(path, "w") as f:
            f.write("\n".join(_lines(gen, per_part, 300, 200, deletes=True)) + "\n")
        paths.append(path)
    return paths


def _same(a, b):
    for x, y in zip(a, b):
        np.testing.assert_array_equal(np.asarray(x), np.asarray(y))


def test_history_parse_matches_full_parse_cpu(tmp_path):
    gen = np.random.default_rng(5)
    _write_parts(str(tmp_path), gen, 4, 700)
    past = read_past_data(str(tmp_path)).values()
    assert isinstance(past, TextLines) and len(past.segments) == 4
    new = TextLines.from_strings(_lines(gen, 500, 400, 250))
    data = concat_lines([new, past])
    assert [k is None for k, _, _ in data.segments] == [True, False, False, False, False]

    h = RatingsHistory()
    for default_ts in (0, 123, als_batch._NO_TS):
        u1, i1 = ingest.IdDict(), ingest.IdDict()
        ref = ingest.parse_ratings(data, u1, i1, default_ts=default_ts)
        u2, i2 = ingest.IdDict(), ingest.IdDict()
        got = h.parse_ratings(data, u2, i2, default_ts=default_ts)
        _same(ref[:2], got[:2])
        np.testing.assert_array_equal(np.isnan(ref[2]), np.isnan(got[2]))
        np.testing.assert_array_equal(np.nan_to_num(ref[2]), np.nan_to_num(got[2]))
        _same(ref[3:], got[3:])
        assert u1.keys() == u2.keys() and i1.keys() == i2.keys()
    # the four part files were parsed once, then reused; the unkeyed new data every time
    assert h.stats["misses"] == 4 + 3 and h.stats["hits"] == 2 * 4
    assert len(h) == 4


def test_history_evicts_aged_out_parts_cpu(tmp_path):
    gen = np.random.default_rng(6)
    paths = _write_parts(str(tmp_path), gen, 3, 300)
    h = RatingsHistory()
    h.parse_ratings(read_past_data(str(tmp_path)).values(), ingest.IdDict(), ingest.IdDict(), 0)
    assert len(h) == 3
    os.remove(paths[0])
    os.rmdir(os.path.dirname(paths[0]))
    h.parse_ratings(read_past_data(str(tmp_path)).values(), ingest.IdDict(), ingest.IdDict(), 0)
    assert len(h) == 2 and h.stats["misses"] == 3
    # a rewritten part file (new size / mtime) is parsed again
    with open(paths[1], "a") as f:
        f.write("u1,i1,1.0\n")
    h.parse_ratings(read_past_data(str(tmp_path)).values(), ingest.IdDict(), ingest.IdDict(), 0)
    assert h.stats["misses"] == 4 and len(h) == 2
    # input with no keyed segment at all (every past file aged out) releases the cache too
    # (segments nothing names must not stay resident on the device)
    h.parse_ratings(TextLines.from_strings(_lines(gen, 10, 5, 5)), ingest.IdDict(),
                    ingest.IdDict(), 0)
    assert len(h) == 0 and h.resident_bytes() == 0


def test_als_parse_ratings_with_history_decay_cpu(tmp_path):
    gen = np.random.default_rng(7)
    _write_parts(str(tmp_path), gen, 2, 400)
    data = concat_lines([TextLines.from_strings(_lines(gen, 200, 100, 100)),
                         read_past_data(str(tmp_path)).values()])
    h = RatingsHistory()
    now = 1_600_000_000_000 + 2 * 10**9
    for _ in range(2):
        raw_a, raw_b = [], []
        a = als_batch.parse_ratings(data, ingest.IdDict(), ingest.IdDict(), 0.9, 0.01,
                                    now_ms=now, raw_out=raw_a)
        b = als_batch.parse_ratings(data, ingest.IdDict(), ingest.IdDict(), 0.9, 0.01,
                                    now_ms=now, raw_out=raw_b, history=h)
        for x, y in zip(list(a) + raw_a, list(b) + raw_b):
            np.testing.assert_array_equal(np.nan_to_num(np.asarray(x, dtype=np.float64)),
                                          np.nan_to_num(np.asarray(y, dtype=np.float64)))
    assert h.stats["hits"] == 2


@pytest.mark.gpu
def test_history_device_resident_matches(tmp_path):
    import torch
    gen = np.random.default_rng(8)
    _write_parts(str(tmp_path), gen, 3, 2000)
    data = concat_lines([TextLines.from_strings(_lines(gen, 500, 400, 250)),
                         read_past_data(str(tmp_path)).values()])
    h = RatingsHistory(torch.device("cuda", 0))
    for _ in range(2):
        u1, i1 = ingest.IdDict(), ingest.IdDict()
        ref = ingest.parse_ratings(data, u1, i1, default_ts=7)
        got = h.parse_ratings(data, ingest.IdDict(), ingest.IdDict(), default_ts=7)
        _same(ref[:2], got[:2])
        _same(ref[3:], got[3:])
    assert h.stats["hits"] == 3
    assert all(sg.u.is_cuda for sg in h._segs.values())


def _numeric_lines(gen, n, users, items, odd=False):
    """Numeric-ID rating lines in every form the device parser takes (plain, missing / empty
    fields, exponents, signs, CRLF, extra fields); ``odd``: also a line it must hand back."""
    out = []
    for j in range(n):
        u, i = int(gen.integers(users)), int(gen.integers(items))
        r = gen.random()
        if r < 0.55:
            out.append("%d,%d,%.1f,%d" % (u, i, gen.uniform(0, 5), 1_600_000_000_000 + j))
        elif r < 0.62:
            out.append("%d,%d" % (u, i))
        elif r < 0.68:
            out.append("%d,%d," % (u, i))
        elif r < 0.73:
            out.append("%d,%d,,%d" % (u, i, 1_600_000_000_000 + j))
        elif r < 0.78:
            out.append("%d,%d,%.3e,%d" % (u, i, gen.uniform(-3, 3), j))
        elif r < 0.83:
            out.append("%d,%d,+%.2f" % (u, i, gen.uniform(0, 2)))
        elif r < 0.88:
            out.append("%d,%d,%.4f,%d\r" % (u, i, gen.uniform(0, 9), j))
        elif r < 0.93:
            out.append("%d,%d,2.5,%d,extra,fields" % (u, i, j))
        else:
            out.append("%d,%d,-%.2f," % (u, i, gen.uniform(0, 1)))
    if odd:
        out.insert(len(out) // 2, "007,%d,1.0" % int(gen.integers(items)))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("odd", [False, True])
def test_history_device_parse_matches_host_parse(tmp_path, monkeypatch, odd):
    """The GPU rating parse (oryx_rating_lines + first-appearance numbering on the device)
    gives the host parser's dictionaries, codes, strengths (NaN where empty) and timestamps
    bitwise; a range with a line it does not take (a non-canonical key) is parsed on the host
    instead.  Also through ``parse_ratings(device_out=True)``, the build's path."""
    import torch
    from oryx_amd.models.als import history as hist_mod
    monkeypatch.setattr(RatingsHistory, "DEVICE_PARSE_MIN_BYTES", 0)
    gen = np.random.default_rng(9)
    root = str(tmp_path)
    for p in range(3):
        d = os.path.join(root, "oryx-%d.data" % (1000 + p))
        os.makedirs(d)
        with open(os.path.join(d, "part-00000.txt"), "w", newline="") as f:
            f.write("\n".join(_numeric_lines(gen, 3000, 900, 400, odd=odd and p == 1)) + "\n")
    data = concat_lines([TextLines.from_strings(_numeric_lines(gen, 1500, 1000, 450)),
                         read_past_data(root).values()])
    h = RatingsHistory(torch.device("cuda", 0))
    for default_ts in (0, 77):
        u1, i1 = ingest.IdDict(), ingest.IdDict()
        ref = ingest.parse_ratings(data, u1, i1, default_ts=default_ts)
        u2, i2 = ingest.IdDict(), ingest.IdDict()
        got = h.parse_ratings(data, u2, i2, default_ts=default_ts)
        _same(ref[:2], got[:2])
        np.testing.assert_array_equal(np.isnan(ref[2]), np.isnan(got[2]))
        np.testing.assert_array_equal(np.nan_to_num(ref[2]), np.nan_to_num(got[2]))
        _same(ref[3:], got[3:])
        assert u1.keys() == u2.keys() and i1.keys() == i2.keys()
    assert h.stats.get("device_parsed_bytes", 0) > 0
    assert h.stats.get("device_fallbacks", 0) == (1 if odd else 0)
    # the build's path: columns stay on the device
    u3, i3 = ingest.IdDict(), ingest.IdDict()
    raw = []
    dv = als_batch.parse_ratings(data, u3, i3, raw_out=raw, now_ms=5, history=h,
                                 device_out=True)
    assert all(isinstance(x, torch.Tensor) and x.is_cuda for x in dv)
    u4, i4 = ingest.IdDict(), ingest.IdDict()
    raw_h = []
    hv = als_batch.parse_ratings(data, u4, i4, raw_out=raw_h, now_ms=5)
    for x, y in zip(list(dv) + raw, list(hv) + raw_h):
        np.testing.assert_array_equal(np.nan_to_num(x.cpu().numpy().astype(np.float64)),
                                      np.nan_to_num(np.asarray(y, dtype=np.float64)))
    assert hist_mod._DEVICE_PARSE


def test_history_adopts_new_interval_parse_cpu(tmp_path, monkeypatch):
    """The new interval's parse is reused when its part file is read back."""
    from oryx_amd.layers.batch import save_interval_data
    monkeypatch.setattr(RatingsHistory, "UNKEYED_MIN_BYTES", 1)
    gen = np.random.default_rng(9)
    h = RatingsHistory()
    new = TextLines.from_strings(_lines(gen, 800, 300, 200))
    ref = ingest.parse_ratings(new, ingest.IdDict(), ingest.IdDict(), 0)
    h.parse_ratings(concat_lines([new, read_past_data(str(tmp_path)).values()]),
                    ingest.IdDict(), ingest.IdDict(), 0)
    save_interval_data(str(tmp_path), 1234, Dataset.from_values(new))
    new2 = TextLines.from_strings(_lines(gen, 100, 300, 200))
    data = concat_lines([new2, read_past_data(str(tmp_path)).values()])
    u1, i1 = ingest.IdDict(), ingest.IdDict()
    want = ingest.parse_ratings(data, u1, i1, 0)
    got = h.parse_ratings(data, ingest.IdDict(), ingest.IdDict(), 0)
    assert h.stats["adopted"] == 1 and h.stats["misses"] == 2
    _same(want[:2], got[:2])
    _same(want[3:], got[3:])
    assert len(ref[0]) == 800


def test_history_clear_drops_everything_cpu(monkeypatch):
    monkeypatch.setattr(RatingsHistory, "UNKEYED_MIN_BYTES", 1)
    gen = np.random.default_rng(10)
    h = RatingsHistory()
    h.parse_ratings(TextLines.from_strings(_lines(gen, 300, 50, 50)), ingest.IdDict(),
                    ingest.IdDict(), 0)
    assert h.resident_bytes() > 0
    h.clear()
    assert len(h) == 0 and h.resident_bytes() == 0


def test_known_items_with_test_split_cover_all_data_cpu(tmp_path):
    """With a held-out test split, the published X rows' known items still cover every event
    of the generation (train + test + past): the build's parse of the training lines plus a
    parse of only the test lines, not a re-parse of all the data."""
    import json
    from oryx_amd.transport.producer import MockTopicProducer
    from oryx_amd.utils import config as cfg
    gen = np.random.default_rng(8)
    _write_parts(str(tmp_path / "past"), gen, 2, 400)
    past = read_past_data(str(tmp_path / "past"))
    new = Dataset.from_values(TextLines.from_strings(
        ["u%d,i%d,%.2f,%d" % (gen.integers(80), gen.integers(60), gen.uniform(0.5, 4),
                               1_700_000_000_000 + j * 1000) for j in range(3000)]))
    conf = cfg.overlay_on({
        "oryx.batch.update-class": '"com.cloudera.oryx.app.batch.mllib.als.ALSUpdate"',
        "oryx.ml.eval.test-fraction": 0.3,
        "oryx.ml.eval.candidates": 1,
        "oryx.als.hyperparams.features": 4,
        "oryx.als.iterations": 2,
        "oryx.gpu.device": '"cpu"',
    }, cfg.get_default())
    upd = als_batch.ALSUpdate(conf)
    MockTopicProducer.clear()
    upd.run_update(None, 1_700_000_999_999, new, past, str(tmp_path / "model"),
                   MockTopicProducer())
    assert upd._raw_parse is None and getattr(upd, "_split_test", None) is None
    xs = [json.loads(m) for k, m in MockTopicProducer.get_key_messages()
          if k == "UP" and m.startswith('["X"')]
    assert xs
    want = als_batch.known_items(list(new.values()) + list(past.values()))
    for x in xs:
        assert set(x[3]) == want[x[1]], x[1]
