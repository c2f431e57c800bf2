"""Feature-row parsing of the k-means / RDF batch layers (models/features.py): a buffer made of
several segments (the new interval followed by past part files, as a later generation sees it)
parses to the same rows and categorical encodings as one parse of the concatenated text, with
and without the resident history.  Regression: categorical fields of every segment after the
first were read at the wrong byte offsets (values such as "," became categories).  On a GPU the
all-numeric parse runs on the device (csrc/kernels/csv.hip) and matches the host parser
bitwise."""

import numpy as np
import pytest
import torch

from oryx_amd.models.features import FeatureHistory, parse_features
from oryx_amd.models.schema import InputSchema
from oryx_amd.textlines import TextLines, concat_lines
from oryx_amd.utils import config as cfg


def _schema():
    conf = cfg.overlay_on({
        "oryx.input-schema.feature-names": '["a", "b", "c", "color", "label"]',
        "oryx.input-schema.categorical-features": '["color", "label"]',
        "oryx.input-schema.target-feature": '"label"',
    }, cfg.get_default())
    return InputSchema(conf)


def _lines(rs, n, colors):
    out = []
    for _ in range(n):
        a, b, c = rs.normal(0, 1, 3).round(2)
        out.append("%s,%s,%s,%s,%s" % (a, b, c, colors[rs.integers(0, len(colors))],
                                       "yes" if a + b > 0 else "no"))
    return out


def test_multi_segment_parse_matches_one_parse_cpu():
    rs = np.random.default_rng(3)
    schema = _schema()
    seg1 = _lines(rs, 300, ["red", "green"])
    seg2 = _lines(rs, 500, ["blue", "green", "violet"])
    seg3 = _lines(rs, 200, ["red", "cyan"])
    parts = []
    for i, seg in enumerate((seg1, seg2, seg3)):
        tl = TextLines.from_strings(seg)
        if i:
            tl.with_key(("part", i))       # past part files carry a key
        parts.append(tl)
    multi = concat_lines(parts)
    assert len(multi.segment_list()) >= 1
    one = parse_features(TextLines.from_strings(seg1 + seg2 + seg3), schema,
                         torch.device("cpu"))
    for hist in (None, FeatureHistory(torch.device("cpu"))):
        for _ in range(2):                 # second pass: the history's cached segments
            got = parse_features(multi, schema, torch.device("cpu"), history=hist)
            assert got.values == one.values
            assert sorted(got.values[3]) == ["blue", "cyan", "green", "red", "violet"]
            assert sorted(got.values[4]) == ["no", "yes"]
            assert torch.equal(torch.nan_to_num(got.full, -7.0),
                               torch.nan_to_num(one.full, -7.0))


def _numeric_schema(n):
    names = ["f%d" % i for i in range(n)]
    conf = cfg.overlay_on({
        "oryx.input-schema.feature-names": "[%s]" % ",".join('"%s"' % x for x in names),
        "oryx.input-schema.numeric-features": "[%s]" % ",".join('"%s"' % x for x in names),
    }, cfg.get_default())
    return InputSchema(conf)


def test_general_parser_takes_crlf_lines():
    """A block the native parser refuses (a quoted field) goes through the general parser,
    which strips a CRLF line's CR as the native parsers do (it read '\r' as a value)."""
    schema = _numeric_schema(3)
    tl = TextLines.from_strings(['"1.5",2,3\r', "4,5,\r", "7,8,9"])
    blk = parse_features(tl, schema, torch.device("cpu"), dtype=torch.float64)
    got = blk.full.numpy()
    assert got[0].tolist() == [1.5, 2.0, 3.0] and got[2].tolist() == [7.0, 8.0, 9.0]
    assert got[1][:2].tolist() == [4.0, 5.0] and np.isnan(got[1][2])


def _numeric_lines(rs, n, F):
    out = []
    for j in range(n):
        vals = []
        for f in range(F):
            kind = rs.integers(0, 9)
            x = rs.normal(0, 50)
            if kind == 0:
                vals.append("")                              # empty: NaN
            elif kind == 1:
                vals.append("%de%d" % (rs.integers(-999, 999), rs.integers(-20, 20)))
            elif kind == 2:
                vals.append("+%.6f" % abs(x))
            elif kind == 3:
                vals.append("%d" % int(x))
            elif kind == 4:
                vals.append("%.15g" % x)                     # 15 significant digits
            else:
                vals.append("%.2f" % x)
        out.append(",".join(vals) + ("\r" if j % 7 == 0 else ""))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("wide", [False, True])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_device_csv_parse_matches_host_bitwise(cuda, dtype, wide, monkeypatch):
    """csv.hip on the device == the host parser, bitwise (NaN where empty), for numeric rows
    with signs, exponents, 17-digit values, empty fields, trailing commas and CR line ends;
    lines outside the fast path are parsed on the host and written in (same results).  Both
    kernels: one thread per line, and one wave per line (``wide``: a line past the wave's LDS
    capacity goes to the host too)."""
    from oryx_amd import native
    from oryx_amd.models import features as feats
    native.require_kernels()
    monkeypatch.setattr(feats, "WIDE_LINE_MIN_BYTES", 0 if wide else 1 << 40)
    rs = np.random.default_rng(11)
    F = 37
    schema = _numeric_schema(F)
    lines = _numeric_lines(rs, 5000, F)
    lines[17] = lines[17][:lines[17].rfind(",")] + ","           # trailing comma: empty last
    # 17 significant digits (mantissa past 2^53) and an exponent past 22: those lines are
    # parsed on the host and written into the device matrix
    long = ["%.17g," % rs.normal(0, 50) + ",".join(["2.5"] * (F - 1)) for _ in range(40)]
    mixed = list(lines)
    for j, l in zip(range(3, 5000, 125), long):
        mixed[j] = l
    mixed[9] = "1.5E+30," + ",".join(["1"] * (F - 1))
    mixed[12] = "1." + "0" * 13000 + "," + ",".join(["3"] * (F - 1))  # past 12 KB
    mixed[4999] = ",".join(["7"] * F)                                # the last line
    variants = {"plain": lines, "mixed": mixed}
    for name, ls in variants.items():
        tl = TextLines.from_strings(ls)
        monkeypatch.setenv("ORYX_GPU_CSV", "0")
        host = parse_features(tl, schema, torch.device(cuda), dtype=dtype)
        monkeypatch.setenv("ORYX_GPU_CSV", "1")
        hist = FeatureHistory(torch.device(cuda), keep=False)
        dev = hist.parse(tl, schema, dtype)
        assert dev.full.dtype == dtype and dev.full.shape == host.full.shape
        a = host.full.cpu().numpy().view(np.int64 if dtype == torch.float64 else np.int32)
        b = dev.full.cpu().numpy().view(np.int64 if dtype == torch.float64 else np.int32)
        assert np.array_equal(a, b), name
        assert hist.stats.get("device_parsed_bytes", 0) > 0, name


@pytest.mark.gpu
@pytest.mark.parametrize("wide", [False, True])
def test_device_csv_parse_with_categoricals_matches_host(cuda, wide, monkeypatch):
    """Categorical fields through the device parser: spans on the device, codes on the host
    -- the same matrix (bitwise) and the same distinct values in first-appearance order as the
    host parser, over several segments and through the resident history; by either kernel
    (one thread or one wave per line)."""
    from oryx_amd import native
    from oryx_amd.models import features as feats
    native.require_kernels()
    monkeypatch.setattr(feats, "WIDE_LINE_MIN_BYTES", 0 if wide else 1 << 40)
    rs = np.random.default_rng(5)
    schema = _schema()
    parts = []
    for i, colors in enumerate((["red", "green"], ["blue", "", "violet"], ["red", "cyan"])):
        tl = TextLines.from_strings(_lines(rs, 700 + 300 * i, colors))
        if i:
            tl.with_key(("part", i))
        parts.append(tl)
    multi = concat_lines(parts)
    for dtype in (torch.float32, torch.float64):
        monkeypatch.setenv("ORYX_GPU_CSV", "0")
        host = parse_features(multi, schema, torch.device(cuda), dtype=dtype)
        monkeypatch.setenv("ORYX_GPU_CSV", "1")
        hist = FeatureHistory(torch.device(cuda))
        for _ in range(2):
            dev = parse_features(multi, schema, torch.device(cuda), dtype=dtype, history=hist)
            assert dev.values == host.values
            a = torch.nan_to_num(host.full, -7.0).cpu().numpy()
            b = torch.nan_to_num(dev.full, -7.0).cpu().numpy()
            assert np.array_equal(a, b)
        assert hist.stats.get("device_parsed_bytes", 0) > 0


def test_lazy_split_selection_parse_matches_materialized_cpu(monkeypatch):
    _lazy_split_case(torch.device("cpu"), monkeypatch)


@pytest.mark.gpu
def test_lazy_split_selection_parse_matches_materialized_gpu(cuda, monkeypatch):
    from oryx_amd import native
    native.require_kernels()
    monkeypatch.setenv("ORYX_GPU_CSV", "1")
    _lazy_split_case(torch.device(cuda), monkeypatch)


def _lazy_split_case(dev, monkeypatch):
    """A train / test split as LineSelections of the interval (MLUpdate's default split):
    the parser parses the interval once and selects rows, renumbering categorical codes in
    the selection's own first-appearance order -- the same block as a parse of the selected
    text -- and the interval's parse is adopted when its bytes come back as a part file."""
    from oryx_amd.textlines import LineConcat, LineSelection
    monkeypatch.setattr(FeatureHistory, "UNKEYED_MIN_BYTES", 1)
    rs = np.random.default_rng(7)
    schema = _schema()
    new = TextLines.from_strings(_lines(rs, 900, ["red", "green", "blue", "cyan", ""]))
    past = TextLines.from_strings(_lines(rs, 400, ["violet", "red"])).with_key(("part", 0))
    mask = rs.random(len(new)) < 0.2
    mask[0] = True                      # the first line's colour appears first only in test
    train = LineSelection(new, np.flatnonzero(~mask))
    test = LineSelection(new, np.flatnonzero(mask))
    both = concat_lines([train, past])
    assert isinstance(both, LineConcat) and len(both) == len(train) + len(past)
    hist = FeatureHistory(dev)
    got_train = parse_features(both, schema, dev, history=hist)
    got_test = parse_features(test, schema, dev)          # a one-off parser: shared parent
    want_train = parse_features(concat_lines([new.take(~mask), past]), schema, dev)
    want_test = parse_features(new.take(mask), schema, dev)
    for got, want in ((got_train, want_train), (got_test, want_test)):
        assert got.values == want.values
        assert torch.equal(torch.nan_to_num(got.full, -7.0), torch.nan_to_num(want.full, -7.0))
    # the whole interval's parse is what the next generation's part file adopts
    part = TextLines(np.frombuffer(bytes(new.joined()), dtype=np.uint8).copy(), len(new)) \
        .with_key(("part", 1))
    parse_features(concat_lines([part, past]), schema, dev, history=hist)
    assert hist.stats["adopted"] == 1
    assert bytes(train.joined()) == bytes(new.take(~mask).joined())   # bytes on demand


def test_default_split_returns_lazy_selections_cpu():
    from oryx_amd.ml.mlupdate import MLUpdate
    from oryx_amd.textlines import LineSelection
    import types
    upd = types.SimpleNamespace(test_fraction=0.25)
    tl = TextLines.from_strings(["%d" % i for i in range(1000)])
    train, test = MLUpdate.split_new_data_to_train_test(upd, tl)
    assert isinstance(train, LineSelection) and isinstance(test, LineSelection)
    assert len(train) + len(test) == 1000
    assert sorted(int(x) for x in list(train) + list(test)) == list(range(1000))


@pytest.mark.gpu
def test_staged_h2d_copy_bitwise(cuda):
    """The pinned, natively staged host -> device copy of the parser's text (several 64 MB
    pieces and a partial last one, from an offset) equals the source bytes."""
    from oryx_amd.models.features import h2d
    rs = np.random.default_rng(2)
    n = (200 << 20) + 12345
    buf = rs.integers(0, 256, size=n + 77, dtype=np.uint8)
    dst = torch.empty(n + 32, dtype=torch.uint8, device=cuda)
    h2d(buf, 77, n, dst, staged=True)
    torch.cuda.synchronize()
    assert torch.equal(dst[:n].cpu(), torch.from_numpy(buf[77:77 + n]))


def test_native_span_encoding_first_appearance_order_cpu():
    """oryx_encode_spans (per-thread tables merged in row order) numbers values in their
    order of first appearance over all rows, empty spans missing -- as one sequential pass."""
    from oryx_amd.models.features import _encode_spans
    rs = np.random.default_rng(4)
    n = 300_000                                   # several thread ranges
    words = ["v%d" % i for i in range(5000)]
    pick = np.minimum(rs.zipf(1.3, size=n) - 1, len(words) - 1)
    vals = [words[i] if rs.random() > 0.05 else "" for i in pick]
    text = ",".join(vals).encode()
    offs, lens, at = [], [], 0
    for v in vals:
        offs.append(at)
        lens.append(len(v))
        at += len(v) + 1
    seg = np.frombuffer(text, dtype=np.uint8)
    so = np.array(offs, dtype=np.int64)[:, None]
    sl = np.array(lens, dtype=np.int32)[:, None]
    values, codes = _encode_spans(seg, so, sl, [0], np.float64)
    want_vals, want_codes = {}, []
    for v in vals:
        want_codes.append(np.nan if v == "" else want_vals.setdefault(v, len(want_vals)))
    assert values[0] == list(want_vals)
    assert np.array_equal(np.nan_to_num(codes[0], nan=-1.0),
                          np.nan_to_num(np.array(want_codes, dtype=np.float64), nan=-1.0))


def test_interval_saved_as_several_part_files_is_adopted_cpu(monkeypatch, tmp_path):
    """A large interval is saved as several part files (textlines.part_edges; the batch
    layer writes them concurrently); the next generation adopts each of them from the
    interval's parse -- no re-parse -- with the rows and categorical encodings a parse of the
    files gives."""
    from oryx_amd import textlines
    from oryx_amd.api import Dataset
    from oryx_amd.layers.batch import read_past_data, save_interval_data
    from oryx_amd.textlines import LineSelection
    monkeypatch.setattr(FeatureHistory, "UNKEYED_MIN_BYTES", 1)
    monkeypatch.setattr(textlines, "PART_FILE_BYTES", 4000)
    monkeypatch.setattr(textlines, "SPLIT_MIN_BYTES", 4000)
    rs = np.random.default_rng(9)
    schema = _schema()
    new = TextLines.from_strings(_lines(rs, 1500, ["red", "green", "blue", "", "cyan"]))
    dev = torch.device("cpu")
    hist = FeatureHistory(dev)
    mask = rs.random(len(new)) < 0.1
    parse_features(LineSelection(new, np.flatnonzero(~mask)), schema, dev, history=hist)
    data_dir = "file:" + str(tmp_path / "data") + "/"
    save_interval_data(data_dir, 77, Dataset.from_values(new), split=True)
    past = read_past_data(data_dir).values()
    assert len(past.segment_list()) > 4            # several part files
    assert sorted(past) == sorted(new)
    before = hist.stats["parsed_bytes"]
    got = parse_features(past, schema, dev, history=hist)
    assert hist.stats["parsed_bytes"] == before    # every part file adopted
    assert hist.stats["adopted"] == len(past.segment_list())
    want = parse_features(TextLines(np.frombuffer(bytes(past.joined()), dtype=np.uint8).copy()),
                          schema, dev)
    assert got.values == want.values
    assert torch.equal(torch.nan_to_num(got.full, -7.0), torch.nan_to_num(want.full, -7.0))
    # and once cached under their keys, the part files are hits
    parse_features(past, schema, dev, history=hist)
    assert hist.stats["hits"] == len(past.segment_list())
