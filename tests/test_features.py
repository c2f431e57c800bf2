"""Feature-row parsing of the k-means / RDF batch layers (models/features.py): a buffer made of
several segments (the new interval followed by past part files, as a later generation sees it)
parses to the same rows and categorical encodings as one parse of the concatenated text, with
and without the resident history.  Regression: categorical fields of every segment after the
first were read at the wrong byte offsets (values such as "," became categories)."""

import numpy as np
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
