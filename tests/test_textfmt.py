"""Factor-row text codecs: the host shortest-float formatter / parser (csrc/runtime/
fastfloat.h) against std::to_chars / std::from_chars, the Python RowText helpers, and the GPU
formatter (csrc/kernels/textfmt.hip) byte-for-byte against the host one."""

import json
import os
import shutil
import subprocess

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _special_matrix(rows=300, k=67, seed=0):
    g = np.random.default_rng(seed)
    x = g.normal(size=(rows, k)).astype(np.float32)
    x[1] = g.normal(scale=1e4, size=k)
    x[2] = g.normal(scale=1e-6, size=k)
    bits = g.integers(0, 2 ** 32, size=k, dtype=np.uint64).astype(np.uint32)
    x[3] = bits.view(np.float32)
    sp = [0.0, -0.0, 1.0, -1.0, 100.0, 33871888.0, 1e-7, 3.4e38, 1.4e-45, 123456.7, np.inf,
          -np.inf]
    x[4, :min(k, 12)] = sp[:min(k, 12)]
    x[5, :min(k, 3)] = [np.nan, 0.1, 1e10][:min(k, 3)]
    return x


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_fastfloat_matches_std_charconv(tmp_path):
    exe = str(tmp_path / "ffc")
    subprocess.run(["g++", "-O2", "-std=c++17", os.path.join(ROOT, "csrc", "runtime", "tests",
                                                              "fastfloat_check.cpp"), "-o", exe],
                   check=True, timeout=300)
    r = subprocess.run([exe, "99991"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr


def test_host_rows_round_trip_exactly():
    from oryx_amd import ingest
    x = _special_matrix()
    rows = ingest.format_float_rows(x)
    for j, text in enumerate(rows):
        vals = json.loads(text.replace("NaN", '"nan"').replace("-Infinity", '"-inf"')
                          .replace("Infinity", '"inf"'))
        back = np.array([float(v) for v in vals], dtype=np.float32)
        assert np.array_equal(back.view(np.uint32)[~np.isnan(back)],
                              x[j].view(np.uint32)[~np.isnan(x[j])]), text
    assert rows[4].startswith("[0.0,-0.0,1.0,-1.0,100.0,33871888.0,1e-07,3.4e+38,1e-45,")
    assert rows[5].startswith("[NaN,0.1,1e+10,")


def test_row_text_take_and_rows():
    from oryx_amd.ops import textfmt
    x = np.arange(12, dtype=np.float32).reshape(4, 3) / 4
    rt = textfmt.format_rows(x)
    assert rt.rows() == ["[0.0,0.25,0.5]", "[0.75,1.0,1.25]", "[1.5,1.75,2.0]",
                         "[2.25,2.5,2.75]"]
    sub = rt.take(np.array([2, 0]))
    assert sub.rows() == ["[1.5,1.75,2.0]", "[0.0,0.25,0.5]"]


def test_parse_up_batch_reads_formatted_rows_exactly():
    """The native UP parser (fast-path float parse) recovers the exact floats."""
    from oryx_amd import ingest
    x = _special_matrix(rows=50, k=20)
    x = np.where(np.isfinite(x), x, 1.0).astype(np.float32)
    rows = ingest.format_float_rows(x)
    msgs = ['["Y","i%d",%s]' % (j, r) for j, r in enumerate(rows)]
    kinds, ids, vecs, known = ingest.parse_up_batch(msgs, 20)
    assert (kinds == 1).all()
    assert np.array_equal(vecs.view(np.uint32), x.view(np.uint32))


@pytest.mark.gpu
def test_gpu_formatter_matches_host_bytes():
    from oryx_amd import native
    from oryx_amd.ops import textfmt
    assert native.kernels_available()
    for k in (1, 7, 64, 67, 130, 250):
        x = _special_matrix(rows=257, k=k, seed=k)
        host = textfmt.format_rows(x)
        dev = textfmt.format_rows(torch.from_numpy(x).cuda())
        assert np.array_equal(host.ends, dev.ends), k
        assert bytes(host.blob) == bytes(dev.blob), k
    # a strided view (leading dimension > k)
    big = torch.from_numpy(_special_matrix(rows=64, k=80)).cuda()
    view = big[:, :50]
    assert bytes(textfmt.format_rows(view).blob) == \
        bytes(textfmt.format_rows(view.cpu().numpy()).blob)


def test_assemble_row_messages_matches_python():
    import json
    from oryx_amd import ingest
    from oryx_amd.ops.textfmt import format_rows
    rng = np.random.default_rng(3)
    mat = rng.standard_normal((50, 7)).astype(np.float32)
    ids = ["u%d" % j for j in range(48)] + ['q"\\x\n', "\u00e9\U0001F600"]
    rows = format_rows(mat)
    r = rows.rows()
    y = ingest.assemble_row_messages("Y", ids, rows)
    assert list(y) == ['["Y",%s,%s]' % (json.dumps(a), b) for a, b in zip(ids, r)]
    lines = ingest.assemble_row_messages("", ids, rows)
    assert list(lines) == ["[%s,%s]" % (json.dumps(a), b) for a, b in zip(ids, r)]
    # known arrays by index, -1 skips the row
    from oryx_amd.ops.textfmt import RowText
    kt = ['["a"]', "[]", '["b","c"]']
    blob = "".join(kt).encode()
    known = RowText(blob, np.cumsum([len(k) for k in kt]))
    kidx = np.array([j % 4 - 1 for j in range(50)])
    x = ingest.assemble_row_messages("X", ids, rows, known, kidx)
    want = ['["X",%s,%s,%s]' % (json.dumps(a), b, kt[k]) for a, b, k in zip(ids, r, kidx)
            if k >= 0]
    assert list(x) == want


def test_known_items_text_and_gzip(tmp_path):
    import gzip
    import json
    from oryx_amd import ingest
    items = ingest.IdDict()
    items.encode(["i0", "i\u00e91", 'i"2'])
    uu = np.array([0, 0, 2, 2, 2])
    ii = np.array([1, 0, 2, 1, 0])
    kt = ingest.known_items_text(items, uu, ii, 4).rows()
    names = items.keys()
    assert kt == ["[%s,%s]" % (json.dumps(names[1]), json.dumps(names[0])), "[]",
                  "[" + ",".join(json.dumps(names[j]) for j in (2, 1, 0)) + "]", "[]"]
    # several gzip members (slices of 8 MB) read back as one stream
    data = np.random.default_rng(0).integers(32, 127, size=(20 << 20), dtype=np.uint8)
    p = str(tmp_path / "x.gz")
    ingest.write_gzip(p, data)
    with gzip.open(p, "rb") as f:
        assert f.read() == data.tobytes()
    ingest.write_gzip(p, b"")
    with gzip.open(p, "rb") as f:
        assert f.read() == b""


def test_indexed_gzip_and_feature_files_round_trip(tmp_path):
    import gzip
    import os
    from oryx_amd import ingest
    from oryx_amd.models.als.batch import read_features, write_features
    rng = np.random.default_rng(5)
    mat = rng.standard_normal((3000, 9)).astype(np.float32)
    mat[4, 2] = np.nan
    mat[5, 0] = np.inf
    ids = ["id%d" % j for j in range(3000)]
    ids[1] = 'q"é\\'
    write_features(str(tmp_path / "X"), ids, mat)
    raw = open(tmp_path / "X" / "part-00000.gz", "rb").read()
    # the indexed members are a plain gzip stream to other readers, and inflate natively
    assert bytes(ingest.read_gzip(raw)) == gzip.decompress(raw)
    got_ids, got = read_features(str(tmp_path / "X"))
    assert got_ids == ids
    assert np.array_equal(got, mat, equal_nan=True)
    # a part written by another gzip writer, with a bare-number id: the general paths
    os.makedirs(tmp_path / "Y")
    with gzip.open(tmp_path / "Y" / "part-00000.gz", "wt") as f:
        f.write('[7,[1.5,-2]]\n\n["b",[3,4e-3]]\n')
    assert read_features(str(tmp_path / "Y"))[0] == ["7", "b"]
    assert np.allclose(read_features(str(tmp_path / "Y"))[1], [[1.5, -2], [3, 4e-3]])
    # a damaged member is reported, not returned
    bad = bytearray(raw)
    bad[len(bad) // 2] ^= 0x55
    with pytest.raises(Exception):
        ingest.read_gzip(bytes(bad))
