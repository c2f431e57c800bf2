"""oryx_topn_prep (csrc/runtime/oryx_ingest.cpp): the native packing of a top-N batch's
launch inputs -- query rows, the union of the LSH buckets as merged store-position ranges
with their 16-row tile prefix, per-query bucket bitmaps, sorted excluded positions -- against
a numpy reference of the same layout (CPU; the GPU tests check the scans it feeds)."""

import ctypes

import numpy as np

from oryx_amd import native

MAX_BATCH = 16


def _reference(targets, kp, cands, excl, nb, bucket_start, n, pos, nd=0):
    nq, k = targets.shape
    words = (nb + 31) // 32
    Q = np.zeros((MAX_BATCH, kp), np.float32)
    Q[:nq, :k] = targets
    bits = None
    if any(c is not None for c in cands):
        mask = np.zeros((nq, words * 32), bool)
        for j, c in enumerate(cands):
            if c is None:
                mask[j, :nb] = True
            else:
                mask[j, c] = True
        bits = np.packbits(mask, axis=1, bitorder="little").view(np.uint32)
        sel = np.nonzero(mask[:, :nb].any(0))[0]
        st, en = bucket_start[sel], bucket_start[sel + 1]
        keep = en > st
        st, en = st[keep], en[keep]
        if len(st):
            brk = np.nonzero(st[1:] != en[:-1])[0] + 1
            rs = np.stack([st[np.r_[0, brk]], en[np.r_[brk - 1, len(en) - 1]]], 1)
        else:
            rs = np.zeros((0, 2), np.int64)
    else:
        rs = np.array([[0, n]], np.int64) if n > 0 else np.zeros((0, 2), np.int64)
    if nd:                          # the delta segment [n, n + nd), scanned by every query
        if len(rs) and rs[-1, 1] == n:
            rs = rs.copy()
            rs[-1, 1] = n + nd
        else:
            rs = np.concatenate([rs, np.array([[n, n + nd]], np.int64)])
    if not len(rs):
        return None
    tiles = (rs[:, 1] - rs[:, 0] + 15) // 16
    t0 = np.zeros(len(rs) + 1, np.int64)
    np.cumsum(tiles, out=t0[1:])
    ptr = ex = None
    if any(e is not None and len(e) for e in excl):
        ptr = np.zeros(nq + 1, np.int32)
        chunks = []
        for j, e in enumerate(excl):
            e = np.asarray(e if e is not None else [], np.int64)
            e = e[(e >= 0) & (e < len(pos))]
            p = np.sort(pos[e])
            p = p[p >= 0].astype(np.int32)
            chunks.append(p)
            ptr[j + 1] = ptr[j] + len(p)
        ex = np.concatenate(chunks) if ptr[-1] else np.zeros(1, np.int32)
    return Q, rs, t0, bits, ptr, ex


def test_topn_prep_matches_numpy_packing():
    lib = native.runtime()
    vp = ctypes.c_void_p
    rng = np.random.default_rng(3)
    checked = 0
    for _ in range(300):
        k = int(rng.integers(1, 60))
        kp = (k + 15) // 16 * 16
        nb = int(rng.choice([1, 7, 32, 33, 100, 1024]))
        counts = rng.integers(0, 20, nb)
        counts[rng.random(nb) < 0.3] = 0
        bucket_start = np.zeros(nb + 1, np.int64)
        np.cumsum(counts, out=bucket_start[1:])
        n = int(bucket_start[-1])
        nd = int(rng.integers(0, 40)) if rng.random() < 0.5 else 0
        nrows = n + nd + int(rng.integers(0, 50))
        pos = np.full(nrows, -1, np.int64)
        pos[rng.permutation(nrows)[:n + nd]] = np.arange(n + nd)
        nq = int(rng.integers(1, 9))
        lsh = rng.random() < 0.7
        cands = [np.unique(rng.integers(0, nb, int(rng.integers(0, min(nb, 20) + 1))))
                 if lsh and rng.random() < 0.8 else None for _ in range(nq)]
        if not lsh:
            cands = [None] * nq
        excl = [rng.integers(-2, nrows + 3, int(rng.integers(0, 30))).tolist()
                if rng.random() < 0.6 else None for _ in range(nq)]
        targets = rng.standard_normal((nq, k)).astype(np.float32)
        ref = _reference(targets, kp, cands, excl, nb, bucket_start, n, pos, nd)
        cp = ca = c = None
        if any(x is not None for x in cands):
            cl = [x if x is not None else np.zeros(0, np.int64) for x in cands]
            cp = np.zeros(nq + 1, np.int64)
            np.cumsum([len(x) for x in cl], out=cp[1:])
            c = np.concatenate(cl) if cp[-1] else np.zeros(1, np.int64)
            ca = np.array([x is None for x in cands], np.uint8)
        ep = er = None
        if any(e is not None and len(e) for e in excl):
            el = [e if e is not None else [] for e in excl]
            ep = np.zeros(nq + 1, np.int64)
            np.cumsum([len(e) for e in el], out=ep[1:])
            er = np.array([v for e in el for v in e], np.int64)
        out = np.zeros(1 << 20, np.uint8)
        info = np.zeros(9, np.int64)
        rc = lib.oryx_topn_prep(nq, k, kp, MAX_BATCH, targets.ctypes.data_as(vp),
                                cp.ctypes.data_as(vp) if cp is not None else None,
                                c.ctypes.data_as(vp) if c is not None else None,
                                ca.ctypes.data_as(vp) if ca is not None else None, nb,
                                (nb + 31) // 32, bucket_start.ctypes.data_as(vp), n,
                                ep.ctypes.data_as(vp) if ep is not None else None,
                                er.ctypes.data_as(vp) if er is not None else None,
                                pos.ctypes.data_as(vp), len(pos), n, n + nd,
                                out.ctypes.data_as(vp), len(out), info.ctypes.data_as(vp))
        if ref is None:
            assert rc == 1
            continue
        assert rc == 0
        Q, rs, t0, bits, ptr, ex = ref
        nr, nt, o_rs, o_t0, o_bits, o_ptr, o_ex, used, n_ex = (int(v) for v in info)
        assert nr == len(rs) and nt == int(t0[-1])
        assert np.array_equal(out[:Q.nbytes].view(np.float32).reshape(Q.shape), Q)
        assert np.array_equal(out[o_rs:o_rs + rs.nbytes].view(np.int64).reshape(-1, 2), rs)
        assert np.array_equal(out[o_t0:o_t0 + t0.nbytes].view(np.int64), t0)
        assert (o_bits >= 0) == (bits is not None) and (o_ptr >= 0) == (ptr is not None)
        if bits is not None:
            assert np.array_equal(out[o_bits:o_bits + bits.nbytes].view(np.uint32).reshape(
                bits.shape), bits)
        if ptr is not None:
            assert np.array_equal(out[o_ptr:o_ptr + ptr.nbytes].view(np.int32), ptr)
            assert n_ex == len(ex)
            assert np.array_equal(out[o_ex:o_ex + ex.nbytes].view(np.int32), ex)
        assert used <= len(out) and all(o % 16 == 0 for o in (o_rs, o_t0) if o >= 0)
        checked += 1
    assert checked > 200
