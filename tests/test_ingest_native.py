"""ingest.IdDict's cached key list under concurrency (the serving model's known-items
dictionary is read by every handler thread): concurrent key_list calls while the dictionary
grows return the keys in code order, build the cache once (no duplicated segments), and after
that hand back the cached list itself (no per-request copy of a million keys)."""

import threading

from oryx_amd import ingest


def test_key_list_concurrent_growth_cpu():
    d = ingest.IdDict()
    d.encode(["k%d" % i for i in range(50_000)])
    errs = []
    stop = threading.Event()

    def reader():
        try:
            while not stop.is_set():
                keys = d.key_list()
                n = len(keys)
                for j in (0, n // 2, n - 1):
                    if keys[j] != "k%d" % j:
                        errs.append((j, keys[j]))
                        return
        except Exception as e:   # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=reader) for _ in range(8)]
    for t in ts:
        t.start()
    for lo in range(50_000, 150_000, 5_000):
        d.encode(["k%d" % i for i in range(lo, lo + 5_000)])
    stop.set()
    for t in ts:
        t.join(30)
    assert not errs, errs[:3]
    keys = d.key_list()
    assert len(keys) == 150_000 and keys[-1] == "k149999"
    again = d.key_list()
    assert again.base is keys.base             # cached: views of one array, no copy
    assert d._keys_cache[1] == len(d)          # no duplicated segments
    assert list(d._keys_cache[0][:len(d)]) == ["k%d" % i for i in range(150_000)]
    import gc
    assert not gc.is_tracked(d._keys_cache[0])  # invisible to the cyclic GC
