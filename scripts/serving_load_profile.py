#!/usr/bin/env python3
"""Profile of the serving model load from the update topic (single thread: the manager's
consume over an UpdateIterator, cProfile by own time).  Args: items users features."""
import sys, os, time, json, cProfile, pstats, tempfile, shutil
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench_serving as b
from oryx_amd import ingest
from oryx_amd.transport import log as tlog
from oryx_amd.utils import config as cfg, pmml as pmmlu
from oryx_amd.serving.layer import UpdateIterator
from oryx_amd.models.als.serving import ALSServingModelManager
items, users, features = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
Y, X, item_ids, user_ids, counts, known = b.make_data(items, users, features, 7)
work = tempfile.mkdtemp(dir=os.environ.get("ORYX_TTR_DIR", "/dev/shm")); root = work + "/log"
tlog.maybe_create_topic(root, "OryxUpdate", 1, max_message=1 << 30)
topic = tlog.Topic(root, "OryxUpdate")
doc = pmmlu.build_skeleton_pmml()
for k_, v_ in (("X","X/"),("Y","Y/"),("features",features),("lambda",0.001),("implicit",True),("alpha",1.0)): doc.add_extension(k_, v_)
doc.add_extension_content("XIDs", user_ids); doc.add_extension_content("YIDs", item_ids)
topic.append_batch([("MODEL", pmmlu.to_string(doc))])
chunk = 1 << 20
for lo in range(0, items, chunk):
    hi = min(items, lo + chunk)
    topic.append_block(ingest.assemble_row_messages("Y", item_ids[lo:hi], ingest.format_float_rows_blob(Y[lo:hi])), key="UP")
pos = np.r_[0, np.cumsum(counts)]
names = ingest.IdDict(); names.encode(item_ids)
for lo in range(0, users, chunk):
    hi = min(users, lo + chunk)
    uu = np.repeat(np.arange(hi - lo), counts[lo:hi])
    kt = ingest.known_items_text(names, uu, known[pos[lo]:pos[hi]], hi - lo)
    topic.append_block(ingest.assemble_row_messages("X", user_ids[lo:hi], ingest.format_float_rows_blob(X[lo:hi]), kt, np.arange(hi - lo)), key="UP")
topic.close()
conf = cfg.overlay_on({"oryx.serving.api.read-only": "true"}, cfg.get_default())
mgr = ALSServingModelManager(conf)
t = tlog.Topic(root, "OryxUpdate")
cons = tlog.TopicConsumer(t, start="earliest")
it = UpdateIterator(cons, poll_ms=0)
class Limited:
    def __init__(s, it): s.it = it
    def __iter__(s): return s
    def __next__(s):
        if not s.it._pending and all(r.position >= t.end_offset(r.partition) for r in cons.readers): raise StopIteration
        return next(s.it)
    def __getattr__(s, a): return getattr(s.it, a)
pr = cProfile.Profile(); t0 = time.perf_counter(); pr.enable()
mgr.consume(Limited(it))
pr.disable(); el = time.perf_counter() - t0
m = mgr.get_model()
print("rows", m.get_num_items(), m.get_num_users(), "s", el, "rows/s", (items+users)/el)
pstats.Stats(pr).sort_stats('tottime').print_stats(18)
shutil.rmtree(work)
