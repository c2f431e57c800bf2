"""Example (word co-occurrence) app: batch/speed/serving semantics of
[example]/batch/ExampleBatchLayerUpdate.java, speed/ExampleSpeedModelManager.java and
serving/{Add,Distinct}.java."""

import json

from oryx_amd.api import Dataset, KeyMessage
from oryx_amd.models.example.batch import ExampleBatchLayerUpdate, count_distinct_other_words
from oryx_amd.models.example.serving import ExampleServingModelManager
from oryx_amd.models.example.speed import ExampleSpeedModelManager
from oryx_amd.transport.producer import MockTopicProducer
from oryx_amd.utils import config as cfg

from .serving_harness import Client


def test_count_distinct_other_words():
    got = count_distinct_other_words(["a b c", "a b", "b d", "e"])
    assert got == {"a": 2, "b": 3, "c": 2, "d": 1}


def test_batch_publishes_model():
    MockTopicProducer.clear()
    ExampleBatchLayerUpdate().run_update(None, 1, Dataset([(None, "a b")]),
                                         Dataset([(None, "b c")]), "/tmp", MockTopicProducer())
    (k, m), = MockTopicProducer.get_key_messages()
    assert k == "MODEL" and json.loads(m) == {"a": 1, "b": 2, "c": 1}


def test_speed_updates():
    mgr = ExampleSpeedModelManager()
    mgr.consume(iter([KeyMessage("MODEL", '{"a":1,"b":2}'), KeyMessage("UP", "x,1")]))
    ups = sorted(mgr.build_updates(Dataset([(None, "a c")])))
    assert ups == ["a,2", "c,1"]


def test_serving_endpoints():
    mgr = ExampleServingModelManager(cfg.get_default())
    mgr.consume(iter([KeyMessage("MODEL", '{"a":1,"b":2}'), KeyMessage("UP", "c,5")]))
    c = Client(["oryx_amd.models.example.resources"], mgr.get_model())
    assert c.get_json("/distinct") == {"a": 1, "b": 2, "c": 5}
    assert c.get_text("/distinct/c").strip() == "5"
    assert c.status("GET", "/distinct/zzz") == 400
    assert c.status("POST", "/add/hello world") == 204
    assert c.status("POST", "/add", body="x y\nz w") == 204
    assert [m for _, m in MockTopicProducer.get_key_messages()] == ["hello world", "x y", "z w"]
    assert [k for k, _ in MockTopicProducer.get_key_messages()] == [None, None, None]
