"""Example configurations: this repo's conf/*.conf and -- when the reference checkout is
present -- the reference's own app/conf/*.conf (read as text by the HOCON parser; SURVEY.md
section 5.6 keeps the key names so those files stay valid).  Every configured batch update,
speed manager and serving manager class loads (Java names through the alias table) and the
serving resource modules resolve to route tables."""

import glob
import importlib
import os

import pytest

from oryx_amd.serving import http
from oryx_amd.serving.layer import resource_modules
from oryx_amd.utils import config as cfg
from oryx_amd.utils import lang

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OURS = sorted(glob.glob(os.path.join(ROOT, "conf", "*.conf")))
THEIRS = sorted(glob.glob("/root/reference/app/conf/*.conf"))


def _check(path):
    conf = cfg.load_file(path)
    for key in ("oryx.batch.update-class", "oryx.speed.model-manager-class",
                "oryx.serving.model-manager-class"):
        name = cfg.get_optional_string(conf, key)
        assert name, key
        assert lang.load_class(name) is not None
    mods = resource_modules(conf)
    assert len(mods) >= 2
    routes = http.collect_routes(mods)
    assert any(r.template == "/ready" for r in routes)
    return conf


@pytest.mark.parametrize("path", OURS, ids=[os.path.basename(p) for p in OURS])
def test_our_example_confs(path):
    conf = _check(path)
    assert conf.get_string("oryx.input-topic.broker").startswith("log:")
    assert conf.get_string("oryx.batch.storage.model-dir").startswith("file://")


@pytest.mark.skipif(not THEIRS, reason="reference checkout not present")
@pytest.mark.parametrize("path", THEIRS, ids=[os.path.basename(p) for p in THEIRS])
def test_reference_example_confs_stay_valid(path):
    conf = _check(path)
    # Kafka / ZooKeeper / HDFS locations parse (they are only used for naming here)
    assert conf.get_string("oryx.input-topic.broker")
    assert conf.get_int("oryx.batch.streaming.generation-interval-sec") > 0
