"""In-process serving test harness (the reference's JerseyTest-based AbstractServingTest):
dispatches requests straight into the router with a mock model manager and MockTopicProducer."""

import json
import urllib.parse

from oryx_amd.api import AbstractServingModelManager
from oryx_amd.serving import http
from oryx_amd.serving.layer import resource_modules
from oryx_amd.serving.resources import INPUT_PRODUCER_KEY, MODEL_MANAGER_KEY
from oryx_amd.transport.producer import MockTopicProducer
from oryx_amd.utils import config as cfg


class MockManager(AbstractServingModelManager):
    def __init__(self, config, model):
        super().__init__(config)
        self.model = model

    def consume(self, updates, context=None):
        for _ in updates:
            pass

    def get_model(self):
        return self.model


class Client:
    def __init__(self, modules, model, overlay=None, read_only=False):
        overlay = dict(overlay or {})
        overlay["oryx.serving.api.read-only"] = "true" if read_only else "false"
        self.config = cfg.overlay_on(overlay, cfg.get_default())
        self.manager = MockManager(self.config, model)
        MockTopicProducer.clear()
        self.context = {MODEL_MANAGER_KEY: self.manager, INPUT_PRODUCER_KEY: MockTopicProducer(),
                        "config": self.config}
        mods = ["oryx_amd.serving.resources"] + list(modules)
        self.router = http.Router(http.collect_routes(mods), "/")

    def request(self, method, path, accept=None, body=b"", headers=None, **query):
        hdrs = {k.lower(): v for k, v in (headers or {}).items()}
        if accept:
            hdrs["accept"] = accept
        parsed = urllib.parse.urlsplit(path)
        q = urllib.parse.parse_qs(parsed.query, keep_blank_values=True)
        for k, v in query.items():
            q[k] = v if isinstance(v, list) else [str(v)]
        if isinstance(body, str):
            body = body.encode("utf-8")
        req = http.Request(method, parsed.path if parsed.path.startswith("/") else "/" + parsed.path,
                           q, hdrs, body, self.context)
        return self.router.dispatch(req)

    def get(self, path, accept=None, **query):
        return self.request("GET", path, accept=accept, **query)

    def get_json(self, path, **query):
        r = self.get(path, accept="application/json", **query)
        assert r.status == 200, (r.status, r.body)
        return json.loads(r.body.decode("utf-8")) if r.body else None

    def get_text(self, path, **query):
        r = self.get(path, **query)
        assert r.status == 200, (r.status, r.body)
        return r.body.decode("utf-8")

    def status(self, method, path, **kw):
        return self.request(method, path, **kw).status
