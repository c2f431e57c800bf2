"""Shared serving resources and helpers (the reference's ``[serving-app]`` base classes).

* :class:`IDValue`, :class:`IDCount` (``[serving-app]/IDEntity.java:25-49``, ``IDValue.java``,
  ``IDCount.java``): CSV ``id,value`` / JSON ``{"id":..,"value":..}``;
* helpers of ``AbstractOryxResource`` (``[serving-app]/AbstractOryxResource.java:54-182``):
  :func:`send_input` (key = Java ``hashCode`` hex of the message), :func:`get_serving_model`
  (503 until ``fraction_loaded >= min-model-load-fraction``, then latched), :func:`check`
  (400), :func:`check_exists` (404), :func:`check_not_read_only` (403),
  :func:`maybe_decompress` for gzip/zip multipart parts;
* ``GET|HEAD /ready`` (``[serving-app]/Ready.java:32-46``), ``/error``, ``/metrics``.
"""

from __future__ import annotations

import gzip
import io
import logging
import os
import zipfile
from typing import Iterable, Iterator, List, Optional

from ..api import OryxServingException
from ..utils.text import java_double_str
from .http import Response, route

log = logging.getLogger(__name__)

__all__ = ["IDValue", "IDCount", "send_input", "get_serving_model", "check", "check_exists",
           "check_not_read_only", "maybe_decompress", "java_string_hash", "input_lines",
           "MODEL_MANAGER_KEY", "INPUT_PRODUCER_KEY"]

MODEL_MANAGER_KEY = "com.cloudera.oryx.lambda.serving.ModelManagerListener.ModelManager"
INPUT_PRODUCER_KEY = "com.cloudera.oryx.lambda.serving.ModelManagerListener.InputProducer"


class IDValue:
    __slots__ = ("id", "value")

    def __init__(self, id_: str, value: float):
        self.id = id_
        self.value = float(value)

    def to_csv(self) -> str:
        return "%s,%s" % (self.id, java_double_str(self.value))

    def to_json(self):
        return {"id": self.id, "value": self.value}

    def __repr__(self):
        return "%s:%s" % (self.id, self.value)

    def __eq__(self, other):
        return isinstance(other, IDValue) and self.id == other.id and self.value == other.value


class IDCount:
    __slots__ = ("id", "count")

    def __init__(self, id_: str, count: int):
        self.id = id_
        self.count = int(count)

    def to_csv(self) -> str:
        return "%s,%d" % (self.id, self.count)

    def to_json(self):
        return {"id": self.id, "count": self.count}

    def __repr__(self):
        return "%s:%d" % (self.id, self.count)


def java_string_hash(s: str) -> int:
    """``String.hashCode`` (UTF-16 code units, 32-bit wrap)."""
    h = 0
    for ch in s.encode("utf-16-be").decode("utf-16-be"):
        code = ord(ch)
        if code > 0xFFFF:  # surrogate pair
            code -= 0x10000
            for unit in (0xD800 + (code >> 10), 0xDC00 + (code & 0x3FF)):
                h = (31 * h + unit) & 0xFFFFFFFF
        else:
            h = (31 * h + code) & 0xFFFFFFFF
    return h


def send_input(req, message: str) -> None:
    producer = req.context.get(INPUT_PRODUCER_KEY)
    if producer is None:
        raise OryxServingException(503, "No input producer available")
    producer.send("%x" % java_string_hash(message), message)


def model_manager(req):
    mgr = req.context.get(MODEL_MANAGER_KEY)
    if mgr is None:
        raise OryxServingException(503, "No model manager")
    return mgr


def get_serving_model(req):
    mgr = model_manager(req)
    model = mgr.get_model()
    state = req.context.setdefault("_load_state", {"loaded": False})
    if state["loaded"]:
        return model
    if model is not None:
        min_frac = mgr.get_config().get_double("oryx.serving.min-model-load-fraction")
        if not (0.0 <= min_frac <= 1.0):
            raise ValueError("bad min-model-load-fraction")
        frac = model.get_fraction_loaded()
        log.info("Model loaded fraction: %s", frac)
        if frac >= min_frac:
            state["loaded"] = True
            return model
    raise OryxServingException(503)


def is_read_only(req) -> bool:
    return model_manager(req).is_read_only()


def check(condition: bool, message: str = "", status: int = 400) -> None:
    if not condition:
        raise OryxServingException(status, message)


def check_exists(condition: bool, entity: str) -> None:
    check(condition, entity, 404)


def check_not_read_only(req) -> None:
    check(not is_read_only(req), "Serving Layer is read-only", 403)


def maybe_decompress(part) -> bytes:
    data = part.data
    ctype = (part.content_type or "").lower()
    if ctype == "application/zip":
        with zipfile.ZipFile(io.BytesIO(data)) as zf:
            return b"".join(zf.read(n) for n in zf.namelist())
    if ctype in ("application/gzip", "application/x-gzip"):
        return gzip.decompress(data)
    return data


def input_lines(req) -> Iterator[str]:
    """Lines of the request body, or of every (decompressed) multipart part."""
    if req.is_multipart():
        parts = req.multipart_parts()
        check(bool(parts), "No parts")
        for part in parts:
            for line in maybe_decompress(part).decode("utf-8").splitlines():
                yield line
    else:
        for line in req.text().splitlines():
            yield line


# ---------------------------------------------------------------- shared endpoints

def _ready(req):
    try:
        get_serving_model(req)
    except OryxServingException:
        return Response(503, b"", None)
    return Response(200, b"", None)


route("GET", "/ready")(_ready)
route("HEAD", "/ready")(_ready)


@route("GET", "/error", produces=("text/html", "text/plain"))
def error_page(req):
    code = int(req.q("code", "500"))
    raise OryxServingException(code, req.q("message", ""))


@route("GET", "/metrics", produces=("text/plain",))
def metrics(req):
    reg = req.context.get("metrics")
    if reg is None:
        return ""
    mgr = req.context.get(MODEL_MANAGER_KEY)
    model = mgr.get_model() if mgr is not None else None
    if model is not None:
        reg.set_gauge("oryx_model_fraction_loaded", model.get_fraction_loaded())
    return reg.render()


def console_page(title: str, body_fragment: str) -> Response:
    here = os.path.dirname(__file__)
    with open(os.path.join(here, "console", "header.html.fragment"), encoding="utf-8") as f:
        header = f.read()
    with open(os.path.join(here, "console", "footer.html.fragment"), encoding="utf-8") as f:
        footer = f.read()
    html = header.replace("{{TITLE}}", title) + body_fragment + footer
    return Response(200, html.encode("utf-8"), "text/html")
