"""Example app endpoints: ``/add`` (POST line / body) and ``/distinct`` (GET all / one word)
(``[example]/serving/Add.java``, ``Distinct.java``).  Input is sent with a null key."""

from __future__ import annotations

from ...api import OryxServingException
from ...serving.http import route
from ...serving.resources import INPUT_PRODUCER_KEY, model_manager

__all__ = []


def _producer(req):
    p = req.context.get(INPUT_PRODUCER_KEY)
    if p is None:
        raise OryxServingException(503, "No input producer available")
    return p


@route("POST", "/add/{line}")
def add_line(req, line):
    _producer(req).send(None, line)


@route("POST", "/add")
def add_body(req):
    prod = _producer(req)
    for line in req.text().splitlines():
        prod.send(None, line)


@route("GET", "/distinct", produces=("text/plain", "application/json"))
def distinct_all(req):
    return dict(model_manager(req).get_model().get_words())


@route("GET", "/distinct/{word}", produces=("text/plain", "application/json"))
def distinct_word(req, word):
    count = model_manager(req).get_model().get_words().get(word)
    if count is None:
        raise OryxServingException(400, "No such word")
    return count
