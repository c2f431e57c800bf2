"""Generic clustering endpoints: ``/assign`` and ``/add``.

Equivalent of ``[serving-app]/clustering/Assign.java`` and ``Add.java`` behind the
``ClusteringServingModel.nearestClusterID(String[])`` interface
(``[serving-app]/clustering/model/ClusteringServingModel.java:23-31``).  A model may also offer
``nearest_cluster_ids(list of token lists)`` so a multi-line POST is assigned in one batched
device pass instead of line by line.
"""

from __future__ import annotations

from typing import List

from ..api import OryxServingException
from ..utils import text
from .http import route
from .resources import check, check_not_read_only, get_serving_model, input_lines, send_input

__all__ = []

_PRODUCES = ("text/plain", "text/csv", "application/json")


def _tokens(datum: str) -> List[str]:
    check(datum is not None and datum != "", "Data is needed to cluster")
    return text.parse_delimited(datum, ",")


def _nearest(model, tokens) -> str:
    try:
        return str(int(model.nearest_cluster_id(tokens)))
    except ValueError as e:
        raise OryxServingException(400, str(e))


@route("GET", "/assign/{datum}", produces=_PRODUCES)
def assign_get(req, datum):
    return _nearest(get_serving_model(req), _tokens(datum))


@route("POST", "/assign", produces=_PRODUCES)
def assign_post(req):
    model = get_serving_model(req)
    toks = [_tokens(line) for line in input_lines(req)]
    batch = getattr(model, "nearest_cluster_ids", None)
    if batch is not None and len(toks) > 1:
        try:
            return [str(int(i)) for i in batch(toks)]
        except ValueError as e:
            raise OryxServingException(400, str(e))
    return [_nearest(model, t) for t in toks]


@route("POST", "/add")
def add_post(req):
    check_not_read_only(req)
    for line in input_lines(req):
        send_input(req, line)


@route("POST", "/add/{datum}")
def add_post_datum(req, datum):
    check_not_read_only(req)
    send_input(req, datum)
