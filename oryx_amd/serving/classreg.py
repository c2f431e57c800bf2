"""Generic classification/regression endpoints: ``/predict`` and ``/train``.

Equivalent of ``[serving-app]/classreg/Predict.java`` and ``Train.java`` behind the
``ClassificationRegressionServingModel.predict(String[])`` interface
(``[serving-app]/classreg/model/ClassificationRegressionServingModel.java:24-32``).
"""

from __future__ import annotations

from ..api import OryxServingException
from ..utils import text
from .http import route
from .resources import check, check_not_read_only, get_serving_model, input_lines, send_input

__all__ = []

_PRODUCES = ("text/plain", "text/csv", "application/json")


def _predict(model, datum: str) -> str:
    check(datum is not None and datum != "", "Missing input data")
    try:
        return model.predict(text.parse_delimited(datum, ","))
    except (ValueError, KeyError) as e:
        raise OryxServingException(400, str(e))


@route("GET", "/predict/{datum}", produces=_PRODUCES)
def predict_get(req, datum):
    return _predict(get_serving_model(req), datum)


@route("POST", "/predict", produces=_PRODUCES)
def predict_post(req):
    model = get_serving_model(req)
    return [_predict(model, line) for line in input_lines(req)]


@route("POST", "/train")
def train_post(req):
    check_not_read_only(req)
    for line in input_lines(req):
        send_input(req, line)


@route("POST", "/train/{datum}")
def train_post_datum(req, datum):
    check_not_read_only(req)
    send_input(req, datum)
