"""RDF REST endpoints: ``/classificationDistribution``, ``/feature/importance`` and the
console; ``/predict`` and ``/train`` come from :mod:`oryx_amd.serving.classreg`
(``[serving-app]/rdf/ClassificationDistribution.java``, ``FeatureImportance.java``)."""

from __future__ import annotations

import os

from ...api import OryxServingException
from ...serving.http import route
from ...serving.resources import IDValue, check, console_page, get_serving_model
from ...utils import text

INCLUDE_RESOURCES = ["oryx_amd.serving.classreg"]

__all__ = []

_PRODUCES = ("text/plain", "text/csv", "application/json")


@route("GET", "/classificationDistribution/{datum}", produces=_PRODUCES)
def classification_distribution(req, datum):
    check(datum is not None and datum != "", "Missing input data")
    model = get_serving_model(req)
    schema = model.get_input_schema()
    check(schema.is_classification(), "Only applicable for classification")
    try:
        prediction = model.make_prediction(text.parse_delimited(datum, ","))
    except (ValueError, KeyError) as e:
        raise OryxServingException(400, str(e))
    probs = prediction.get_category_probabilities()
    names = model.get_encodings().get_encoding_value_map(schema.get_target_feature_index())
    return [IDValue(names[i], float(p)) for i, p in enumerate(probs)]


@route("GET", "/feature/importance", produces=_PRODUCES)
def all_importances(req):
    imp = get_serving_model(req).get_forest().get_feature_importances()
    return [float(v) for v in (imp if imp is not None else [])]


@route("GET", "/feature/importance/{featureNumber}", produces=_PRODUCES)
def importance(req, featureNumber):
    try:
        fnum = int(featureNumber)
    except ValueError:
        raise OryxServingException(404, "Bad feature number")
    imp = get_serving_model(req).get_forest().get_feature_importances()
    check(imp is not None and 0 <= fnum < len(imp), "Bad feature number")
    return float(imp[fnum])


@route("GET", "/", produces=("text/html",))
def console(req):
    here = os.path.dirname(os.path.dirname(os.path.dirname(__file__)))
    with open(os.path.join(here, "serving", "console", "rdf.html.fragment"),
              encoding="utf-8") as f:
        return console_page("Oryx RDF", f.read())


route("GET", "/index.html", produces=("text/html",))(console)
