"""k-means REST endpoints: ``/distanceToNearest`` and the console; ``/assign`` and ``/add``
come from the generic :mod:`oryx_amd.serving.clustering` package (as the reference's
``[serving-app]/clustering`` package serves them for any clustering model).

``/distanceToNearest/{datum}`` (``[serving-app]/kmeans/DistanceToNearest.java:36-50``) returns
the Euclidean distance to the nearest center as a Java ``Double.toString``.
"""

from __future__ import annotations

import os

from ...serving.http import route
from ...serving.resources import check, console_page, get_serving_model
from ...utils import text
from .common import features_from_tokens

INCLUDE_RESOURCES = ["oryx_amd.serving.clustering"]

__all__ = []


@route("GET", "/distanceToNearest/{datum}", produces=("text/plain", "text/csv",
                                                      "application/json"))
def distance_to_nearest(req, datum):
    check(datum is not None and datum != "", "Data is needed to cluster")
    model = get_serving_model(req)
    tokens = text.parse_delimited(datum, ",")
    _, dist = model.closest_cluster(features_from_tokens(tokens, model.get_input_schema()))
    return text.java_double_str(dist)


@route("GET", "/", produces=("text/html",))
def console(req):
    here = os.path.dirname(os.path.dirname(os.path.dirname(__file__)))
    with open(os.path.join(here, "serving", "console", "kmeans.html.fragment"),
              encoding="utf-8") as f:
        return console_page("Oryx k-means", f.read())


route("GET", "/index.html", produces=("text/html",))(console)
