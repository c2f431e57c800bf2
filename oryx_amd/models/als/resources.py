"""ALS REST endpoints (the 19 resources of ``[serving-app]/als/*.java``).

Paths, parameters, defaults and status codes follow the reference:
``/recommend``, ``/recommendToMany``, ``/recommendToAnonymous``, ``/recommendWithContext``,
``/similarity``, ``/similarityToItem``, ``/estimate``, ``/estimateForAnonymous``, ``/because``,
``/mostSurprising``, ``/knownItems``, ``/mostPopularItems``, ``/mostActiveUsers``,
``/popularRepresentativeItems``, ``/item/allIDs``, ``/user/allIDs``, ``/pref`` (POST/DELETE),
``/ingest`` and the console.  Scoring functions (``DotsFunction`` / ``CosineAverageFunction``,
``[serving-app]/als/DotsFunction.java:25-57``, ``CosineAverageFunction.java:25-63``) reduce to
one target vector that the GPU scan scores against every item.
"""

from __future__ import annotations

import math
import os
import time
from typing import List, Optional, Tuple

import numpy as np

from ...serving.http import route
from ...serving.resources import (IDCount, IDValue, check, check_exists, check_not_read_only,
                                  console_page, get_serving_model, input_lines, send_input)
from ...utils import mathx, text
from .common import compute_updated_xu

__all__ = []


def _model(req):
    return get_serving_model(req)


def _paging(req) -> Tuple[int, int]:
    how_many = req.q_int("howMany", 10)
    offset = req.q_int("offset", 0)
    check(how_many > 0, "howMany must be positive")
    check(offset >= 0, "offset must be nonnegative")
    return how_many, offset


def _to_id_values(pairs, how_many: int, offset: int) -> List[IDValue]:
    return [IDValue(i, v) for i, v in list(pairs)[offset:offset + how_many]]


def dots_target(vectors: List[np.ndarray]) -> np.ndarray:
    """``DotsFunction``: mean of the given user vectors (float32 sums as in the reference)."""
    acc = np.zeros_like(vectors[0], dtype=np.float32)
    for v in vectors:
        acc += np.asarray(v, dtype=np.float32)
    return (acc / np.float32(len(vectors))).astype(np.float32)


def cosine_target(vectors: List[np.ndarray]) -> np.ndarray:
    """``CosineAverageFunction``: mean of unit vectors."""
    acc = np.zeros_like(vectors[0], dtype=np.float32)
    for v in vectors:
        acc += (np.asarray(v, dtype=np.float32) / mathx.norm(v)).astype(np.float32)
    return (acc / np.float32(len(vectors))).astype(np.float32)


def _rescorer(model, kind: str, ids, args):
    provider = model.get_rescorer_provider()
    if provider is None:
        return None
    if kind == "recommend":
        return provider.get_recommend_rescorer(ids, args)
    if kind == "anonymous":
        return provider.get_recommend_to_anonymous_rescorer(ids, args)
    if kind == "similar":
        return provider.get_most_similar_items_rescorer(args)
    if kind == "popular":
        return provider.get_most_popular_items_rescorer(args)
    if kind == "active":
        return provider.get_most_active_users_rescorer(args)
    raise ValueError(kind)


def parse_path_segments(segments: List[str]) -> List[Tuple[str, float]]:
    out = []
    for s in segments:
        i = s.find("=")
        out.append((s, 1.0) if i < 0 else (s[:i], float(s[i + 1:])))
    return out


def build_temporary_user_vector(model, parsed: List[Tuple[str, float]],
                                xu: Optional[np.ndarray]) -> Optional[np.ndarray]:
    solver = model.get_yty_solver()
    for item, value in parsed:
        yi = model.get_item_vector(item)
        new = compute_updated_xu(solver, value, xu, yi, model.is_implicit())
        if new is not None:
            xu = new
    return xu


@route("GET", "/recommend/{userID}")
def recommend(req, userID):
    how_many, offset = _paging(req)
    consider_known = req.q_bool("considerKnownItems", False)
    model = _model(req)
    uv = model.get_user_vector(userID)
    check_exists(uv is not None, userID)
    exclude = None if consider_known else model.get_known_items(userID)
    rescorer = _rescorer(model, "recommend", [userID], req.q_list("rescorerParams"))
    top = model.top_n(uv, how_many + offset, exclude=exclude, rescorer=rescorer)
    return _to_id_values(top, how_many, offset)


@route("GET", "/recommendToMany/{userID : .+}")
def recommend_to_many(req, userID):
    check(len(userID) > 0, "Need at least 1 user")
    how_many, offset = _paging(req)
    consider_known = req.q_bool("considerKnownItems", False)
    model = _model(req)
    vecs, known = [], set()
    for u in userID:
        v = model.get_user_vector(u)
        check_exists(v is not None, u)
        vecs.append(v)
        if not consider_known:
            known.update(model.get_known_items(u))
    rescorer = _rescorer(model, "recommend", list(userID), req.q_list("rescorerParams"))
    top = model.top_n(dots_target(vecs), how_many + offset, exclude=known, rescorer=rescorer)
    return _to_id_values(top, how_many, offset)


@route("GET", "/recommendToAnonymous/{itemID : .+}")
def recommend_to_anonymous(req, itemID):
    check(len(itemID) > 0, "Need at least 1 item to make recommendations")
    how_many, offset = _paging(req)
    model = _model(req)
    parsed = parse_path_segments(itemID)
    anon = build_temporary_user_vector(model, parsed, None)
    check(anon is not None, str(itemID))
    known = [i for i, _ in parsed]
    rescorer = _rescorer(model, "anonymous", known, req.q_list("rescorerParams"))
    top = model.top_n(anon, how_many + offset, exclude=set(known), rescorer=rescorer)
    return _to_id_values(top, how_many, offset)


@route("GET", "/recommendWithContext/{userID}/{itemID : .*}")
def recommend_with_context(req, userID, itemID):
    how_many, offset = _paging(req)
    consider_known = req.q_bool("considerKnownItems", False)
    model = _model(req)
    parsed = parse_path_segments(itemID)
    uv = model.get_user_vector(userID)
    check_exists(uv is not None, userID)
    temp = build_temporary_user_vector(model, parsed, uv)
    known = {i for i, _ in parsed}
    if not consider_known:
        known.update(model.get_known_items(userID))
    rescorer = _rescorer(model, "recommend", [userID], req.q_list("rescorerParams"))
    top = model.top_n(temp, how_many + offset, exclude=known, rescorer=rescorer)
    return _to_id_values(top, how_many, offset)


@route("GET", "/similarity/{itemID : .+}")
def similarity(req, itemID):
    check(len(itemID) > 0, "Need at least 1 item to determine similarity")
    how_many, offset = _paging(req)
    model = _model(req)
    vecs = []
    for i in itemID:
        v = model.get_item_vector(i)
        check_exists(v is not None, i)
        vecs.append(v)
    rescorer = _rescorer(model, "similar", None, req.q_list("rescorerParams"))
    top = model.top_n(cosine_target(vecs), how_many + offset, cosine=True, exclude=set(itemID),
                      rescorer=rescorer)
    return _to_id_values(top, how_many, offset)


@route("GET", "/similarityToItem/{toItemID}/{itemID : .+}")
def similarity_to_item(req, toItemID, itemID):
    model = _model(req)
    to = model.get_item_vector(toItemID)
    check_exists(to is not None, toItemID)
    to_norm = mathx.norm(to)
    out = []
    for i in itemID:
        v = model.get_item_vector(i)
        if v is None:
            out.append(0.0)
        else:
            val = mathx.dot(v, to) / (to_norm * mathx.norm(v))
            if math.isinf(val) or math.isnan(val):
                raise RuntimeError("Bad similarity")
            out.append(val)
    return out


@route("GET", "/estimate/{userID}/{itemID : .+}")
def estimate(req, userID, itemID):
    model = _model(req)
    uv = model.get_user_vector(userID)
    check_exists(uv is not None, userID)
    out = []
    for i in itemID:
        v = model.get_item_vector(i)
        if v is None:
            out.append(0.0)
        else:
            val = mathx.dot(v, uv)
            if math.isinf(val) or math.isnan(val):
                raise RuntimeError("Bad estimate")
            out.append(val)
    return out


@route("GET", "/estimateForAnonymous/{toItemID}/{itemID : .+}")
def estimate_for_anonymous(req, toItemID, itemID):
    model = _model(req)
    to = model.get_item_vector(toItemID)
    check_exists(to is not None, toItemID)
    anon = build_temporary_user_vector(model, parse_path_segments(itemID), None)
    return 0.0 if anon is None else mathx.dot(anon, to)


@route("GET", "/because/{userID}/{itemID}")
def because(req, userID, itemID):
    how_many, offset = _paging(req)
    model = _model(req)
    iv = model.get_item_vector(itemID)
    check_exists(iv is not None, itemID)
    known = model.get_known_item_vectors_for_user(userID)
    if not known:
        return []
    iv_norm = mathx.norm(iv)
    sims = [(other, mathx.dot(iv, vec) / (iv_norm * mathx.norm(vec))) for other, vec in known]
    sims.sort(key=lambda p: -p[1])
    return _to_id_values(sims, how_many, offset)


@route("GET", "/mostSurprising/{userID}")
def most_surprising(req, userID):
    how_many, offset = _paging(req)
    model = _model(req)
    uv = model.get_user_vector(userID)
    check_exists(uv is not None, userID)
    known = model.get_known_item_vectors_for_user(userID)
    if not known:
        return []
    dots = [(i, mathx.dot(uv, v)) for i, v in known]
    dots.sort(key=lambda p: p[1])
    return _to_id_values(dots, how_many, offset)


@route("GET", "/knownItems/{userID}")
def known_items(req, userID):
    return sorted(_model(req).get_known_items(userID))


def _top_counts(counts, how_many, offset, rescorer) -> List[IDCount]:
    pairs = list(counts.items())
    if rescorer is not None:
        pairs = [p for p in pairs if not rescorer.is_filtered(p[0])]
    pairs.sort(key=lambda p: -p[1])
    return [IDCount(i, c) for i, c in pairs[offset:offset + how_many]]


@route("GET", "/mostPopularItems")
def most_popular_items(req):
    how_many, offset = req.q_int("howMany", 10), req.q_int("offset", 0)
    model = _model(req)
    rescorer = _rescorer(model, "popular", None, req.q_list("rescorerParams"))
    return _top_counts(model.get_item_counts(), how_many, offset, rescorer)


@route("GET", "/mostActiveUsers")
def most_active_users(req):
    how_many, offset = req.q_int("howMany", 10), req.q_int("offset", 0)
    model = _model(req)
    rescorer = _rescorer(model, "active", None, req.q_list("rescorerParams"))
    return _top_counts(model.get_user_counts(), how_many, offset, rescorer)


@route("GET", "/popularRepresentativeItems")
def popular_representative_items(req):
    model = _model(req)
    k = model.get_features()
    out = []
    for i in range(k):
        unit = np.zeros(k, dtype=np.float32)
        unit[i] = 1.0
        top = model.top_n(unit, 1)
        out.append(top[0][0] if top else None)
    return out


@route("GET", "/item/allIDs")
def all_item_ids(req):
    return _model(req).get_all_item_ids()


@route("GET", "/user/allIDs")
def all_user_ids(req):
    return _model(req).get_all_user_ids()


def validate_and_standardize_strength(raw: Optional[str]) -> str:
    if raw is None or raw.strip() == "":
        return "1"
    try:
        value = np.float32(float(raw))
    except ValueError as e:
        from ...api import OryxServingException
        raise OryxServingException(400, str(e))
    check(not (math.isnan(value) or math.isinf(value)), raw)
    return text.java_float_str(float(value))


@route("POST", "/pref/{userID}/{itemID}")
def pref_post(req, userID, itemID):
    check_not_read_only(req)
    body = req.text()
    line = body.splitlines()[0] if body else None
    value = validate_and_standardize_strength(line)
    send_input(req, "%s,%s,%s,%d" % (userID, itemID, value, int(time.time() * 1000)))


@route("DELETE", "/pref/{userID}/{itemID}")
def pref_delete(req, userID, itemID):
    check_not_read_only(req)
    send_input(req, "%s,%s,,%d" % (userID, itemID, int(time.time() * 1000)))


@route("POST", "/ingest")
def ingest(req):
    check_not_read_only(req)
    for line in input_lines(req):
        if line == "":
            continue
        tokens = text.parse_delimited(line, ",")
        check(len(tokens) >= 2, line)
        user, item = tokens[0], tokens[1]
        if len(tokens) >= 3:
            raw = tokens[2]
            strength = "" if raw == "" else validate_and_standardize_strength(raw)
            if len(tokens) >= 4:
                try:
                    ts = int(tokens[3])
                except ValueError as e:
                    from ...api import OryxServingException
                    raise OryxServingException(400, str(e))
                check(ts > 0, line)
            else:
                ts = int(time.time() * 1000)
        else:
            strength = "1"
            ts = int(time.time() * 1000)
        send_input(req, "%s,%s,%s,%d" % (user, item, strength, ts))


@route("GET", "/", produces=("text/html",))
def console(req):
    here = os.path.dirname(os.path.dirname(os.path.dirname(__file__)))
    with open(os.path.join(here, "serving", "console", "als.html.fragment"),
              encoding="utf-8") as f:
        return console_page("Oryx ALS", f.read())


route("GET", "/index.html", produces=("text/html",))(console)
