"""Sharded (multi-rank) ALS generation: build, evaluate and publish with every rank holding
only its share of the data, the dictionaries, the factors and the output.

The reference's ALS update is one Spark program at every scale
(``[lambda]/batch/BatchUpdateFunction.java:86-155`` -> ``[mllib]/als/ALSUpdate.java:100-230``):
parse on the executors, ``reduceByKey`` per (user, item) after mapping string IDs to ints,
MLlib block ALS, then ``saveAsTextFile`` of X/ and Y/ and per-partition ``UP`` publishing
(``EnqueueFeatureVecsFn``, ``EnqueueFeatureVecsAndKnownItemsFn``).  On an MI355X node each
rank (one GPU) does the same with its share:

1. **parse** its share of the lines natively -- reusing its resident parse of the past part
   files it owns (:mod:`.history`, one history per rank) -- and apply time decay on the host;
2. **global dictionaries** (:class:`~oryx_amd.parallel.shuffle.ShardedDict`): user / item key
   blobs go to their owner rank (``crc32 % W``), which numbers them in a native dictionary;
   codes come back the same way -- no Python string per ID;
3. **route** every event (24 bytes: packed user|item code, decayed strength, raw timestamp) to
   its user's owner in ONE device all-to-all; the owner aggregates per (user, item) in time
   order on the GPU (``reduceByKey``) and, when the training data is the whole data set,
   also derives each user's known items from the same events;
4. **dense ids aligned with ownership**: the j-th used user of owner r gets dense id
   ``j * W + r`` -- exactly the row the trainer's round-robin row sharding gives rank r
   (``ALSTrainer``: row d lives on rank ``d % W``), so every rank's factor rows are the rows
   of the IDs it owns.  Items get dense ids the same way from an all-reduced used mask.
   Dense ids nobody uses (the shards are padded to the largest) are empty rows that stay
   zero;
5. **outputs stay sharded**: each rank formats its own factor rows on its GPU
   (``textfmt.hip``), writes ``X/part-<rank>.gz`` / ``Y/part-<rank>.gz`` (the reference's
   part files) and publishes its own ``UP`` rows with its own ID strings and known items;
   only the PMML's ``XIDs`` / ``YIDs`` lists travel to rank 0.

Evaluation routes the test events to their user's owner as well: AUC / RMSE are per-rank
partial sums over the owner's X rows and an all-gathered Y (``Evaluation.java:49-136``).
"""

from __future__ import annotations

import logging
import math
import os
import time
from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import numpy as np
import torch

from ... import ingest
from ...ops import textfmt
from ...parallel import dist, shuffle
from . import evaluation

log = logging.getLogger(__name__)

__all__ = ["ShardedModel", "route_events", "build", "evaluate", "publish"]

_NO_TS = -(1 << 62)          # parse marker of a line without a timestamp (models/als/batch)
_MASK32 = (1 << 32) - 1


@dataclass
class RoutedEvents:
    """This rank's events after routing to their user's owner (device tensors)."""
    lu: torch.Tensor          # int64 owner-local user code
    gi: torch.Tensor          # int64 global item code
    s: torch.Tensor           # fp64 decayed strength (NaN = delete)
    ts: torch.Tensor          # int64 raw timestamp (_NO_TS: none)


@dataclass
class ShardedModel:
    """What one candidate's sharded build keeps for its evaluation and publishing."""
    U: shuffle.ShardedDict
    I: shuffle.ShardedDict
    user_j: torch.Tensor      # int64 [U.size]: j of each owned user (-1: unused)
    item_dense: torch.Tensor  # int64 [I.total]: dense id of each global item (-1: unused)
    used_u: np.ndarray        # owned local user codes in dense (j) order
    used_i: np.ndarray        # owned local item codes in dense (j) order
    counts_u: list
    counts_i: list
    X_local: torch.Tensor     # fp32 [su, k] this rank's user rows (row j)
    Y_local: torch.Tensor     # fp32 [si, k] this rank's item rows
    x_keys: Tuple[np.ndarray, np.ndarray]
    y_keys: Tuple[np.ndarray, np.ndarray]
    x_rows: textfmt.RowText
    y_rows: textfmt.RowText
    known: Optional[Tuple[torch.Tensor, torch.Tensor]]   # (local user, global item) pairs
    n_users: int
    n_items: int


def _sync(dev) -> None:
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def route_events(lines, ctx: dist.DistContext, decay_factor: float, now: int,
                 history=None, U: Optional[shuffle.ShardedDict] = None,
                 timers: Optional[Dict[str, float]] = None):
    """Parse this rank's ``lines``, give users and items global codes and send every event to
    its user's owner.  ``U`` given: users are looked up in it (events of users it lacks are
    dropped) and items get a fresh dictionary.  Returns (events, U, I)."""
    ph = timers if timers is not None else {}
    dev = ctx.device
    tp = time.perf_counter()
    users, items = ingest.IdDict(), ingest.IdDict()
    parse = history.parse_ratings if history is not None else ingest.parse_ratings
    u, i, s, ts0 = parse(lines, users, items, default_ts=_NO_TS)
    if decay_factor < 1.0 and len(s):
        # same arithmetic as batch.parse_ratings (bit-identical decayed strengths)
        ts_eff = np.where(ts0 == _NO_TS, now, ts0)
        days = np.maximum(0, now - ts_eff) / 86400000.0
        s = np.where(ts_eff >= now, s, s * np.power(decay_factor, days))
    ph["parse"] = ph.get("parse", 0.0) + time.perf_counter() - tp
    tp = time.perf_counter()
    if U is None:
        ucode, U = shuffle.ShardedDict.build(users, ctx)
    else:
        ucode = U.lookup(users)
    icode, I = shuffle.ShardedDict.build(items, ctx)
    ph["dictionaries"] = ph.get("dictionaries", 0.0) + time.perf_counter() - tp
    tp = time.perf_counter()
    gu = torch.from_numpy(ucode).to(dev)[torch.from_numpy(u).to(dev)] if len(u) else \
        torch.zeros(0, dtype=torch.int64, device=dev)
    gi = torch.from_numpy(icode).to(dev)[torch.from_numpy(i).to(dev)] if len(i) else \
        torch.zeros(0, dtype=torch.int64, device=dev)
    st = torch.from_numpy(np.ascontiguousarray(s, dtype=np.float64)).to(dev)
    tt = torch.from_numpy(np.ascontiguousarray(ts0, dtype=np.int64)).to(dev)
    ok = gu >= 0
    if not bool(ok.all()):
        gu, gi, st, tt = gu[ok], gi[ok], st[ok], tt[ok]
    assert U.total < (1 << 31) and I.total < (1 << 31)
    packed = (gu << 32) | gi
    owner = U.owner_of_t(gu)
    packed, st, tt = shuffle.route_tensors(owner, ctx, packed, st, tt)
    ev = RoutedEvents((packed >> 32) - U.lo, packed & _MASK32, st, tt)
    _sync(dev)
    ph["route"] = ph.get("route", 0.0) + time.perf_counter() - tp
    return ev, U, I


def known_pairs(ev: RoutedEvents, dev) -> Tuple[torch.Tensor, torch.Tensor]:
    """(local user, global item) of every pair whose last event in time order (lines without
    a timestamp first) is not a delete -- the reference's known items."""
    from .batch import aggregate_scores_device
    if ev.lu.numel() == 0:
        e = torch.zeros(0, dtype=torch.int64, device=dev)
        return e, e
    tk = torch.where(ev.ts == _NO_TS, torch.zeros_like(ev.ts), ev.ts)
    ku, ki, _ = aggregate_scores_device(ev.lu, ev.gi, ev.s, tk, False, dev, to_host=False)
    return ku, ki


def build(upd, ctx: dist.DistContext, lines, features: int, lam: float, alpha: float,
          candidate_path: Optional[str], want_known: bool, history=None):
    """One candidate's sharded build (collective).  Returns (PMML on rank 0 / a skeleton on
    the others, :class:`ShardedModel`) or (None, None) without ratings."""
    from ...utils import pmml as pmmlu, rng
    from .batch import aggregate_scores_device, write_features
    from .trainer import ALS_INIT_SEED, ALSTrainer
    W, R, dev = ctx.world_size, ctx.rank, ctx.device
    ph = upd.phase_seconds
    now = int(time.time() * 1000)
    ev, U, I = route_events(lines, ctx, upd.decay_factor, now, history=history, timers=ph)
    tp = time.perf_counter()
    keep = None
    if upd.decay_zero_threshold > 0.0:
        keep = ev.s > upd.decay_zero_threshold          # drops deletes too, as on one rank
    lu, gi, s, ts = (ev.lu, ev.gi, ev.s, ev.ts) if keep is None else \
        (ev.lu[keep], ev.gi[keep], ev.s[keep], ev.ts[keep])
    ts = torch.where(ts == _NO_TS, torch.full_like(ts, now), ts)
    au, ai, av = aggregate_scores_device(lu, gi, s, ts, upd.implicit, dev, to_host=False)
    del lu, gi, s, ts
    known = known_pairs(ev, dev) if want_known else None
    del ev
    # dense ids: owner r's j-th used user -> j * W + r (the trainer's row of rank r)
    user_used = torch.zeros(U.size, dtype=torch.bool, device=dev)
    user_used[au] = True
    item_cnt = torch.zeros(max(I.total, 1), dtype=torch.int32, device=dev)
    item_cnt[ai] = 1
    if ctx.is_distributed:
        torch.distributed.all_reduce(item_cnt, group=ctx.group)
    item_used = item_cnt[:I.total] > 0
    counts_u = shuffle.all_gather_int(int(user_used.sum()), ctx)
    n_ratings = int(sum(shuffle.all_gather_int(int(au.numel()), ctx)))
    _sync(dev)
    ph["aggregate"] = ph.get("aggregate", 0.0) + time.perf_counter() - tp
    if n_ratings == 0:
        log.info("No ratings after aggregation")
        return None, None
    tp = time.perf_counter()
    user_j = torch.cumsum(user_used, 0) - 1
    user_j = torch.where(user_used, user_j, torch.full_like(user_j, -1))
    # item j within its owner's range: used items before it in the range
    off = torch.as_tensor(I.offsets, device=dev)
    cum0 = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev),
                      torch.cumsum(item_used.to(torch.int64), 0)])
    own_of = torch.searchsorted(off, torch.arange(I.total, device=dev), right=True) - 1
    base = cum0[off]                                   # [W + 1]
    item_dense = torch.where(item_used, (cum0[:-1] - base[own_of]) * W + own_of,
                             torch.full_like(own_of, -1))
    counts_i = [int(x) for x in (base[1:] - base[:-1]).cpu().tolist()]
    n_users, n_items = W * max(counts_u), W * max(counts_i)
    trainer = ALSTrainer(features, lam, alpha, upd.implicit, ctx=ctx, seed=rng.next_seed(),
                         precision=upd.precision, init_seed=ALS_INIT_SEED)
    du = user_j[au] * W + R
    di = item_dense[ai]
    ph["ids_remap"] = ph.get("ids_remap", 0.0) + time.perf_counter() - tp
    tp = time.perf_counter()
    trainer.prepare(du, di, av.to(torch.float32), n_users, n_items)
    del du, di, au, ai, av
    ph["csr_prepare"] = ph.get("csr_prepare", 0.0) + time.perf_counter() - tp
    x_init = y_init = None
    used_u = torch.nonzero(user_used).flatten().cpu().numpy()
    lo_i, hi_i = int(I.offsets[R]), int(I.offsets[R + 1])
    used_i = torch.nonzero(item_used[lo_i:hi_i]).flatten().cpu().numpy()
    x_keys = U.own.keys_blob(used_u)
    y_keys = I.own.keys_blob(used_i)
    if upd.warm_start and upd.current_model_dir:
        x_init, y_init = _warm_start_sharded(upd.current_model_dir, features, x_keys, y_keys,
                                             n_users, n_items, W, R)
    tp = time.perf_counter()
    # random rows keyed by ID: the same start as a one-rank generation of the same data
    trainer.train(upd.iterations, x_init=x_init, y_init=y_init,
                  x_keys=ingest.blob_hash64(*x_keys), y_keys=ingest.blob_hash64(*y_keys))
    _sync(dev)
    ph["train"] = ph.get("train", 0.0) + time.perf_counter() - tp
    tph = getattr(upd, "train_phases", None)
    if tph is not None:
        for key in ("init_ms", "checkpoint_ms", "factors_ms"):
            if key in trainer.timings:
                tph[key[:-3]] = tph.get(key[:-3], 0.0) + trainer.timings[key] / 1e3
        tph["iterations"] = tph.get("iterations", 0.0) + \
            sum(trainer.timings.get("iteration_ms", [])) / 1e3
    tp = time.perf_counter()
    k = features
    X_local = trainer.X[:trainer.su, :k]
    Y_local = trainer.Y[:trainer.si, :k]
    x_rows = textfmt.format_rows(X_local[:counts_u[R]])
    y_rows = textfmt.format_rows(Y_local[:counts_i[R]])
    ph["format_rows"] = ph.get("format_rows", 0.0) + time.perf_counter() - tp
    tp = time.perf_counter()
    if candidate_path is not None:
        # every rank writes its own part files, as the reference's saveAsTextFile partitions
        write_features(os.path.join(candidate_path, "X"), x_keys, x_rows, part=R)
        write_features(os.path.join(candidate_path, "Y"), y_keys, y_rows, part=R)
    ph["write_factors"] = ph.get("write_factors", 0.0) + time.perf_counter() - tp
    tp = time.perf_counter()
    xid = U.all_keys_blob(keep=user_used.cpu().numpy(), to_main=True)
    yid = I.all_keys_blob(keep=item_used[lo_i:hi_i].cpu().numpy(), to_main=True)
    pmml = pmmlu.build_skeleton_pmml()
    pmml.add_extension("X", "X/")
    pmml.add_extension("Y", "Y/")
    pmml.add_extension("features", features)
    pmml.add_extension("lambda", lam)
    pmml.add_extension("implicit", upd.implicit)
    if upd.implicit:
        pmml.add_extension("alpha", alpha)
    if ctx.is_main:
        pmml.add_extension_content("XIDs", ingest.blob_strings(*xid))
        pmml.add_extension_content("YIDs", ingest.blob_strings(*yid))
    ph["pmml"] = ph.get("pmml", 0.0) + time.perf_counter() - tp
    model = ShardedModel(U, I, user_j, item_dense, used_u, used_i, counts_u, counts_i,
                         X_local, Y_local, x_keys, y_keys, x_rows, y_rows, known,
                         n_users, n_items)
    its = trainer.timings.get("iteration_ms", [])
    upd._timings[candidate_path] = {
        "ratings": n_ratings, "users": sum(counts_u), "items": sum(counts_i), "ranks": W,
        "sharded": True, "prepare_s": trainer.timings.get("prepare_s"), "iteration_ms": its,
        "ratings_per_s": (n_ratings * 1e3 / (sum(its) / len(its))) if its else None}
    log.info("ALS (sharded, %d ranks) %d ratings, %d users, %d items, rank %d", W, n_ratings,
             sum(counts_u), sum(counts_i), features)
    # the candidate directory is complete (every rank's parts) before anyone moves it
    dist.barrier(ctx)
    return pmml, model


def _warm_start_sharded(model_dir, features, x_keys, y_keys, n_users, n_items, W, R):
    """Previous generation's factors for this rank's rows (NaN rows: random init), as full
    [n, k] matrices the trainer takes its rows ``R::W`` from."""
    from .batch import read_features
    out = []
    for sub, keys, n in (("X", x_keys, n_users), ("Y", y_keys, n_items)):
        init = np.full((n, features), np.nan, dtype=np.float32)
        try:
            ids, mat = read_features(os.path.join(model_dir, sub))
        except OSError:
            ids, mat = [], None
        if ids and mat is not None and mat.shape[1] == features:
            d = ingest.IdDict()
            d.encode(ids)
            codes = d.find_blob(*keys)
            ok = codes >= 0
            j = np.nonzero(ok)[0]
            init[j * W + R] = mat[codes[ok]]
        out.append(torch.from_numpy(init))
    return out[0], out[1]


def evaluate(upd, ctx: dist.DistContext, m: ShardedModel, test_lines) -> float:
    """AUC (implicit) or -RMSE of a sharded model on this rank's test lines (collective)."""
    from .batch import aggregate_scores_device
    W, dev = ctx.world_size, ctx.device
    now = int(time.time() * 1000)
    tp = time.perf_counter()
    users, items = ingest.IdDict(), ingest.IdDict()
    u, i, s, ts = ingest.parse_ratings(test_lines, users, items, default_ts=now)
    if upd.decay_factor < 1.0 and len(s):
        days = np.maximum(0, now - ts) / 86400000.0
        s = np.where(ts >= now, s, s * np.power(upd.decay_factor, days))
    if upd.decay_zero_threshold > 0.0:
        keep = s > upd.decay_zero_threshold
        u, i, s, ts = u[keep], i[keep], s[keep], ts[keep]
    gu = m.U.lookup(users)
    gi = m.I.lookup(items)
    gu = gu[u] if len(u) else u
    gi = gi[i] if len(i) else i
    ok = (gu >= 0) & (gi >= 0)        # pairs the model cannot score are dropped (the join)
    gu_t = torch.from_numpy(np.ascontiguousarray(gu[ok])).to(dev)
    gi_t = torch.from_numpy(np.ascontiguousarray(gi[ok])).to(dev)
    s_t = torch.from_numpy(np.ascontiguousarray(s[ok], dtype=np.float64)).to(dev)
    t_t = torch.from_numpy(np.ascontiguousarray(ts[ok], dtype=np.int64)).to(dev)
    packed = (gu_t << 32) | gi_t
    packed, s_t, t_t = shuffle.route_tensors(m.U.owner_of_t(gu_t), ctx, packed, s_t, t_t)
    au, ai, av = aggregate_scores_device((packed >> 32) - m.U.lo, packed & _MASK32, s_t, t_t,
                                         upd.implicit, dev, to_host=False)
    # rows: X_local[j] for the owner's j-th user; Y gathered rank-major: dense d at
    # (d % W) * si + d // W
    uj = m.user_j[au] if au.numel() else au
    dd = m.item_dense[ai] if ai.numel() else ai
    sel = (uj >= 0) & (dd >= 0)
    uj, dd, av = uj[sel], dd[sel], av[sel]
    si = m.Y_local.shape[0]
    Yg = dist.all_gather_rows(m.Y_local.contiguous(), W * si, ctx) if ctx.is_distributed \
        else m.Y_local
    yrow = (dd % W) * si + torch.div(dd, W, rounding_mode="floor")
    upd.phase_seconds["eval_prepare"] = upd.phase_seconds.get("eval_prepare", 0.0) + \
        time.perf_counter() - tp
    tp = time.perf_counter()
    try:
        if upd.implicit:
            items_all = torch.unique(yrow)
            if ctx.is_distributed:
                parts = shuffle.all_gather_var(items_all.cpu().numpy(), ctx)
                items_all = torch.from_numpy(np.unique(np.concatenate(parts))).to(dev)
            tot, cnt = evaluation.auc_parts(m.X_local, Yg, uj, yrow, items_all)
            tc = shuffle.all_reduce_np(np.array([tot, cnt], dtype=np.float64), ctx)
            auc = float(tc[0] / tc[1]) if tc[1] > 0 else float("nan")
            log.info("AUC: %s", auc)
            return auc
        se, n = evaluation.squared_error_parts(m.X_local, Yg, uj, yrow, av)
        tc = shuffle.all_reduce_np(np.array([se, n], dtype=np.float64), ctx)
        rmse = math.sqrt(tc[0] / tc[1]) if tc[1] > 0 else float("nan")
        log.info("RMSE: %s", rmse)
        return -rmse
    finally:
        upd.phase_seconds["eval"] = upd.phase_seconds.get("eval", 0.0) + \
            time.perf_counter() - tp


def _name_order(names_blob: Tuple[np.ndarray, np.ndarray]) -> np.ndarray:
    """Rank of every key in ID-string order (the order of a user's known items)."""
    strs = ingest.blob_strings(*names_blob)
    rank = np.empty(len(strs), dtype=np.int64)
    rank[np.argsort(np.array(strs, dtype=object), kind="stable")] = np.arange(len(strs))
    return rank


def _known_text(m_U, I: shuffle.ShardedDict, ku: torch.Tensor, ki: torch.Tensor, ctx):
    """Known items of this rank's users as JSON array text per owner-local user code."""
    names_blob = I.all_keys_blob()
    names = ingest.IdDict.from_blob(*names_blob)
    if ku.numel() == 0:
        return ingest.known_items_text(names, np.zeros(0, np.int64), np.zeros(0, np.int64),
                                       m_U.size)
    rank = torch.from_numpy(_name_order(names_blob)).to(ku.device)
    order = torch.argsort(ku * (len(names) + 1) + rank[ki])
    return ingest.known_items_text(names, ku[order].cpu().numpy(), ki[order].cpu().numpy(),
                                   m_U.size)


def publish(upd, ctx: dist.DistContext, m: ShardedModel, all_lines, topic) -> None:
    """Every rank publishes its own Y rows, then its own X rows with their known items
    (collective)."""
    R = ctx.rank
    ph = upd.phase_seconds
    tp = time.perf_counter()
    if len(m.y_rows):
        topic.send_block("UP", ingest.assemble_row_messages("Y", m.y_keys, m.y_rows))
    log.info("Rank %d sent %d item / Y rows as model updates", R, len(m.y_rows))
    dist.barrier(ctx)
    ph["publish_y"] = ph.get("publish_y", 0.0) + time.perf_counter() - tp
    tp = time.perf_counter()
    if upd.no_known_items:
        if len(m.x_rows):
            topic.send_block("UP", ingest.assemble_row_messages("X", m.x_keys, m.x_rows))
    else:
        if m.known is not None:
            kt = _known_text(m.U, m.I, m.known[0], m.known[1], ctx)
        else:
            # the training data was not the whole data set: route all of it once more
            ev, _, I2 = route_events(all_lines, ctx, 1.0, 0, history=upd._history_for(ctx.device),
                                     U=m.U)
            ku, ki = known_pairs(ev, ctx.device)
            kt = _known_text(m.U, I2, ku, ki, ctx)
        if len(m.x_rows):
            topic.send_block("UP", ingest.assemble_row_messages(
                "X", m.x_keys, m.x_rows, kt, m.used_u.astype(np.int64)))
    log.info("Rank %d sent %d user / X rows as model updates", R, len(m.x_rows))
    dist.barrier(ctx)
    ph["publish_x"] = ph.get("publish_x", 0.0) + time.perf_counter() - tp


def publish_from_files(upd, ctx: dist.DistContext, model_path: str, all_lines, topic) -> None:
    """Publish a model no rank of this world built in memory (the winner of another candidate
    group): the factors come from its ``X/`` / ``Y/`` part files.  Each rank sends the Y rows
    of its stripe, then the X rows of the users it owns (``crc32 % W``) with their known
    items from every rank's share of ``all_lines`` (collective)."""
    from .batch import read_features
    W, R = ctx.world_size, ctx.rank
    y_ids, Y = read_features(os.path.join(model_path, "Y"))
    mine = np.arange(R, len(y_ids), W)
    if len(mine):
        topic.send_block("UP", ingest.assemble_row_messages(
            "Y", [y_ids[j] for j in mine.tolist()], textfmt.format_rows(Y[mine])))
    dist.barrier(ctx)
    x_ids, X = read_features(os.path.join(model_path, "X"))
    xd = ingest.IdDict()
    xd.encode(x_ids)
    own = np.nonzero(xd.owners(W) == R)[0]
    keys = xd.keys_blob(own)
    if upd.no_known_items:
        if len(own):
            topic.send_block("UP", ingest.assemble_row_messages(
                "X", keys, textfmt.format_rows(X[own])))
    else:
        ev, U, I = route_events(all_lines, ctx, 1.0, 0, history=upd._history_for(ctx.device))
        ku, ki = known_pairs(ev, ctx.device)
        kt = _known_text(U, I, ku, ki, ctx)
        code = U.own.find_blob(*keys)          # users without any event are not sent
        ok = code >= 0
        if ok.any():
            topic.send_block("UP", ingest.assemble_row_messages(
                "X", xd.keys_blob(own[ok]), textfmt.format_rows(X[own[ok]]), kt, code[ok]))
    dist.barrier(ctx)
