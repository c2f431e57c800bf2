"""ML tier: candidate models, hyperparameter search, train/test split, atomic publish.

Equivalent of ``MLUpdate`` (``[ml]/MLUpdate.java:59-372``):

1. choose hyperparameter combos (``oryx.ml.eval.candidates``) -- :mod:`.hyperparams`;
2. build ``candidates`` models in parallel (``oryx.ml.eval.parallelism``), each on a fresh
   train/test split, into ``model-dir/.temporary/<ts>/<i>/model.pmml``;
3. evaluate each on its test split; pick the highest eval (NaN ignored; with test fraction 0
   the single model is kept);
4. atomically rename the best candidate to ``model-dir/<ts>`` and delete the rest;
5. publish ``MODEL`` (inline PMML when <= ``oryx.update-topic.message.max-size``) or
   ``MODEL-REF`` (path), then optional additional model data (e.g. ALS factor rows).

Data is a :class:`~oryx_amd.api.Dataset` of (key, message) pairs; apps see message lists.
GPU candidates run concurrently on one device from separate threads (the device queue
serialises them); on several ranks with ``oryx.ml.eval.parallelism`` > 1 the ranks split into
disjoint process groups that train different candidates at once (``_run_update_grouped``),
otherwise candidates run one after another across all ranks.

Sharded apps (``sharded_data = True``) on several ranks: each rank holds only its share of the
data; every rank runs the whole candidate loop (split, build, evaluate -- the apps' collective
versions, so every rank gets the same eval and picks the same winner), rank 0 writes the
candidate files, promotes the winner and sends ``MODEL``, and every rank publishes its own
share of the additional model data (the reference publishes per partition from executors).
"""

from __future__ import annotations

import abc
import json
import logging
import os
import time
from typing import Any, List, Optional, Sequence, Tuple

import numpy as np

from ..api import BatchLayerUpdate, Dataset, TopicProducer
from ..textlines import LineSelection, TextLines, concat_lines
from .. import tracing
from ..parallel import dist
from ..utils import ioutils, lang, pmml as pmmlu, rng
from . import hyperparams as hp

__all__ = ["MLUpdate", "MODEL_FILE_NAME"]

log = logging.getLogger(__name__)

MODEL_FILE_NAME = "model.pmml"
TIMINGS_FILE_NAME = "timings.json"


def _with_dist(context, ctx: dist.DistContext):
    """``context`` with its distributed context replaced by ``ctx`` (a subgroup)."""
    if context is None or isinstance(context, dist.DistContext):
        return ctx
    if hasattr(context, "dist"):
        import copy
        c = copy.copy(context)
        c.dist = ctx
        return c
    return ctx


class MLUpdate(BatchLayerUpdate):
    # True when build_model / evaluate / publish_additional_model_data accept this rank's share
    # of the data and do their own cross-rank exchanges
    sharded_data = False

    def __init__(self, config):
        self.config = config
        self.dist_ctx = None
        self.promoted_from: Optional[str] = None
        self.test_fraction = config.get_double("oryx.ml.eval.test-fraction")
        candidates = config.get_int("oryx.ml.eval.candidates")
        self.eval_parallelism = config.get_int("oryx.ml.eval.parallelism")
        self.max_message_size = config.get_int("oryx.update-topic.message.max-size")
        if not (0.0 <= self.test_fraction <= 1.0):
            raise ValueError("test-fraction must be in [0,1]")
        if candidates <= 0 or self.eval_parallelism <= 0 or self.max_message_size <= 0:
            raise ValueError("candidates, parallelism and max-size must be > 0")
        if self.test_fraction == 0.0 and candidates > 1:
            log.info("Eval is disabled (test fraction = 0) so candidates is overridden to 1")
            candidates = 1
        self.candidates = candidates

    # ---------------------------------------------------------------- app hooks
    def get_test_fraction(self) -> float:
        return self.test_fraction

    def get_hyper_parameter_values(self) -> List[hp.HyperParamValues]:
        return []

    @abc.abstractmethod
    def build_model(self, context, train_data: List[str], hyper_parameters: List[Any],
                    candidate_path: str) -> Optional[pmmlu.PMMLDoc]: ...

    @abc.abstractmethod
    def evaluate(self, context, model: pmmlu.PMMLDoc, model_parent_path: str,
                 test_data: List[str], train_data: List[str]) -> float: ...

    def can_publish_additional_model_data(self) -> bool:
        return False

    def publish_additional_model_data(self, context, pmml: pmmlu.PMMLDoc, new_data: List[str],
                                      past_data: Optional[List[str]], model_parent_path: str,
                                      model_update_topic: TopicProducer) -> None:
        pass

    def split_new_data_to_train_test(self, new_data: List[str]
                                     ) -> Tuple[List[str], List[str]]:
        """Default: random split with probability ``test_fraction`` per datum."""
        gen = rng.get_random().generator
        mask = gen.random(len(new_data)) < self.test_fraction
        if isinstance(new_data, TextLines) and not isinstance(new_data, LineSelection):
            # lazy selections: no text is copied unless a consumer asks for the bytes (the
            # feature apps' parser selects parsed rows instead, models/features.py)
            return (LineSelection(new_data, np.flatnonzero(~mask)),
                    LineSelection(new_data, np.flatnonzero(mask)))
        if isinstance(new_data, TextLines):
            return new_data.take(~mask), new_data.take(mask)
        train = [d for d, m in zip(new_data, mask) if not m]
        test = [d for d, m in zip(new_data, mask) if m]
        return train, test

    # ---------------------------------------------------------------- driver
    def run_update(self, context, timestamp: int, new_data: Dataset,
                   past_data: Optional[Dataset], model_dir: str,
                   model_update_topic: Optional[TopicProducer]) -> None:
        try:
            self._run_update(context, timestamp, new_data, past_data, model_dir,
                             model_update_topic)
        finally:
            # files an app writes in the background (ALS factor parts) are complete before
            # the generation ends, whatever path it took
            join = getattr(self, "join_files", None)
            if join is not None:
                join()

    def _run_update(self, context, timestamp: int, new_data: Dataset,
                    past_data: Optional[Dataset], model_dir: str,
                    model_update_topic: Optional[TopicProducer]) -> None:
        if new_data is None:
            raise ValueError("new_data is required")
        # candidate path -> (PMML document, its serialized text) of the models this process
        # wrote this generation: the winner is published from memory, not re-read and
        # re-serialized (a rank-64 model's PMML lists every user and item ID)
        self._written = {}
        new_msgs = new_data.values()
        past_msgs = past_data.values() if past_data is not None else None

        values = self.get_hyper_parameter_values()
        per_param = hp.choose_values_per_hyper_param(len(values), self.candidates)
        combos = hp.choose_hyper_parameter_combos(values, self.candidates, per_param)
        dctx = self._dist_ctx(context)
        self.dist_ctx = dctx
        # trainers that checkpoint or warm-start find their files under the model dir
        self.current_model_dir = ioutils.to_local_path(model_dir) if model_dir else None
        n_groups = min(self.eval_parallelism, self.candidates, dctx.world_size)
        if dctx.is_distributed and n_groups > 1:
            self._run_update_grouped(context, new_msgs, past_msgs, combos, model_dir,
                                     model_update_topic, dctx, n_groups)
            return
        if dctx.is_distributed and self.sharded_data:
            self._run_update_sharded(context, new_msgs, past_msgs, combos, model_dir,
                                     model_update_topic, dctx)
            return
        # multi-rank: every candidate runs in its own shared-seed scope so all ranks make the
        # same splits whatever rank 0 does in between (evaluation, publishing)
        self._candidate_seed_base = rng.next_seed() if dctx.is_distributed else None
        if dctx.is_distributed and not dctx.is_main:
            for i in range(self.candidates):
                with rng.shared_seed_scope(self._candidate_seed_base + i):
                    train, _ = self._split_train_test(new_msgs, past_msgs)
                    if train:
                        self.build_model(context, train, combos[i % len(combos)], None)
            return

        model_dir_local = ioutils.to_local_path(model_dir)
        candidates_path = os.path.join(model_dir_local, ".temporary",
                                       str(int(time.time() * 1000)))
        os.makedirs(candidates_path, exist_ok=True)
        best = self._find_best_candidate_path(context, new_msgs, past_msgs, combos,
                                              candidates_path)
        final_path = os.path.join(model_dir_local, str(int(time.time() * 1000)))
        # apps may keep what they built in memory, keyed by candidate path
        self.promoted_from = best
        if best is None:
            log.info("Unable to build any model")
        else:
            os.replace(best, final_path)
        ioutils.delete_recursively(candidates_path)

        if model_update_topic is None:
            log.info("No update topic configured, not publishing models to a topic")
            return
        self._publish_final(context, final_path, new_msgs, past_msgs, model_update_topic)

    def _run_update_sharded(self, context, new_msgs, past_msgs, combos, model_dir,
                            model_update_topic, dctx) -> None:
        main = dctx.is_main
        model_dir_local = ioutils.to_local_path(model_dir)
        stamp = dist.broadcast_object(int(time.time() * 1000) if main else None, dctx)
        candidates_path = os.path.join(model_dir_local, ".temporary", str(stamp))
        if main:
            os.makedirs(candidates_path, exist_ok=True)
        results = [self._build_and_eval(i, combos, context, new_msgs, past_msgs,
                                        candidates_path) for i in range(self.candidates)]
        self._promote_and_publish(context, results, new_msgs, past_msgs, model_dir_local,
                                  candidates_path, stamp, model_update_topic, dctx)

    def _pick_best(self, results) -> Optional[int]:
        best_i, best_eval = None, float("-inf")
        for i, (path, ev) in enumerate(results):
            if path is None:
                continue
            if ev == ev:
                if ev > best_eval:
                    best_eval, best_i = ev, i
            elif best_i is None and self.test_fraction == 0.0:
                best_i = i
        return best_i

    def _run_update_grouped(self, context, new_msgs, past_msgs, combos, model_dir,
                            model_update_topic, dctx, n_groups) -> None:
        """Candidate parallelism across GPUs (``MLUpdate.java:251-261`` runs candidates with
        ``collectInParallel``): the ranks split into ``n_groups`` disjoint process groups and
        group g builds and evaluates candidates g, g + G, ... with its own collectives, so
        G candidates train at once on disjoint GPUs.  Sharded apps first replicate the data
        into every group (member m of each group receives the shares of the ranks r with
        r mod group-size == m).  Each group's first rank writes its candidates' files; the
        (path, eval) results are exchanged over the control plane and every rank picks the
        same winner, which is promoted and published as in the single-group flow."""
        g, sub = dist.split_groups(dctx, n_groups)
        G = dctx.world_size // sub.world_size
        model_dir_local = ioutils.to_local_path(model_dir)
        stamp = dist.broadcast_object(int(time.time() * 1000) if dctx.is_main else None, dctx)
        seed_base = dist.broadcast_object(rng.next_seed() if dctx.is_main else None, dctx)
        candidates_path = os.path.join(model_dir_local, ".temporary", str(stamp))
        if dctx.is_main:
            os.makedirs(candidates_path, exist_ok=True)
        dist.barrier(dctx)
        if self.sharded_data:
            from ..parallel import shuffle
            my_new = shuffle.replicate_to_groups(list(new_msgs), dctx, sub.world_size)
            my_past = shuffle.replicate_to_groups(list(past_msgs), dctx, sub.world_size) \
                if past_msgs is not None else None
        else:
            my_new, my_past = new_msgs, past_msgs
        sub_context = _with_dist(context, sub)
        self.dist_ctx = sub
        mine = {}
        try:
            for i in range(g, self.candidates, G):
                with rng.shared_seed_scope(seed_base + i):
                    if self.sharded_data or sub.is_main or not sub.is_distributed:
                        mine[i] = self._build_and_eval_inner(i, combos, sub_context, my_new,
                                                             my_past, candidates_path)
                    else:
                        # non-sharded followers only join the group's collective build
                        train, _ = self._split_train_test(my_new, my_past)
                        if train:
                            self.build_model(sub_context, train, combos[i % len(combos)], None)
        finally:
            self.dist_ctx = dctx
        reported = mine if sub.is_main else {}
        gathered = [None] * dctx.world_size
        import torch.distributed as tdist
        tdist.all_gather_object(gathered, reported, group=dctx.control)
        merged = {}
        for d in gathered:
            merged.update(d or {})
        results = [merged.get(i, (None, float("nan"))) for i in range(self.candidates)]
        log.info("Candidate results over %d groups: %s", G, [ev for _, ev in results])
        if self.sharded_data:
            self._promote_and_publish(context, results, new_msgs, past_msgs, model_dir_local,
                                      candidates_path, stamp, model_update_topic, dctx)
            return
        # non-sharded apps publish from rank 0 with its full copy of the data
        best_i = self._pick_best(results)
        final_path = os.path.join(model_dir_local, str(stamp + 1))
        self.promoted_from = results[best_i][0] if best_i is not None else None
        if dctx.is_main:
            if best_i is None:
                log.info("Unable to build any model")
            else:
                os.replace(results[best_i][0], final_path)
            ioutils.delete_recursively(candidates_path)
        dist.barrier(dctx)
        if not dctx.is_main or best_i is None:
            return
        if model_update_topic is None:
            log.info("No update topic configured, not publishing models to a topic")
            return
        self._publish_final(context, final_path, new_msgs, past_msgs, model_update_topic)

    def _publish_final(self, context, final_path, new_msgs, past_msgs, model_update_topic):
        best_model_path = os.path.join(final_path, MODEL_FILE_NAME)
        if not os.path.exists(best_model_path):
            return
        t_p = time.perf_counter()
        needed = self.can_publish_additional_model_data()
        not_too_large = os.path.getsize(best_model_path) <= self.max_message_size
        best_model = text = None
        if needed or not_too_large:
            best_model, text = self._promoted_model(best_model_path)
        if not_too_large:
            model_update_topic.send("MODEL", text)
        else:
            model_update_topic.send("MODEL-REF", ioutils.to_uri(best_model_path))
        self._phase("model_publish", time.perf_counter() - t_p)
        if needed:
            self.publish_additional_model_data(context, best_model, new_msgs, past_msgs,
                                               final_path, model_update_topic)

    def _promote_and_publish(self, context, results, new_msgs, past_msgs, model_dir_local,
                             candidates_path, stamp, model_update_topic, dctx) -> None:
        """Sharded flow after the candidates: rank 0 promotes the winner and sends ``MODEL``;
        every rank publishes its share of the additional model data."""
        main = dctx.is_main
        best_i = self._pick_best(results)
        final_path = os.path.join(model_dir_local, str(stamp + 1))
        self.promoted_from = results[best_i][0] if best_i is not None else None
        if main:
            if best_i is None:
                log.info("Unable to build any model")
            else:
                os.replace(results[best_i][0], final_path)
            ioutils.delete_recursively(candidates_path)
        dist.barrier(dctx)
        if model_update_topic is None or best_i is None:
            if model_update_topic is None:
                log.info("No update topic configured, not publishing models to a topic")
            return
        best_model_path = os.path.join(final_path, MODEL_FILE_NAME)
        # the PMML (with every ID of the model) is parsed only where it is needed: rank 0 sends
        # it, the others only when the app publishes from it
        t_p = time.perf_counter()
        best_model, text = self._promoted_model(best_model_path) \
            if main or self.publish_needs_model() else (None, None)
        if main:
            if os.path.getsize(best_model_path) <= self.max_message_size:
                model_update_topic.send("MODEL", text)
            else:
                model_update_topic.send("MODEL-REF", ioutils.to_uri(best_model_path))
        self._phase("model_publish", time.perf_counter() - t_p)
        dist.barrier(dctx)
        if self.can_publish_additional_model_data():
            self.publish_additional_model_data(context, best_model, new_msgs, past_msgs,
                                               final_path, model_update_topic)

    def _global_count(self, n: int) -> int:
        d = self.dist_ctx
        if d is None or not d.is_distributed or not self.sharded_data:
            return n
        from ..parallel import shuffle
        return int(sum(shuffle.all_gather_int(n, d)))

    @staticmethod
    def _dist_ctx(context):
        c = context if isinstance(context, dist.DistContext) else getattr(context, "dist", None)
        return c if c is not None else dist.get_context()

    def _find_best_candidate_path(self, context, new_msgs, past_msgs, combos,
                                  candidates_path) -> Optional[str]:
        # collective-using trainers must not interleave across candidates on multiple ranks
        par = 1 if self._dist_ctx(context).is_distributed else \
            min(self.eval_parallelism, self.candidates)
        results = lang.collect_in_parallel(
            self.candidates,
            lambda i: self._build_and_eval(i, combos, context, new_msgs, past_msgs,
                                           candidates_path), par)
        best_path, best_eval = None, float("-inf")
        for path, ev in results:
            if path is None or not os.path.exists(path):
                continue
            if ev == ev:  # not NaN
                if ev > best_eval:
                    log.info("Best eval / model path is now %s / %s", ev, path)
                    best_eval, best_path = ev, path
            elif best_path is None and self.test_fraction == 0.0:
                best_path = path
        return best_path

    def _build_and_eval(self, i, combos, context, new_msgs, past_msgs, candidates_path):
        base = getattr(self, "_candidate_seed_base", None)
        if base is not None:
            with rng.shared_seed_scope(base + i):
                return self._build_and_eval_inner(i, combos, context, new_msgs, past_msgs,
                                                  candidates_path)
        return self._build_and_eval_inner(i, combos, context, new_msgs, past_msgs,
                                          candidates_path)

    def _build_and_eval_inner(self, i, combos, context, new_msgs, past_msgs, candidates_path):
        params = combos[i % len(combos)]
        candidate_path = os.path.join(candidates_path, str(i))
        log.info("Building candidate %d with params %s", i, params)
        t_split = time.perf_counter()
        train, test = self._split_train_test(new_msgs, past_msgs)
        self._phase("split", time.perf_counter() - t_split)
        ev = float("nan")
        n_train, n_test = self._global_count(len(train)), self._global_count(len(test))
        timing = {"candidate": i, "params": [str(p) for p in params], "train": n_train,
                  "test": n_test}
        # sharded: every rank builds / evaluates (collectives), rank 0 writes the files
        writer = not (self.sharded_data and self.dist_ctx is not None and
                      self.dist_ctx.is_distributed and not self.dist_ctx.is_main)
        if not n_train:
            log.info("No train data to build a model")
        else:
            t0 = time.perf_counter()
            with tracing.range("mlupdate.build"):
                model = self.build_model(context, train, params, candidate_path)
            timing["build_s"] = time.perf_counter() - t0
            if model is None:
                log.info("Unable to build a model")
                if not writer:
                    return None, ev
            else:
                if writer:
                    t_w = time.perf_counter()
                    os.makedirs(candidate_path, exist_ok=True)
                    model_path = os.path.join(candidate_path, MODEL_FILE_NAME)
                    log.info("Writing model to %s", model_path)
                    text = pmmlu.to_string(model)
                    ioutils.write_text(model_path, text)
                    self._written[candidate_path] = (model, text)
                    self._phase("pmml_write", time.perf_counter() - t_w)
                if not n_test:
                    log.info("No test data available to evaluate model")
                else:
                    log.info("Evaluating model")
                    t1 = time.perf_counter()
                    with tracing.range("mlupdate.evaluate"):
                        ev = float(self.evaluate(context, model, candidate_path, test, train))
                    timing["evaluate_s"] = time.perf_counter() - t1
                timing.update(self.build_timings(candidate_path))
                # per-candidate timing record next to the model (moves with the winner)
                if writer:
                    with open(os.path.join(candidate_path, TIMINGS_FILE_NAME), "w") as f:
                        json.dump(dict(timing, eval=ev if ev == ev else None), f)
        timing["eval"] = ev if ev == ev else None
        # the candidate's train / test buffers (the whole interval's text for the apps that
        # parse on the device) are freed here, as a phase of their own
        t_r = time.perf_counter()
        del train, test
        self._phase("release", time.perf_counter() - t_r)
        tracing.record(dict(timing, event="candidate"))
        log.info("Model eval for params %s: %s (%s)", params, ev, candidate_path)
        return candidate_path, ev

    def _phase(self, name: str, seconds: float) -> None:
        """Add to the app's ``phase_seconds`` (when it keeps one: bench_batch reads it)."""
        ph = getattr(self, "phase_seconds", None)
        if isinstance(ph, dict):
            ph[name] = ph.get(name, 0.0) + seconds

    def _promoted_model(self, path: str):
        """(PMML document, serialized text) of the promoted model at ``path``: from memory
        when this process wrote it, else read from the file."""
        got = getattr(self, "_written", {}).get(getattr(self, "promoted_from", None))
        if got is not None:
            return got
        text = ioutils.read_text(path)
        return pmmlu.from_string(text), text

    def publish_needs_model(self) -> bool:
        """Whether :meth:`publish_additional_model_data` on a non-zero rank of a sharded
        generation reads the promoted model (the PMML); apps that publish from what each rank
        built return False so those ranks skip parsing it."""
        return True

    def build_timings(self, candidate_path: str) -> dict:
        """App-specific timing details of the last build (e.g. ALS iteration ms, ratings/s)."""
        return {}

    def _split_train_test(self, new_msgs, past_msgs):
        # TextLines buffers stay buffers (concat_lines / the apps' native splits)
        if self.test_fraction <= 0.0:
            return concat_lines([new_msgs, past_msgs]), []
        if self.test_fraction >= 1.0:
            return concat_lines([past_msgs]), new_msgs
        if not new_msgs:
            return list(past_msgs or []), []
        train, test = self.split_new_data_to_train_test(new_msgs)
        return concat_lines([train, past_msgs]), test
