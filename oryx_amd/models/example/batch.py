"""Example app (word co-occurrence): batch layer.

Equivalent of ``ExampleBatchLayerUpdate`` (``[example]/batch/ExampleBatchLayerUpdate.java:39-70``):
for every word, the number of DISTINCT other words it has appeared with on a line (lines split
on single spaces), over all new + past data; published as ``MODEL`` = that JSON map.
"""

from __future__ import annotations

import json
from typing import Dict, Iterable, Set

from ...api import BatchLayerUpdate

__all__ = ["ExampleBatchLayerUpdate", "count_distinct_other_words"]


def count_distinct_other_words(lines: Iterable[str]) -> Dict[str, int]:
    others: Dict[str, Set[str]] = {}
    for line in lines:
        toks = set(line.split(" "))
        if len(toks) < 2:
            continue
        for a in toks:
            s = others.setdefault(a, set())
            s.update(toks)
            s.discard(a)
    return {w: len(s) for w, s in others.items() if s}


class ExampleBatchLayerUpdate(BatchLayerUpdate):
    def __init__(self, config=None):
        self.config = config

    def run_update(self, context, timestamp, new_data, past_data, model_dir, model_update_topic):
        lines = list(new_data.values())
        if past_data is not None:
            lines += list(past_data.values())
        model = count_distinct_other_words(lines)
        if model_update_topic is not None:
            model_update_topic.send("MODEL", json.dumps(model, separators=(",", ":")))
