"""Example app: speed layer (``[example]/speed/ExampleSpeedModelManager.java:38-85``).

``MODEL`` replaces the word -> count map (keeping only its keys); ``buildUpdates`` counts the
interval's distinct co-occurring words and adds them to the current counts, emitting
``word,newCount`` lines.
"""

from __future__ import annotations

import json
import threading
from typing import Dict, List

from ...api import SpeedModelManager
from .batch import count_distinct_other_words

__all__ = ["ExampleSpeedModelManager"]


class ExampleSpeedModelManager(SpeedModelManager):
    def __init__(self, config=None):
        self.distinct_other_words: Dict[str, int] = {}
        self._lock = threading.Lock()

    def consume(self, updates, context=None) -> None:
        for km in updates:
            if km.key == "MODEL":
                model = json.loads(km.message)
                with self._lock:
                    for w in [w for w in self.distinct_other_words if w not in model]:
                        del self.distinct_other_words[w]
                    self.distinct_other_words.update({k: int(v) for k, v in model.items()})
            elif km.key == "UP":
                continue
            else:
                raise ValueError("Unknown key " + str(km.key))

    def build_updates(self, new_data) -> List[str]:
        out = []
        for word, count in count_distinct_other_words(new_data.values()).items():
            with self._lock:
                new = self.distinct_other_words.get(word, 0) + count
                self.distinct_other_words[word] = new
            out.append("%s,%d" % (word, new))
        return out

    def close(self) -> None:
        pass
