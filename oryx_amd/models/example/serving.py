"""Example app: serving model and manager
(``[example]/serving/ExampleServingModel.java``, ``ExampleServingModelManager.java:36-75``)."""

from __future__ import annotations

import json
import threading
from typing import Dict

from ...api import AbstractServingModelManager, ServingModel

__all__ = ["ExampleServingModel", "ExampleServingModelManager"]


class ExampleServingModel(ServingModel):
    def __init__(self, words: Dict[str, int]):
        self._words = words

    def get_fraction_loaded(self) -> float:
        return 1.0

    def get_words(self) -> Dict[str, int]:
        return self._words


class ExampleServingModelManager(AbstractServingModelManager):
    def __init__(self, config):
        super().__init__(config)
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
                word, count = km.message.split(",")[:2]
                with self._lock:
                    self.distinct_other_words[word] = int(count)
            else:
                raise ValueError("Unknown key " + str(km.key))

    def get_model(self) -> ExampleServingModel:
        return ExampleServingModel(self.distinct_other_words)
