"""Public API for app authors (the reference's ``framework/oryx-api``).

Interfaces mirror ``[api]``:

* :class:`KeyMessage` (``[api]/KeyMessage.java:28``, ``KeyMessageImpl.java:27-70``)
* :class:`TopicProducer` (``[api]/TopicProducer.java:29-56``)
* :class:`BatchLayerUpdate` (``[api]/batch/BatchLayerUpdate.java:38-59``)
* :class:`SpeedModelManager`, :class:`SpeedModel` (``[api]/speed/SpeedModelManager.java:37-67``,
  ``[api]/speed/SpeedModel.java:23-30``)
* :class:`ServingModelManager`, :class:`AbstractServingModelManager`, :class:`ServingModel`
  (``[api]/serving/ServingModelManager.java:35-75``,
  ``[api]/serving/AbstractServingModelManager.java:26-48``, ``[api]/serving/ServingModel.java:23-30``)
* :class:`OryxServingException` (``[api]/serving/OryxServingException.java:26-55``)
* :class:`HasCSV` (``[api]/serving/HasCSV.java:25``)

Data handed to batch updates is a :class:`Dataset` of (key, message) string pairs (the RDD
equivalent).  The Scala adapter classes of the reference have no counterpart: Python classes
implement these ABCs directly.
"""

from __future__ import annotations

import abc
import collections.abc
from dataclasses import dataclass
from typing import Any, Generic, Iterable, Iterator, List, Optional, Sequence, Tuple, TypeVar

K = TypeVar("K")
M = TypeVar("M")
U = TypeVar("U")

__all__ = ["KeyMessage", "MessageBlock", "TopicProducer", "BatchLayerUpdate",
           "SpeedModelManager", "SpeedModel", "ServingModelManager", "AbstractServingModelManager", "ServingModel",
           "OryxServingException", "HasCSV", "Dataset"]


@dataclass(frozen=True)
class KeyMessage(Generic[K, M]):
    key: Optional[K]
    message: M

    def get_key(self):
        return self.key

    def get_message(self):
        return self.message


class MessageBlock(collections.abc.Sequence):
    """A run of text messages held as one byte buffer plus end offsets (what the native /
    GPU formatters produce) -- a read-only sequence of ``str`` that producers can append to
    the log in one native call (:meth:`TopicProducer.send_block`) without materialising a
    Python string per message.  ``ends[j]`` is the end of message j; message j starts after
    the separator byte that follows message j - 1 (``sep`` = 1) or right at its end (0)."""

    __slots__ = ("buf", "ends", "sep", "_cache")

    def __init__(self, buf, ends, sep: int = 1):
        import numpy as _np
        self.buf = buf                       # bytes or uint8 numpy array
        self.ends = _np.asarray(ends, dtype=_np.int64)
        self.sep = int(sep)
        self._cache = None

    def starts(self):
        import numpy as _np
        if len(self.ends) == 0:
            return self.ends
        return _np.r_[0, self.ends[:-1] + self.sep]

    def lengths(self):
        return self.ends - self.starts()

    def __len__(self) -> int:
        return len(self.ends)

    def _all(self) -> List[str]:
        if self._cache is None:
            text = str(memoryview(self.buf)[:int(self.ends[-1]) if len(self.ends) else 0],
                       "utf-8")
            st = self.starts().tolist()
            self._cache = [text[a:b] for a, b in zip(st, self.ends.tolist())] \
                if text.isascii() else [bytes(memoryview(self.buf)[a:b]).decode("utf-8")
                                        for a, b in zip(st, self.ends.tolist())]
        return self._cache

    def __getitem__(self, j):
        return self._all()[j]

    def __iter__(self) -> Iterator[str]:
        return iter(self._all())

    def __eq__(self, other) -> bool:
        return list(self) == list(other) if isinstance(other, (list, tuple, MessageBlock)) \
            else NotImplemented

    def __repr__(self) -> str:
        return "MessageBlock(%d messages)" % len(self)


class TopicProducer(abc.ABC, Generic[K, M]):
    """Sends keyed messages to a topic."""

    @abc.abstractmethod
    def get_update_broker(self) -> str: ...

    @abc.abstractmethod
    def get_topic(self) -> str: ...

    @abc.abstractmethod
    def send(self, key: Optional[K], message: M) -> None: ...

    def send_many(self, pairs: Iterable[Tuple[Optional[K], M]]) -> None:
        for k, m in pairs:
            self.send(k, m)

    def send_block(self, key: Optional[K], block: "MessageBlock") -> None:
        """Send every message of ``block`` with ``key`` (in order)."""
        self.send_many((key, m) for m in block)

    def close(self) -> None:
        pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False


class Dataset:
    """An immutable, in-memory collection of (key, message) pairs for one batch interval.

    Plays the role of the reference's ``JavaPairRDD<K,M>``: batch updates receive the
    interval's new data and all past data.  Heavy numeric work happens after parsing, on
    device tensors, so a plain list is the right container here.  Data read in bulk from the
    log or from text part files has no keys: it is held as the message list alone
    (:meth:`from_values`), and pairs are only materialised if someone iterates them.
    """

    __slots__ = ("_pairs", "_values")

    def __init__(self, pairs: Iterable[Tuple[Any, Any]] = ()):
        self._pairs = list(pairs)
        self._values = None

    @classmethod
    def from_values(cls, values: List[Any]) -> "Dataset":
        """Messages with null keys (the list is kept, not copied)."""
        d = cls.__new__(cls)
        d._pairs = None
        d._values = values
        return d

    def _p(self) -> List[Tuple[Any, Any]]:
        if self._pairs is None:
            self._pairs = [(None, v) for v in self._values]
        return self._pairs

    @property
    def keyless(self) -> bool:
        """True when every key is null and the messages are held as one list."""
        return self._values is not None

    def __len__(self):
        return len(self._values) if self._values is not None else len(self._pairs)

    def __iter__(self) -> Iterator[Tuple[Any, Any]]:
        return iter(self._p())

    def __getstate__(self):
        return (self._pairs if self._values is None else None, self._values)

    def __setstate__(self, state):
        self._pairs, self._values = state

    def is_empty(self) -> bool:
        return len(self) == 0

    def count(self) -> int:
        return len(self)

    def keys(self) -> List[Any]:
        if self._values is not None:
            return [None] * len(self._values)
        return [k for k, _ in self._pairs]

    def values(self) -> List[Any]:
        if self._values is not None:
            return self._values
        return [m for _, m in self._pairs]

    def union(self, other: "Dataset") -> "Dataset":
        if self.keyless and isinstance(other, Dataset) and other.keyless:
            return Dataset.from_values(self._values + other._values)
        return Dataset(self._p() + list(other))

    def filter(self, fn) -> "Dataset":
        return Dataset(p for p in self._p() if fn(p))

    def map_values(self, fn) -> "Dataset":
        return Dataset((k, fn(m)) for k, m in self._p())

    def collect(self) -> List[Tuple[Any, Any]]:
        return list(self._p())


class BatchLayerUpdate(abc.ABC, Generic[K, M, U]):
    """Called once per batch interval with new and past data."""

    @abc.abstractmethod
    def run_update(self, context: Any, timestamp: int, new_data: Dataset,
                   past_data: Optional[Dataset], model_dir: str,
                   model_update_topic: Optional[TopicProducer]) -> None: ...


class SpeedModel(abc.ABC):
    @abc.abstractmethod
    def get_fraction_loaded(self) -> float: ...


class SpeedModelManager(abc.ABC, Generic[K, M, U]):
    """Consumes the update topic into an in-memory model; turns new input into updates."""

    @abc.abstractmethod
    def consume(self, updates: Iterator[KeyMessage], context: Any = None) -> None: ...

    @abc.abstractmethod
    def build_updates(self, new_data: Dataset) -> Iterable[U]: ...

    def close(self) -> None:
        pass


class ServingModel(abc.ABC):
    @abc.abstractmethod
    def get_fraction_loaded(self) -> float: ...


class ServingModelManager(abc.ABC, Generic[U]):
    @abc.abstractmethod
    def consume(self, updates: Iterator[KeyMessage], context: Any = None) -> None: ...

    @abc.abstractmethod
    def get_config(self): ...

    @abc.abstractmethod
    def get_model(self) -> Optional[ServingModel]: ...

    @abc.abstractmethod
    def is_read_only(self) -> bool: ...

    def close(self) -> None:
        pass


class AbstractServingModelManager(ServingModelManager[U]):
    """Stores the config and reads ``oryx.serving.api.read-only``."""

    def __init__(self, config):
        self._config = config
        self._read_only = config.get_bool("oryx.serving.api.read-only")

    def get_config(self):
        return self._config

    def is_read_only(self) -> bool:
        return self._read_only


class OryxServingException(Exception):
    """An HTTP status + message raised from a serving resource."""

    def __init__(self, status: int, message: Optional[str] = None):
        super().__init__(message or "")
        self.status = int(status)
        self.message = message

    def get_status_code(self) -> int:
        return self.status


class HasCSV(abc.ABC):
    @abc.abstractmethod
    def to_csv(self) -> str: ...
