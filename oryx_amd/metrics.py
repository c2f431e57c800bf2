"""Prometheus-style metrics registry (new; the reference has none -- SURVEY.md section 5.5).

Counters, gauges and fixed-bucket latency histograms rendered in the Prometheus text
exposition format at the serving layer's ``/metrics`` endpoint; layers record request
latencies, model size / fraction loaded, training throughput (ratings/s), fold-in latency
and collective bandwidth.
"""

from __future__ import annotations

import bisect
import threading
from typing import Dict, List, Tuple

__all__ = ["Registry", "default_registry"]

_BUCKETS = (0.0005, 0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0,
            10.0)


class _Histogram:
    def __init__(self, buckets=_BUCKETS):
        self.buckets = list(buckets)
        self.counts = [0] * (len(self.buckets) + 1)
        self.sum = 0.0
        self.n = 0

    def observe(self, v: float) -> None:
        self.counts[bisect.bisect_left(self.buckets, v)] += 1
        self.sum += v
        self.n += 1


class Registry:
    def __init__(self):
        self._lock = threading.Lock()
        self._counters: Dict[Tuple[str, Tuple], float] = {}
        self._gauges: Dict[Tuple[str, Tuple], float] = {}
        self._hist: Dict[Tuple[str, Tuple], _Histogram] = {}

    @staticmethod
    def _key(name, labels):
        return name, tuple(sorted((labels or {}).items()))

    def inc(self, name: str, value: float = 1.0, labels=None) -> None:
        k = self._key(name, labels)
        with self._lock:
            self._counters[k] = self._counters.get(k, 0.0) + value

    def set_gauge(self, name: str, value: float, labels=None) -> None:
        with self._lock:
            self._gauges[self._key(name, labels)] = float(value)

    def observe(self, name: str, value: float, labels=None) -> None:
        k = self._key(name, labels)
        with self._lock:
            h = self._hist.get(k)
            if h is None:
                h = self._hist[k] = _Histogram()
            h.observe(value)

    def observe_request(self, path: str, status: int, seconds: float) -> None:
        endpoint = "/" + path.strip("/").split("/")[0] if path else "/"
        self.observe("oryx_http_request_seconds", seconds, {"endpoint": endpoint})
        self.inc("oryx_http_requests_total", 1, {"endpoint": endpoint, "status": str(status)})

    def get(self, name: str, labels=None) -> float:
        k = self._key(name, labels)
        with self._lock:
            if k in self._counters:
                return self._counters[k]
            return self._gauges.get(k, 0.0)

    @staticmethod
    def _fmt_labels(labels: Tuple, extra: Tuple = ()) -> str:
        items = list(labels) + list(extra)
        if not items:
            return ""
        return "{" + ",".join('%s="%s"' % (k, str(v).replace('"', '\\"')) for k, v in items) + "}"

    def render(self) -> str:
        out: List[str] = []
        with self._lock:
            for (name, labels), v in sorted(self._counters.items()):
                out.append("%s%s %r" % (name, self._fmt_labels(labels), v))
            for (name, labels), v in sorted(self._gauges.items()):
                out.append("%s%s %r" % (name, self._fmt_labels(labels), v))
            for (name, labels), h in sorted(self._hist.items()):
                cum = 0
                for b, c in zip(h.buckets + [float("inf")], h.counts):
                    cum += c
                    le = "+Inf" if b == float("inf") else repr(b)
                    out.append("%s_bucket%s %d" % (name, self._fmt_labels(labels, (("le", le),)),
                                                   cum))
                out.append("%s_sum%s %r" % (name, self._fmt_labels(labels), h.sum))
                out.append("%s_count%s %d" % (name, self._fmt_labels(labels), h.n))
        return "\n".join(out) + "\n"


_default = Registry()


def default_registry() -> Registry:
    return _default
