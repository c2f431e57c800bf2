"""RNG management with a global deterministic test mode.

``RandomManager`` (``[common]/random/RandomManager.java:29-98``): every generator handed out
is tracked; :func:`use_test_seed` reseeds all live and future generators to a fixed seed
(``ORYX_TEST_SEED`` env var, default 1234567890123456789) so tests are deterministic.
Generators are numpy PCG64 (the reference used Well19937c; exact streams are not shared).
Torch generators on devices are seeded through :func:`torch_generator`.
"""

from __future__ import annotations

import os
import threading
import weakref
from typing import Optional

import numpy as np

__all__ = ["get_random", "get_random_seeded", "use_test_seed", "is_test_seed", "test_seed",
           "torch_generator", "next_seed", "shared_seed_scope"]


def _parse_seed() -> int:
    s = os.environ.get("ORYX_TEST_SEED", "1234567890123456789")
    try:
        return int(s)
    except ValueError:
        return int(s, 16)


_TEST_SEED = _parse_seed() & ((1 << 63) - 1)
_lock = threading.Lock()
_instances: "weakref.WeakSet" = weakref.WeakSet()
_use_test_seed = False


class _TrackedGenerator(np.random.Generator):
    """A Generator whose bit generator can be swapped for a test-seeded one."""


def _new_gen(seed: Optional[int]) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64(seed))


class RandomGenerator:
    """Thin wrapper so reseeding replaces the underlying generator in place."""

    __slots__ = ("_gen", "__weakref__")

    def __init__(self, seed: Optional[int] = None):
        self._gen = _new_gen(seed)

    def set_seed(self, seed: int) -> None:
        self._gen = _new_gen(seed)

    def __getattr__(self, name):
        return getattr(self._gen, name)

    # Java-ish helpers used across the framework
    def next_int(self, n: int) -> int:
        return int(self._gen.integers(0, n))

    def next_double(self) -> float:
        return float(self._gen.random())

    def next_gaussian(self) -> float:
        return float(self._gen.standard_normal())

    def next_long(self) -> int:
        return int(self._gen.integers(-(1 << 63), (1 << 63) - 1))

    @property
    def generator(self) -> np.random.Generator:
        return self._gen


_scope = threading.local()


class shared_seed_scope:
    """Within the scope, the i-th :func:`get_random` call returns a generator seeded with
    ``hash(seed, i)`` -- so ranks that execute the same code path under the same broadcast seed
    draw identical random streams (identical train/test splits, hyperparameter combos, ...)."""

    def __init__(self, seed: int):
        self.seed = int(seed) & ((1 << 62) - 1)

    def __enter__(self):
        self._prev = getattr(_scope, "state", None)
        _scope.state = [self.seed, 0]
        return self

    def __exit__(self, *exc):
        _scope.state = self._prev
        return False


def get_random() -> RandomGenerator:
    st = getattr(_scope, "state", None)
    if st is not None:
        st[1] += 1
        return RandomGenerator((st[0] * 1000003 + st[1]) & ((1 << 64) - 1))
    if _use_test_seed:
        return RandomGenerator(_TEST_SEED)
    r = RandomGenerator()
    with _lock:
        _instances.add(r)
    return r


def get_random_seeded(seed: int) -> RandomGenerator:
    return RandomGenerator(seed & ((1 << 64) - 1))


def use_test_seed() -> None:
    global _use_test_seed
    _use_test_seed = True
    with _lock:
        for r in list(_instances):
            r.set_seed(_TEST_SEED)
        _instances.clear()


def is_test_seed() -> bool:
    return _use_test_seed


def test_seed() -> int:
    return _TEST_SEED


def next_seed(r: Optional[RandomGenerator] = None) -> int:
    r = r or get_random()
    return int(r.generator.integers(0, (1 << 62)))


def torch_generator(device="cpu", seed: Optional[int] = None):
    import torch
    g = torch.Generator(device=device)
    if seed is None:
        seed = _TEST_SEED if _use_test_seed else next_seed()
    g.manual_seed(int(seed) & ((1 << 63) - 1))
    return g
