"""Hyperparameter value generators and combination search.

Behavior of ``HyperParams`` and its value classes (``[ml]/param/HyperParams.java:32-193``,
``ContinuousRange.java:37-57``, ``DiscreteRange.java:37-65``, ``ContinuousAround.java:36-53``,
``DiscreteAround.java:36-49``, ``Unordered.java:36-40``):

* config values: a number -> fixed; a 2-element numeric list -> range; strings -> unordered;
* ``choose_values_per_hyper_param``: smallest v with v^numParams >= candidates;
* ``choose_hyper_parameter_combos``: the full grid (<= 65536 combos), shuffled; when fewer
  candidates than combos are wanted, a random subset.

Deliberate fix: the reference draws a random permutation but
then takes the *first* ``howMany`` combinations; here the permutation is actually used.
"""

from __future__ import annotations

import abc
import math
from typing import Any, List, Sequence

from ..utils import rng

__all__ = ["HyperParamValues", "ContinuousRange", "DiscreteRange", "ContinuousAround",
           "DiscreteAround", "Unordered", "fixed", "range_of", "around", "unordered_from_values",
           "from_config", "choose_hyper_parameter_combos", "choose_values_per_hyper_param",
           "MAX_COMBOS"]

MAX_COMBOS = 65536


def _java_round(x: float) -> int:
    return int(math.floor(x + 0.5))


class HyperParamValues(abc.ABC):
    @abc.abstractmethod
    def get_trial_values(self, num: int) -> List[Any]: ...

    def __repr__(self):
        return "%s[...%s...]" % (type(self).__name__, self.get_trial_values(3))


class ContinuousRange(HyperParamValues):
    def __init__(self, lo: float, hi: float):
        if lo > hi:
            raise ValueError("min > max")
        self.min, self.max = float(lo), float(hi)

    def get_trial_values(self, num: int) -> List[float]:
        if num <= 0:
            raise ValueError("num must be > 0")
        if self.max == self.min:
            return [self.min]
        if num == 1:
            return [(self.max + self.min) / 2.0]
        if num == 2:
            return [self.min, self.max]
        diff = (self.max - self.min) / (num - 1.0)
        vals = [self.min]
        for _ in range(1, num - 1):
            vals.append(vals[-1] + diff)
        vals.append(self.max)
        return vals


class DiscreteRange(HyperParamValues):
    def __init__(self, lo: int, hi: int):
        if lo > hi:
            raise ValueError("min > max")
        self.min, self.max = int(lo), int(hi)

    def get_trial_values(self, num: int) -> List[int]:
        if num <= 0:
            raise ValueError("num must be > 0")
        if self.max == self.min:
            return [self.min]
        if num == 1:
            return [(self.max + self.min) // 2 if (self.max + self.min) >= 0
                    else -((-(self.max + self.min)) // 2)]
        if num == 2:
            return [self.min, self.max]
        if num > (self.max - self.min):
            return list(range(self.min, self.max + 1))
        diff = (self.max - self.min) / (num - 1.0)
        vals = [self.min]
        for _ in range(1, num - 1):
            vals.append(_java_round(vals[-1] + diff))
        vals.append(self.max)
        return vals


class ContinuousAround(HyperParamValues):
    def __init__(self, around_value: float, step: float):
        if step <= 0:
            raise ValueError("step must be > 0")
        self.around, self.step = float(around_value), float(step)

    def get_trial_values(self, num: int) -> List[float]:
        if num <= 0:
            raise ValueError("num must be > 0")
        if num == 1:
            return [self.around]
        value = self.around - ((num - 1.0) / 2.0) * self.step
        vals = []
        for _ in range(num):
            vals.append(value)
            value += self.step
        if num % 2 != 0:
            vals[num // 2] = self.around
        return vals


class DiscreteAround(HyperParamValues):
    def __init__(self, around_value: int, step: int):
        if step <= 0:
            raise ValueError("step must be > 0")
        self.around, self.step = int(around_value), int(step)

    def get_trial_values(self, num: int) -> List[int]:
        if num <= 0:
            raise ValueError("num must be > 0")
        if num == 1:
            return [self.around]
        # Java int division truncates toward zero
        half = (num - 1) * self.step
        value = self.around - int(half / 2)
        vals = []
        for _ in range(num):
            vals.append(value)
            value += self.step
        return vals


class Unordered(HyperParamValues):
    def __init__(self, values: Sequence[Any]):
        values = list(values)
        if not values:
            raise ValueError("no values")
        self.values = values

    def get_trial_values(self, num: int) -> List[Any]:
        if num <= 0:
            raise ValueError("num must be > 0")
        return self.values[:num] if num < len(self.values) else list(self.values)


def fixed(value):
    if isinstance(value, int) and not isinstance(value, bool):
        return DiscreteRange(value, value)
    return ContinuousRange(float(value), float(value))


def range_of(lo, hi):
    if isinstance(lo, int) and isinstance(hi, int):
        return DiscreteRange(lo, hi)
    return ContinuousRange(float(lo), float(hi))


def around(value, step):
    if isinstance(value, int) and isinstance(step, int):
        return DiscreteAround(value, step)
    return ContinuousAround(float(value), float(step))


def unordered_from_values(values):
    return Unordered(values)


def _parse_int(s: str):
    s = s.strip()
    if s and (s.isdigit() or (s[0] in "+-" and s[1:].isdigit())):
        return int(s)
    raise ValueError(s)


def from_config(config, key: str) -> HyperParamValues:
    v = config.get_value(key)
    if isinstance(v, list):
        strs = config.get_string_list(key)
        try:
            return range_of(_parse_int(strs[0]), _parse_int(strs[1]))
        except (ValueError, IndexError):
            pass
        try:
            return range_of(float(strs[0]), float(strs[1]))
        except (ValueError, IndexError):
            pass
        return unordered_from_values(strs)
    s = config.get_string(key)
    try:
        return fixed(_parse_int(s))
    except ValueError:
        pass
    try:
        return fixed(float(s))
    except ValueError:
        pass
    return unordered_from_values([s])


def choose_hyper_parameter_combos(ranges: Sequence[HyperParamValues], how_many: int,
                                  per_param: int) -> List[List[Any]]:
    if how_many <= 0:
        raise ValueError("how_many must be > 0")
    if per_param < 0:
        raise ValueError("per_param must be >= 0")
    num_params = len(ranges)
    if num_params == 0 or per_param == 0:
        return [[]]
    if per_param ** num_params > MAX_COMBOS:
        raise ValueError("too many combinations")
    param_ranges = [r.get_trial_values(per_param) for r in ranges]
    how_many_combos = 1
    for vals in param_ranges:
        how_many_combos *= len(vals)
    all_combos = []
    for combo in range(how_many_combos):
        combination = []
        for p in range(num_params):
            which = combo
            for i in range(p):
                which //= len(param_ranges[i])
            which %= len(param_ranges[p])
            combination.append(param_ranges[p][which])
        all_combos.append(combination)
    gen = rng.get_random().generator
    if how_many >= how_many_combos:
        order = gen.permutation(how_many_combos)
        return [all_combos[i] for i in order]
    indices = gen.permutation(how_many_combos)[:how_many]
    result = [all_combos[i] for i in indices]
    gen.shuffle(result)
    return result


def choose_values_per_hyper_param(num_params: int, candidates: int) -> int:
    if num_params < 1:
        return 0
    v = 0
    while True:
        v += 1
        if v ** num_params >= candidates:
            return v
