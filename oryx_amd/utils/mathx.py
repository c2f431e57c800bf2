"""Small linear algebra on the host: vector math, rank-revealing solver, weighted mean.

* ``VectorMath`` (``[common]/math/VectorMath.java:38-108``): dot (float products accumulated in
  double), norm, transposeTimesSelf (Gramian), random Gaussian vector.
* ``LinearSystemSolver`` / ``Solver`` (``[common]/math/LinearSystemSolver.java:35-63``,
  ``[common]/math/Solver.java:33-44``): column-pivoted (rank-revealing) QR with singularity
  threshold ``1e-5 * ||M||_inf``; near-singular input raises
  :class:`SingularMatrixSolverException` with the apparent rank computed like commons-math
  ``RRQRDecomposition.getRank(0.01)``.
* ``DoubleWeightedMean`` (``[common]/math/DoubleWeightedMean.java:29-114``).

The device-side equivalents (batched Cholesky, Gramian SYRK) live in :mod:`oryx_amd.ops`.
"""

from __future__ import annotations

import logging
import math
from typing import Iterable, Optional

import numpy as np
import scipy.linalg

__all__ = ["dot", "norm", "transpose_times_self", "random_vector_f", "parse_vector",
           "Solver", "SingularMatrixSolverException", "get_solver", "is_non_singular",
           "DoubleWeightedMean", "SINGULARITY_THRESHOLD_RATIO"]

log = logging.getLogger(__name__)

SINGULARITY_THRESHOLD_RATIO = 1.0e-5


def dot(x, y) -> float:
    x = np.asarray(x, dtype=np.float32)
    y = np.asarray(y, dtype=np.float32)
    return float(np.sum((x * y).astype(np.float64)))


def norm(x) -> float:
    x = np.asarray(x, dtype=np.float32)
    return math.sqrt(float(np.sum((x * x).astype(np.float64))))


def transpose_times_self(vectors) -> Optional[np.ndarray]:
    """Gramian VᵀV of a collection/array of row vectors (float64 result); None if empty."""
    if vectors is None:
        return None
    if isinstance(vectors, np.ndarray):
        m = vectors
    else:
        vs = list(vectors)
        if not vs:
            return None
        m = np.stack([np.asarray(v, dtype=np.float32) for v in vs])
    if m.size == 0:
        return None
    m32 = m.astype(np.float32)
    # float products, double accumulation (as the reference)
    return (m32.astype(np.float64).T @ m32.astype(np.float64))


def random_vector_f(features: int, random) -> np.ndarray:
    gen = getattr(random, "generator", random)
    return gen.standard_normal(features).astype(np.float32)


def parse_vector(values) -> np.ndarray:
    return np.array([float(v) for v in values], dtype=np.float64)


class SingularMatrixSolverException(ArithmeticError):
    def __init__(self, apparent_rank: int, message: str):
        super().__init__(message)
        self.apparent_rank = apparent_rank


class Solver:
    """Solves ``M x = b`` for a fixed non-singular ``M`` via its pivoted QR factorization."""

    def __init__(self, q: np.ndarray, r: np.ndarray, perm: np.ndarray):
        self._q = q
        self._r = r
        self._perm = perm
        self._inverse: Optional[np.ndarray] = None

    def solve(self, b) -> np.ndarray:
        b = np.asarray(b, dtype=np.float64)
        y = self._q.T @ b
        z = scipy.linalg.solve_triangular(self._r, y)
        x = np.empty_like(z)
        x[self._perm] = z
        return x

    def solve_f_to_f(self, b) -> np.ndarray:
        return self.solve(np.asarray(b, dtype=np.float32).astype(np.float64)).astype(np.float32)

    def solve_d_to_d(self, b) -> np.ndarray:
        return self.solve(b)

    def inverse(self) -> np.ndarray:
        """Explicit M⁻¹ (float64), cached; used to batch fold-ins as one GEMM on device."""
        if self._inverse is None:
            n = self._r.shape[0]
            self._inverse = self.solve(np.eye(n))
        return self._inverse

    def __repr__(self):
        return "Solver[RRQR %dx%d]" % self._r.shape


def _inf_norm(m: np.ndarray) -> float:
    return float(np.max(np.sum(np.abs(m), axis=1))) if m.size else 0.0


def _rrqr(m: np.ndarray):
    q, r, p = scipy.linalg.qr(m, pivoting=True)
    return q, r, p


def _apparent_rank(r: np.ndarray, drop_threshold: float = 0.01) -> int:
    rows, cols = r.shape
    rank = 1
    last_norm = np.linalg.norm(r)
    r_norm = last_norm
    while rank < min(rows, cols):
        this_norm = np.linalg.norm(r[rank:, rank:])
        if this_norm == 0 or (this_norm / last_norm) * r_norm < drop_threshold:
            break
        last_norm = this_norm
        rank += 1
    return rank


def get_solver(m) -> Optional[Solver]:
    if m is None:
        return None
    m = np.asarray(m, dtype=np.float64)
    threshold = _inf_norm(m) * SINGULARITY_THRESHOLD_RATIO
    q, r, p = _rrqr(m)
    diag = np.abs(np.diag(r))
    if diag.size and np.all(diag > threshold):
        return Solver(q, r, p)
    rank = _apparent_rank(r, 0.01)
    log.warning("%d x %d matrix is near-singular (threshold %s). Add more data or decrease the "
                "number of features, to <= about %d", m.shape[0], m.shape[1], threshold, rank)
    raise SingularMatrixSolverException(rank, "Apparent rank: %d" % rank)


def is_non_singular(m) -> bool:
    m = np.asarray(m, dtype=np.float64)
    threshold = _inf_norm(m) * SINGULARITY_THRESHOLD_RATIO
    _, r, _ = _rrqr(m)
    diag = np.abs(np.diag(r))
    return bool(diag.size and np.all(diag > threshold))


class DoubleWeightedMean:
    """Running weighted mean; ``mean += (w / W) * (x - mean)``."""

    __slots__ = ("count", "total_weight", "mean")

    def __init__(self, count: int = 0, total_weight: float = 0.0, mean: float = float("nan")):
        self.count = count
        self.total_weight = total_weight
        self.mean = mean

    def copy(self) -> "DoubleWeightedMean":
        return DoubleWeightedMean(self.count, self.total_weight, self.mean)

    def clear(self) -> None:
        self.count, self.total_weight, self.mean = 0, 0.0, float("nan")

    def increment(self, datum: float, weight: float = 1.0) -> None:
        if weight < 0.0:
            raise ValueError("weight must be >= 0")
        if self.count == 0:
            self.count = 1
            self.mean = float(datum)
            self.total_weight = float(weight)
        else:
            self.count += 1
            self.total_weight += weight
            self.mean += (weight / self.total_weight) * (datum - self.mean)

    def increment_all(self, data: Iterable[float]) -> None:
        for d in data:
            self.increment(d)

    @property
    def result(self) -> float:
        return self.mean

    def get_n(self) -> int:
        return self.count

    def __eq__(self, other):
        return isinstance(other, DoubleWeightedMean) and self.count == other.count and \
            self.total_weight == other.total_weight and (
                self.mean == other.mean or (math.isnan(self.mean) and math.isnan(other.mean)))

    def __hash__(self):
        return hash((self.count, self.total_weight, self.mean))

    def __repr__(self):
        return repr(self.mean)
