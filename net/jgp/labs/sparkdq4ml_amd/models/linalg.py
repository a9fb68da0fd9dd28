"""``org.apache.spark.ml.linalg`` local vectors/matrices (``Vectors.dense(40.0)``,
``DataQuality4MachineLearningApp.java:136,150``).  ``toString`` follows Spark: ``[v0,v1,...]``
with Java doubles, sparse as ``(size,[indices],[values])``."""
from __future__ import annotations

from typing import Iterable, Sequence

import numpy as np

from ..utils.javafmt import java_double_str

__all__ = ["Vector", "DenseVector", "SparseVector", "Vectors", "DenseMatrix", "Matrices"]


class Vector:
    def toArray(self) -> np.ndarray:
        raise NotImplementedError

    def size(self) -> int:
        return len(self)

    def dot(self, other) -> float:
        o = other.toArray() if isinstance(other, Vector) else np.asarray(other, dtype=np.float64)
        return float(np.dot(self.toArray(), o))

    def toString(self) -> str:
        return str(self)

    def apply(self, i):
        return self[i]

    def numNonzeros(self):
        return int(np.count_nonzero(self.toArray()))

    def compressed(self) -> "Vector":
        arr = self.toArray()
        nnz = int(np.count_nonzero(arr))
        # Spark: sparse iff 1.5 * (nnz + 1.0) < size
        if 1.5 * (nnz + 1.0) < len(arr):
            idx = np.nonzero(arr)[0]
            return SparseVector(len(arr), idx, arr[idx])
        return DenseVector(arr)


class DenseVector(Vector):
    def __init__(self, values: Iterable[float]):
        self.values = np.asarray(list(values) if not isinstance(values, np.ndarray) else values, dtype=np.float64)

    def toArray(self):
        return self.values

    def __len__(self):
        return int(self.values.shape[0])

    def __getitem__(self, i):
        return float(self.values[i])

    def __iter__(self):
        return iter(self.values.tolist())

    def __eq__(self, other):
        return isinstance(other, Vector) and len(self) == len(other) and np.array_equal(self.toArray(), other.toArray())

    def __hash__(self):
        return hash(self.values.tobytes())

    def __str__(self):
        return "[" + ",".join(java_double_str(v) for v in self.values) + "]"

    def __repr__(self):
        return f"DenseVector({self.values.tolist()})"

    def copy(self):
        return DenseVector(self.values.copy())


class SparseVector(Vector):
    def __init__(self, size: int, indices: Sequence[int], values: Sequence[float]):
        self._size = int(size)
        self.indices = np.asarray(indices, dtype=np.int32)
        self.values = np.asarray(values, dtype=np.float64)

    def toArray(self):
        a = np.zeros(self._size, dtype=np.float64)
        a[self.indices] = self.values
        return a

    def __len__(self):
        return self._size

    def __getitem__(self, i):
        pos = np.searchsorted(self.indices, i)
        return float(self.values[pos]) if pos < len(self.indices) and self.indices[pos] == i else 0.0

    def __eq__(self, other):
        return isinstance(other, Vector) and len(self) == len(other) and np.array_equal(self.toArray(), other.toArray())

    def __hash__(self):
        return hash(self.toArray().tobytes())

    def __str__(self):
        return (f"({self._size},[" + ",".join(str(int(i)) for i in self.indices) + "],["
                + ",".join(java_double_str(v) for v in self.values) + "])")

    __repr__ = __str__


class Vectors:
    @staticmethod
    def dense(*values) -> DenseVector:
        if len(values) == 1 and not isinstance(values[0], (int, float, np.floating, np.integer)):
            return DenseVector(values[0])
        return DenseVector([float(v) for v in values])

    @staticmethod
    def sparse(size, *args) -> SparseVector:
        if len(args) == 1:
            pairs = sorted(dict(args[0]).items()) if isinstance(args[0], dict) else sorted(args[0])
            return SparseVector(size, [p[0] for p in pairs], [p[1] for p in pairs])
        return SparseVector(size, args[0], args[1])

    @staticmethod
    def zeros(n) -> DenseVector:
        return DenseVector(np.zeros(n))

    @staticmethod
    def norm(v: Vector, p: float) -> float:
        return float(np.linalg.norm(v.toArray(), ord=p))

    @staticmethod
    def sqdist(a: Vector, b: Vector) -> float:
        d = a.toArray() - b.toArray()
        return float(np.dot(d, d))


class DenseMatrix:
    """Column-major dense matrix (``org.apache.spark.ml.linalg.DenseMatrix``)."""

    def __init__(self, numRows, numCols, values, isTransposed=False):
        self.numRows, self.numCols = int(numRows), int(numCols)
        self.values = np.asarray(values, dtype=np.float64)
        self.isTransposed = isTransposed

    def toArray(self):
        order = "C" if self.isTransposed else "F"
        return self.values.reshape((self.numRows, self.numCols), order=order)

    def __getitem__(self, ij):
        return float(self.toArray()[ij])

    def __str__(self):
        return str(self.toArray())


class Matrices:
    @staticmethod
    def dense(numRows, numCols, values):
        return DenseMatrix(numRows, numCols, values)
