"""Minimal ``pyspark.ml.linalg``-compatible vector/matrix types.

When pyspark is importable its own classes are re-exported so models interoperate with Spark;
otherwise these numpy-backed equivalents provide the same constructor/attribute surface used
by the reference's model properties (``PCAModel.pc`` -> DenseMatrix column-major,
``coefficients`` -> DenseVector, ``interceptVector``, ``coefficientMatrix``, ...).
"""
from __future__ import annotations

from typing import Any, Iterable, List, Sequence, Union

import numpy as np

try:  # pragma: no cover - exercised only when pyspark is installed
    from pyspark.ml.linalg import (  # type: ignore
        DenseMatrix,
        DenseVector,
        Matrices,
        SparseMatrix,
        SparseVector,
        Vector,
        Vectors,
    )

    HAVE_PYSPARK_LINALG = True
except Exception:  # noqa: BLE001
    HAVE_PYSPARK_LINALG = False

    class Vector:
        def toArray(self) -> np.ndarray:
            raise NotImplementedError

    class DenseVector(Vector):
        def __init__(self, ar: Union[Sequence[float], np.ndarray]) -> None:
            self.array = np.asarray(ar, dtype=np.float64).reshape(-1)

        def toArray(self) -> np.ndarray:
            return self.array

        @property
        def values(self) -> np.ndarray:
            return self.array

        @property
        def size(self) -> int:
            return int(self.array.shape[0])

        def __len__(self) -> int:
            return self.size

        def __getitem__(self, i: Any) -> Any:
            return self.array[i]

        def __iter__(self) -> Any:
            return iter(self.array)

        def dot(self, other: Any) -> float:
            o = other.toArray() if hasattr(other, "toArray") else np.asarray(other)
            return float(np.dot(self.array, o))

        def norm(self, p: float) -> float:
            return float(np.linalg.norm(self.array, p))

        def numNonzeros(self) -> int:
            return int(np.count_nonzero(self.array))

        def __eq__(self, other: Any) -> bool:
            if hasattr(other, "toArray"):
                return np.array_equal(self.array, other.toArray())
            return False

        def __hash__(self) -> int:
            return hash(self.array.tobytes())

        def __repr__(self) -> str:
            return "DenseVector([%s])" % ", ".join("%g" % v for v in self.array)

        __str__ = __repr__

    class SparseVector(Vector):
        def __init__(self, size: int, *args: Any) -> None:
            self.size = int(size)
            if len(args) == 1:
                pairs = args[0]
                if isinstance(pairs, dict):
                    pairs = sorted(pairs.items())
                idx = [int(p[0]) for p in pairs]
                val = [float(p[1]) for p in pairs]
            else:
                idx, val = args
            self.indices = np.asarray(idx, dtype=np.int32)
            self.values = np.asarray(val, dtype=np.float64)

        def toArray(self) -> np.ndarray:
            out = np.zeros(self.size, dtype=np.float64)
            out[self.indices] = self.values
            return out

        def __len__(self) -> int:
            return self.size

        def numNonzeros(self) -> int:
            return int(np.count_nonzero(self.values))

        def dot(self, other: Any) -> float:
            o = other.toArray() if hasattr(other, "toArray") else np.asarray(other)
            return float(np.dot(self.values, o[self.indices]))

        def __eq__(self, other: Any) -> bool:
            if hasattr(other, "toArray"):
                return np.array_equal(self.toArray(), other.toArray())
            return False

        def __hash__(self) -> int:
            return hash((self.size, self.indices.tobytes(), self.values.tobytes()))

        def __repr__(self) -> str:
            return "SparseVector(%d, {%s})" % (
                self.size,
                ", ".join("%d: %g" % (i, v) for i, v in zip(self.indices, self.values)),
            )

        __str__ = __repr__

    class Vectors:
        @staticmethod
        def dense(*elements: Any) -> DenseVector:
            if len(elements) == 1 and not isinstance(elements[0], (float, int)):
                return DenseVector(elements[0])
            return DenseVector([float(e) for e in elements])

        @staticmethod
        def sparse(size: int, *args: Any) -> SparseVector:
            return SparseVector(size, *args)

        @staticmethod
        def zeros(size: int) -> DenseVector:
            return DenseVector(np.zeros(size))

    class DenseMatrix:
        """Column-major dense matrix (Spark layout)."""

        def __init__(self, numRows: int, numCols: int, values: Iterable[float], isTransposed: bool = False) -> None:
            self.numRows = int(numRows)
            self.numCols = int(numCols)
            self.values = np.asarray(list(values) if not isinstance(values, np.ndarray) else values, dtype=np.float64)
            self.isTransposed = isTransposed

        def toArray(self) -> np.ndarray:
            if self.isTransposed:
                return self.values.reshape((self.numRows, self.numCols))
            return self.values.reshape((self.numRows, self.numCols), order="F")

        def __repr__(self) -> str:
            return "DenseMatrix(%d, %d, %s)" % (self.numRows, self.numCols, list(self.values[:16]))

        def __eq__(self, other: Any) -> bool:
            return hasattr(other, "toArray") and np.array_equal(self.toArray(), other.toArray())

    class SparseMatrix:
        def __init__(self, numRows: int, numCols: int, colPtrs: Any, rowIndices: Any, values: Any,
                     isTransposed: bool = False) -> None:
            self.numRows, self.numCols = int(numRows), int(numCols)
            self.colPtrs = np.asarray(colPtrs, dtype=np.int32)
            self.rowIndices = np.asarray(rowIndices, dtype=np.int32)
            self.values = np.asarray(values, dtype=np.float64)
            self.isTransposed = isTransposed

        def toArray(self) -> np.ndarray:
            out = np.zeros((self.numRows, self.numCols))
            for j in range(self.numCols):
                for p in range(self.colPtrs[j], self.colPtrs[j + 1]):
                    out[self.rowIndices[p], j] = self.values[p]
            return out

    class Matrices:
        @staticmethod
        def dense(numRows: int, numCols: int, values: Iterable[float]) -> DenseMatrix:
            return DenseMatrix(numRows, numCols, values)

        @staticmethod
        def sparse(numRows: int, numCols: int, colPtrs: Any, rowIndices: Any, values: Any) -> SparseMatrix:
            return SparseMatrix(numRows, numCols, colPtrs, rowIndices, values)


def as_dense_array(v: Any) -> np.ndarray:
    """Vector / list / ndarray -> 1-D float64 ndarray."""
    if hasattr(v, "toArray"):
        return np.asarray(v.toArray())
    return np.asarray(v, dtype=np.float64)


def compressed_vector(arr: np.ndarray) -> Vector:
    """Return a SparseVector when it uses less space, like Spark's ``Vector.compressed``."""
    arr = np.asarray(arr, dtype=np.float64)
    nnz = int(np.count_nonzero(arr))
    if 1.5 * (nnz + 1.0) < arr.shape[0]:
        idx = np.nonzero(arr)[0]
        return Vectors.sparse(arr.shape[0], idx.tolist(), arr[idx].tolist())
    return Vectors.dense(arr)


def compressed_matrix(mat: np.ndarray) -> Any:
    """Dense-or-sparse (CSC) matrix, whichever is smaller (Spark ``Matrix.compressed``)."""
    mat = np.asarray(mat, dtype=np.float64)
    nnz = int(np.count_nonzero(mat))
    r, c = mat.shape
    if nnz * 1.5 + c + 1 < r * c:
        col_ptrs = [0]
        rows: List[int] = []
        vals: List[float] = []
        for j in range(c):
            nz = np.nonzero(mat[:, j])[0]
            rows.extend(nz.tolist())
            vals.extend(mat[nz, j].tolist())
            col_ptrs.append(len(rows))
        return Matrices.sparse(r, c, col_ptrs, rows, vals)
    return DenseMatrix(r, c, mat.reshape(-1, order="F"))
