"""C ABI (``native/include/srml/srml.h``) access from Python and its build helpers.

The host-array entry points mirror the reference JNI library (``jvm/native/src/rapidsml_jni.cu``):
``dgemm`` (N4), ``dgemm_cov`` (N3), ``cal_svd`` (N5), ``accumulate_cov`` (N8). They live in the
same ``libsrml_ops.so`` as the kernels.
"""
from __future__ import annotations

import ctypes
from typing import Tuple

import numpy as np

from ..ops import native as _native

_P = ctypes.c_void_p


def _lib() -> ctypes.CDLL:
    lib = _native.lib()
    if not getattr(lib, "_srml_capi_typed", False):
        lib.srml_capi_dgemm.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_double, _P, ctypes.c_int, _P, ctypes.c_int, ctypes.c_double, _P,
                                        ctypes.c_int, ctypes.c_int]
        lib.srml_capi_dgemm_cov.argtypes = [_P, ctypes.c_long, ctypes.c_int, _P, ctypes.c_int]
        lib.srml_capi_cal_svd.argtypes = [_P, ctypes.c_int, _P, _P, ctypes.c_int]
        lib.srml_capi_accumulate_cov.argtypes = [_P, _P, ctypes.c_long]
        lib.srml_capi_version.restype = ctypes.c_char_p
        for f in ("srml_capi_dgemm", "srml_capi_dgemm_cov", "srml_capi_cal_svd", "srml_capi_accumulate_cov"):
            getattr(lib, f).restype = ctypes.c_int
        lib._srml_capi_typed = True
    return lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError("%s failed with status %d" % (what, rc))


def dgemm_cov(X: np.ndarray, device: int = 0) -> np.ndarray:
    """XᵀX of a (rows, cols) fp64 matrix on the GPU (reference JNI ``dgemmCov``)."""
    X = np.ascontiguousarray(X, dtype=np.float64)
    C = np.empty((X.shape[1], X.shape[1]), dtype=np.float64)
    _check(_lib().srml_capi_dgemm_cov(_ptr(X), X.shape[0], X.shape[1], _ptr(C), device), "dgemm_cov")
    return C


def cal_svd(A: np.ndarray, device: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    """(U, S) of a symmetric PSD matrix: U columns = eigenvectors (descending), S = sqrt(eigenvalues)."""
    A = np.ascontiguousarray(A, dtype=np.float64)
    m = A.shape[0]
    U = np.empty(m * m, dtype=np.float64)
    S = np.empty(m, dtype=np.float64)
    _check(_lib().srml_capi_cal_svd(_ptr(A), m, _ptr(U), _ptr(S), device), "cal_svd")
    return U.reshape(m, m).T.copy(), S  # column-major buffer -> (m, m) with eigenvectors as columns


def dgemm(A: np.ndarray, B: np.ndarray, transa: bool = False, transb: bool = False, alpha: float = 1.0,
          device: int = 0) -> np.ndarray:
    """alpha op(A) op(B) for row-major numpy inputs through the column-major C ABI."""
    A = np.ascontiguousarray(A, dtype=np.float64)
    B = np.ascontiguousarray(B, dtype=np.float64)
    oa = A.T if transa else A
    ob = B.T if transb else B
    m, k = oa.shape
    n = ob.shape[1]
    Ac = np.asfortranarray(oa)
    Bc = np.asfortranarray(ob)
    C = np.zeros((m, n), dtype=np.float64, order="F")
    _check(_lib().srml_capi_dgemm(0, 0, m, n, k, alpha, Ac.ctypes.data, max(m, 1), Bc.ctypes.data, max(k, 1), 0.0,
                                  C.ctypes.data, max(m, 1), device), "dgemm")
    return np.ascontiguousarray(C)


def accumulate_cov(acc: np.ndarray, c: np.ndarray) -> np.ndarray:
    assert acc.dtype == np.float64 and c.dtype == np.float64 and acc.flags.c_contiguous and c.flags.c_contiguous
    _check(_lib().srml_capi_accumulate_cov(_ptr(acc), _ptr(c), acc.size), "accumulate_cov")
    return acc


def version() -> str:
    return _lib().srml_capi_version().decode()
