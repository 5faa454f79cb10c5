"""Normal-equation solvers behind LinearRegression (models/linear.py): the minimum-norm solve of
singular systems (duplicated / collinear columns), eigen path vs the proximal-point Cholesky
recursion used past the device Jacobi eigensolver's n <= 4096."""
import pytest
import torch

from spark_rapids_ml_nai_amd import ops
from spark_rapids_ml_nai_amd.models import linear


def _singular_system(m: int, k: int, dup: int, seed: int):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(m, k, dtype=torch.float64, generator=g)
    X = torch.cat([X, 2.0 * X[:, :dup] - X[:, 1: dup + 1]], 1)  # collinear columns: rank k
    A = X.T @ X / m
    b = X.T @ torch.randn(m, dtype=torch.float64, generator=g) / m
    return A, b


def _pinv_solve(A: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    return torch.linalg.pinv(A, hermitian=True, rtol=A.shape[0] * torch.finfo(torch.float64).eps) @ b


@pytest.mark.parametrize("m,k,dup", [(400, 150, 50), (1000, 300, 3), (300, 100, 99)])
def test_min_norm_prox_matches_pseudo_inverse(m, k, dup):
    A, b = _singular_system(m, k, dup, m + k)
    ref = _pinv_solve(A, b)
    got = linear._min_norm_prox(A, b)
    torch.testing.assert_close(got, ref, rtol=1e-6, atol=1e-9)
    torch.testing.assert_close(linear._min_norm_eig(A, b), ref, rtol=1e-8, atol=1e-10)


def test_spd_factor_solve_cpu():
    A, b = _singular_system(500, 80, 0, 3)
    L, ok = ops.spd_factor(A)
    assert ok
    torch.testing.assert_close(A @ ops.spd_factor_solve(L, b), b, rtol=1e-10, atol=1e-12)


@pytest.mark.gpu
def test_min_norm_solve_wide_device(gpu_device):
    """n > 4096 singular normal equations on the device: potrf/potrs proximal recursion ==
    the CPU pseudo-inverse."""
    A, b = _singular_system(6000, 4000, 200, 11)
    ref = _pinv_solve(A, b)
    got = linear._min_norm_solve(A.to(gpu_device), b.to(gpu_device)).cpu()
    assert A.shape[0] > 4096
    torch.testing.assert_close(got, ref, rtol=1e-6, atol=1e-8)
