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


@pytest.mark.gpu
@pytest.mark.parametrize("fit_intercept", [True, False])
@pytest.mark.parametrize("standardization", [True, False])
@pytest.mark.parametrize("reg,l1", [(0.0, 0.0), (0.3, 0.0), (0.1, 0.5)])
def test_device_lsq_statistics_and_solve_match_cpu(gpu_device, fit_intercept, standardization, reg, l1):
    """The native second-order statistics (in-place all-reduce buffers, one-pass scatter shift, label
    sums) match the CPU pass (the device Gram's fp32 products: ~1e-6 relative), and on the SAME
    statistics the native system preparation / back-transform (srml_lsq_prepare / srml_lsq_finish)
    gives the torch formulas' coefficients and intercept — a constant column included."""
    from dataclasses import replace

    from spark_rapids_ml_nai_amd.parallel.context import WorkerContext

    g = torch.Generator().manual_seed(7)
    m, n = 3000, 40
    X = (torch.randn(m, n, generator=g) * torch.linspace(0.5, 3.0, n) + 2.0).float()
    X[:, 5] = 1.25  # constant column: dropped from the system, zero coefficient
    w = torch.randn(n, generator=g)
    y = (X.double() @ w.double() + 0.7 + 0.1 * torch.randn(m, generator=g, dtype=torch.float64)).float()
    st_c = linear.lsq_stats(X, y, m, WorkerContext.single(torch.device("cpu")))
    st_g = linear.lsq_stats(X.to(gpu_device), y.to(gpu_device), m, WorkerContext.single(torch.device(gpu_device)))
    # (the device column moments / Gram accumulate fp32 partials: ~1e-7 relative)
    torch.testing.assert_close(st_g.xbar.cpu(), st_c.xbar, rtol=1e-6, atol=1e-9)
    torch.testing.assert_close(st_g.sumsq.cpu(), st_c.sumsq, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(st_g.xty.cpu(), st_c.xty, rtol=1e-6, atol=1e-4)
    torch.testing.assert_close(st_g.scatter.cpu(), st_c.scatter, rtol=1e-4, atol=1e-2)
    assert st_g.ybar == pytest.approx(st_c.ybar, rel=1e-10) and st_g.ystd == pytest.approx(st_c.ystd, rel=1e-8)
    # the same (device) statistics through the native and the torch formulas
    st_h = replace(st_g, xbar=st_g.xbar.cpu(), sumsq=st_g.sumsq.cpu(), scatter=st_g.scatter.cpu(), xty=st_g.xty.cpu())
    a = linear.lsq_solve(st_h, reg, l1, fit_intercept, standardization, 200, 1e-12)
    b = linear.lsq_solve(st_g, reg, l1, fit_intercept, standardization, 200, 1e-12)
    tol = 1e-8 if reg == 0.0 or l1 == 0.0 else 1e-6  # (coordinate descent: host vs device sweeps to 1e-12)
    torch.testing.assert_close(torch.tensor(b["coef_"]), torch.tensor(a["coef_"]), rtol=tol, atol=tol)
    assert b["intercept_"] == pytest.approx(a["intercept_"], rel=tol, abs=tol)
    assert abs(b["coef_"][5]) < 1e-12
