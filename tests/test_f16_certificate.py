"""The fp16 KMeans filter's certificate (ops.certify_tau16 / f16_radius_terms), checked on the CPU by
emulating the filter exactly as the kernel computes it (fp32 x - mu, power-of-two scale, fp16
round-to-nearest of both operands) and comparing certified rows against the fp64 arg-min."""
import math

import numpy as np
import pytest
import torch

from spark_rapids_ml_nai_amd import ops


def _scale(V: torch.Tensor) -> float:
    a = float(V.abs().max())
    return 2.0 ** (13 - (math.frexp(a)[1] - 1))


def _emulate(X: torch.Tensor, C: torch.Tensor, mu: torch.Tensor):
    n = X.shape[1]
    V = X.float() - mu.float()
    W = C.float() - mu.float()
    s = _scale(V)
    Vh = (V * s).half().double() / s
    Wh = (W * s).half().double() / s
    cn = (W.double() ** 2).sum(1)
    d_f = cn.view(1, -1) - 2.0 * Vh @ Wh.T
    tau = ops.certify_tau16(n)
    xadd, z, z2 = ops.f16_radius_terms(n, s, tau)
    xs0 = V.double().norm(dim=1)
    xs = xs0 + xadd
    g = 2.0 * tau * cn.sqrt()
    b = d_f.argmin(1)
    adj = d_f - xs.view(-1, 1) * g.view(1, -1)
    adj.scatter_(1, b.view(-1, 1), float("inf"))
    low = adj.min(1).values
    cert = low > d_f.gather(1, b.view(-1, 1)).view(-1) + xs * g[b] + 2.0 * (z * xs0 + z2)
    d = cn.view(1, -1) - 2.0 * V.double() @ W.double().T
    return b, cert, d, s


@pytest.mark.parametrize("case", ["generic", "ties", "offset", "wide_range"])
def test_f16_certified_rows_match_fp64_argmin(case):
    g = torch.Generator().manual_seed(7)
    m, n, k = 3000, 257, 300
    X = torch.randn(m, n, generator=g, dtype=torch.float64)
    C = torch.randn(k, n, generator=g, dtype=torch.float64)
    if case == "ties":
        C[1::2] = C[0::2] + 1e-6 * torch.randn(k // 2, n, generator=g, dtype=torch.float64)
        X[: m // 4] = 0.5 * (C[0] + C[2]) + 1e-7 * torch.randn(m // 4, n, generator=g, dtype=torch.float64)
    elif case == "offset":
        X += 1e4
        C += 1e4
    elif case == "wide_range":  # a few huge columns: most elements fall below fp16's normal range
        X[:, :3] *= 1e7
        C[:, :3] *= 1e7
        X[:, 3:] *= 1e-3
        C[:, 3:] *= 1e-3
    X, C = X.float(), C.float()
    mu = X.double().mean(0).float()
    b, cert, d, s = _emulate(X, C, mu)
    assert 2.0 ** 13 <= s * float((X - mu).abs().max()) < 2.0 ** 14
    exact = d.argmin(1)
    assert torch.equal(b[cert], exact[cert])
    frac = float(cert.double().mean())
    if case == "ties":
        assert not bool(cert[: m // 4].any())  # bisector rows are never certified
    elif case == "generic":
        assert frac > 0.5


def test_f16_radius_terms_consistent():
    n, s = 3000, 2.0 ** 12
    tau = ops.certify_tau16(n)
    assert tau > 2.0 * 2.0 ** -11 + n * 2.0 ** -24  # covers the rounding + the filter's accumulation
    assert tau > ops.certify_tau(n)  # wider than the 3-product bf16 filter's radius
    xadd, z, z2 = ops.f16_radius_terms(n, s, tau)
    # xadd = (z + the fp32 rounding of ||c - mu||^2 at the largest representable centre) / (2 tau)
    assert xadd == pytest.approx((z + 2.0 ** -24 * math.sqrt(n) * 32768.0 / s) / (2 * tau))
    a = 2.0 ** -14 / s
    assert z >= 2 * a * math.sqrt(n) and z2 >= 2 * n * a * a
    np.testing.assert_allclose(ops.f16_radius_terms(n, 2 * s, tau)[1], z / 2)
