"""Poisson bagging (ops.rf_bootstrap) on the CPU path: distribution and layout; per-segment stats."""
import math

import numpy as np
import pytest
import torch

from spark_rapids_ml_nai_amd import ops


def test_rf_bootstrap_layout_and_distribution():
    T, m, rate = 5, 40000, 1.0
    idx, w, bounds = ops.rf_bootstrap(T, m, rate, 99, torch.device("cpu"))
    assert bounds.shape == (T + 1,) and bounds[0] == 0 and bounds[-1] == idx.shape[0] == w.shape[0]
    for t in range(T):
        seg = idx[bounds[t]: bounds[t + 1]].numpy()
        assert (np.diff(seg) > 0).all() and seg.min() >= 0 and seg.max() < m  # ascending, unique, in range
        frac = (bounds[t + 1] - bounds[t]) / m
        assert abs(frac - (1 - math.exp(-rate))) < 0.01  # P(w > 0)
    wt = w.double()
    assert (wt >= 1).all() and (wt <= 255).all()
    assert abs(float(wt.sum()) / (T * m) - rate) < 0.01  # E[w] = rate
    i2, w2, b2 = ops.rf_bootstrap(T, m, rate, 99, torch.device("cpu"))
    assert torch.equal(idx, i2) and torch.equal(w, w2)  # reproducible
    i3, _, _ = ops.rf_bootstrap(T, m, rate, 100, torch.device("cpu"))
    assert not torch.equal(idx, i3)


@pytest.mark.parametrize("regression,crit,S", [(True, 2, 3), (False, 0, 2), (False, 1, 5)])
def test_seg_stats_match_numpy_formulas(regression, crit, S):
    """Per-segment leaf values / weight sums / impurities formed on the device side (torch) equal
    the numpy formulas, including empty segments."""
    from spark_rapids_ml_nai_amd.models import forest

    g = np.random.default_rng(S)
    tot = g.random((500, S)) * 10
    if regression:
        tot[:, 2] = tot[:, 1] ** 2 / np.maximum(tot[:, 0], 1e-9) + g.random(500)
    tot[::7] = 0.0
    st = forest._seg_stats(torch.from_numpy(tot), regression, crit).numpy()
    np.testing.assert_allclose(st[:, :-2], forest._leaf_values_np(tot, regression), rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(st[:, -2], tot[:, 0] if regression else tot.sum(1), rtol=1e-12)
    np.testing.assert_allclose(st[:, -1], forest._impurities_np(tot, crit), rtol=1e-12, atol=1e-14)
