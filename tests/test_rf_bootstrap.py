"""Poisson bagging (ops.rf_bootstrap) on the CPU path: distribution and layout."""
import math

import numpy as np
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
