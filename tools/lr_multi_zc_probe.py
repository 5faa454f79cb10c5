"""Multinomial LogisticRegression with and without the line-search margin cache: fit seconds,
iterations, evaluations (full / margins-only) and objective on a synthetic K-class shard."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from spark_rapids_ml_nai_amd.models import qn as qnm  # noqa: E402
from spark_rapids_ml_nai_amd.models.logistic import logistic_fit  # noqa: E402
from spark_rapids_ml_nai_amd.parallel.context import WorkerContext  # noqa: E402

dev = torch.device("cuda", 0)
for m, n, K in ((500_000, 1000, 5), (200_000, 3000, 10)):
    g = torch.Generator(device=dev).manual_seed(1)
    X = torch.randn(m, n, device=dev, generator=g)
    Wtrue = torch.randn(n, K, device=dev, generator=g) * (2.0 / n ** 0.5)
    y = (X @ Wtrue + torch.randn(m, K, device=dev, generator=g)).argmax(1).float()
    ctx = WorkerContext.single(dev)
    for zc in (False, True, False, True):
        qnm.QN_ZCACHE = zc
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = logistic_fit(X, y, m, ctx, reg=1e-5, l1_ratio=0.0, fit_intercept=True, standardization=False,
                         max_iter=200, tol=1e-30, n_classes=K)
        torch.cuda.synchronize()
        print(json.dumps({"m": m, "n": n, "K": K, "zcache": zc, "fit_s": round(time.perf_counter() - t0, 4),
                          "iters": r.get("num_iters"), "objective": r["objective"], **r["_solver"]}), flush=True)
